// tcpck_bstream.hip -- fixed-stride packed batches of LARGE images streamed in
// byte runs that ignore image boundaries (experiment: the C4 layout, 64-KiB
// images).
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16), a ring sum, so an image's sum is
// the sum of the partial sums of any split of its bytes.
//
// rstream gives each wave whole images, so a 64-KiB image is a 64-step run and
// the grid holds few, long runs; seg's W-wave shapes split an image over a
// block of W waves that meet in LDS and wait for each other.  Here wave w owns
// the byte range [w R, (w + 1) R) of the batch (R a power of two, 8 KiB by
// default, positions counted from the 128-B line at or below the arena), read
// exactly like rstream's runs (16 B per lane and step, U steps in flight, one
// DPP scan per step, the image ends inside the run walked in scalar registers).
// An image that starts and ends inside the run is stored at its end; an image
// cut by a run edge contributes its partial sum (mod 2^16) to a per-image u64
// in a workspace, (1 << 32) + partial, with one device-scope atomic add: the
// wave whose add completes the count (the image's number of runs) finishes the
// image and resets the word to 0, so the workspace is all-zero between
// launches.  REF mode, CHECKSUM and VERIFY.
#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

template <int U, int OP>
__global__ void __launch_bounds__(kBlock) bstream_kernel(ByteRunArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  if (wid >= a.nruns) return;
  const uint32_t sh = a.run_shift;
  const uint64_t S = a.stride;
  const uint64_t off0 = a.off0;                    // arena & 127: positions are arena bytes + off0
  const uint64_t end_pos = off0 + a.count * S;     // one past the batch
  const uint64_t r0 = wid << sh;
  const uint64_t r1 = min(r0 + (uint64_t{1} << sh), end_pos);
  const uint32_t lead = wid == 0 ? static_cast<uint32_t>(off0) : 0u;
  const uint32_t span = static_cast<uint32_t>(r1 - r0);
  const uint32_t nsteps = (span + 1023) >> 10;
  const uint8_t *base = a.arena - off0 + r0;      // 128-B aligned
  const auto rsrc = dev::make_rsrc(base, (span + 15) & ~15u);

  // the first image the run touches and the run-relative end of it
  uint64_t k = (r0 + lead - off0) / S;
  const bool first_cut = off0 + k * S < r0 + lead;  // it started in an earlier run
  uint64_t nb = off0 + (k + 1) * S - r0;             // may lie past the run

  auto parts = [&](uint64_t kk) -> uint32_t {  // runs image kk touches
    return static_cast<uint32_t>(((off0 + (kk + 1) * S - 1) >> sh) - ((off0 + kk * S) >> sh) + 1);
  };
  auto store = [&](uint64_t kk, uint32_t sum) {
    const uint16_t c = dev::finish<kRef>(sum);  // tcp-header.h:262
    if constexpr (OP == kVerify)
      static_cast<uint8_t *>(a.out)[kk] = c == 0 ? 1 : 0;
    else
      static_cast<uint16_t *>(a.out)[kk] = c;
  };
  // image kk's word sum over this run's bytes; complete: the image lies in the run
  auto emit = [&](uint64_t kk, uint32_t sum, bool complete) {
    if (lane != 0) return;
    if (complete) {
      store(kk, sum);
      return;
    }
    const uint64_t v = (uint64_t{1} << 32) | (sum & 0xFFFFu);
    const uint64_t old = __hip_atomic_fetch_add(a.ws + kk, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> 32) + 1 == parts(kk)) {  // the last part: finish, leave the word zero
      store(kk, static_cast<uint32_t>(old) + (sum & 0xFFFFu));
      __hip_atomic_store(a.ws + kk, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = dev::load16_buf_nt(rsrc, lane << 4, static_cast<uint32_t>(u) << 10);
  uint32_t carry = 0, p_last = 0;
  bool cut = first_cut;  // the current image started before this run
  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = g + u;
      const uint32_t sb = st << 10;
      u32x4 w = ring[u];
      if (sb == 0 || sb + 1024 > span) {  // run edge: keep words of [lead, span) only
        const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
        const int32_t lo = min(max(static_cast<int32_t>(lead) - crel, 0), 16);
        const int32_t hi = min(max(static_cast<int32_t>(span) - crel, 0), 16);
        w = dev::apply_mask(w, dev::word_mask(lo, hi));
      }
      const uint32_t tot = dev::ref_chunk_sum_dot(w);
      const uint32_t incl = dev::wave_inclusive_scan(tot);
      while (nb < sb + 1024 && nb < span) {  // image ends strictly inside the run (scalar)
        const uint32_t rel = static_cast<uint32_t>(nb) - sb;
        const uint32_t lb = rel >> 4, r = rel & 15u;
        uint32_t P = carry + dev::read_lane(incl, lb) - dev::read_lane(tot, lb);
        if (r)
          P += dev::words_before<false>(r, dev::read_lane(w.x, lb), dev::read_lane(w.y, lb), dev::read_lane(w.z, lb),
                                        dev::read_lane(w.w, lb));
        emit(k, P - p_last, !cut);
        cut = false;
        p_last = P;
        nb += S;
        ++k;
      }
      carry += dev::read_lane(incl, 63);
      ring[u] = dev::load16_buf_nt(rsrc, lane << 4, (st + U) << 10);
    }
  }
  // the image holding the run's last byte: complete if it also ends here
  if (k < a.count) emit(k, carry - p_last, !cut && nb == span);
}

template <int U, int OP>
hipError_t launch_one(const ByteRunArgs &a, hipStream_t stream) {
  const uint64_t blocks = (a.nruns + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((bstream_kernel<U, OP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_bstream(int op, int variant, ByteRunArgs a, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  if (!a.ws || !a.out || a.stride < 2 || (a.stride & 1)) return hipErrorInvalidValue;
  // param bits 0-4: log2 of the run bytes (0 = 13: 8 KiB; 10..20); bit 8: U8
  const uint32_t shift = (variant & 31) ? static_cast<uint32_t>(variant & 31) : 13u;
  if (shift < 10 || shift > 20) return hipErrorInvalidValue;
  a.run_shift = shift;
  a.off0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) & 127u);
  a.nruns = (a.off0 + a.count * a.stride + (uint64_t{1} << shift) - 1) >> shift;
  a.order = 4u;  // XCD-chunked, groups of 16 blocks (as the run kernels)
  const bool u8 = (variant & 256) != 0;
  switch (op) {
    case kChecksum: return u8 ? launch_one<8, kChecksum>(a, stream) : launch_one<4, kChecksum>(a, stream);
    case kVerify: return u8 ? launch_one<8, kVerify>(a, stream) : launch_one<4, kVerify>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
