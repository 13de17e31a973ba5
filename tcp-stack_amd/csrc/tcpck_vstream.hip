// tcpck_vstream.hip -- fixed-stride packed batches of small images (stride ==
// length, 16 <= S < ~768 B): one contiguous run per wave like rstream, but
// the image boundaries of a step are resolved by the lanes in parallel.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16), and sum(k) = P(end_k) -
// P(start_k) (mod 2^16) with P(x) the word sum of the wave's run before byte x.
//
// rstream walks boundaries one at a time in scalar registers: ~40 instructions
// per boundary, which is fine at 0.7 boundaries per 1 KiB step (1492-B images)
// and ruinous at 10 (96-B images) or 32 (32-B control packets).  Here every
// step costs the same whatever the density:
//   * lane l's 16-B chunk starts at run byte c = 1024 s + 16 l; its offset in
//     its image, m = (c - lead) mod S, is kept per lane and advanced by
//     1024 mod S per step (add, subtract, unsigned min);
//   * a boundary lies in the chunk iff m == 0 (at the chunk start) or
//     S - m < 16 (at r = S - m); S >= 16 means at most one per chunk;
//   * the lane's words before r come from the partial sums of its own
//     v_dot2 chunk-sum chain (q1..q3) and one masked dword: P(boundary) =
//     carry + exclusive scan + head;
//   * the previous boundary is S bytes back: in lane (p - S - 1024 s) / 16 of
//     the same step (ds_bpermute) or, for the step's first boundary, the last
//     boundary of the step before (one SGPR);
//   * results leave from the boundary lanes themselves, to index images_done
//     + rank (mbcnt of the boundary ballot): contiguous u16 stores.
// kFill zeroes each image's checksum word (bytes 28-29, S >= 30) in the stream
// and writes the result there (tcp-header.h:177); kVerify stores checksum == 0.
#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

__device__ __forceinline__ uint32_t lane_bpermute(uint32_t v, uint32_t src_lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src_lane << 2), static_cast<int>(v)));
}

template <int U, int OP>
__global__ void __launch_bounds__(kBlock) vstream_kernel(FixedStreamArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  uint64_t kb, ke;
  dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  if (kb >= ke) return;
  const uint32_t S = static_cast<uint32_t>(a.stride);
  const uint64_t s0 = kb * S;
  const uint64_t A0 = dev::align128_rel(a.arena, s0);
  const uint32_t lead = static_cast<uint32_t>(s0 - A0);
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  const uint32_t span = lead + nimg * S;
  const uint32_t nsteps = (span + 1023) >> 10;
  const uint32_t last_chunk = (span - 1) >> 4;
  uint8_t *base = a.arena + A0;
  const auto rsrc = dev::make_rsrc(base, (last_chunk + 1) << 4);
  auto load_step = [&](uint32_t st) -> u32x4 { return dev::load16_buf_nt(rsrc, lane << 4, st << 10); };

  // per-lane offset of the chunk start in its image, in [0, S)
  const uint32_t delta = 1024u % S;
  uint32_t m = (16u * lane + 128u * S - lead) % S;
  uint32_t carry = 0;   // P at the step start
  uint32_t p_last = 0;  // P at the latest boundary of earlier steps (run start: 0)
  uint32_t done = 0;    // images emitted

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = load_step(static_cast<uint32_t>(u));

  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = g + u;
      const uint32_t sb = st << 10;
      const uint32_t c = sb + (lane << 4);
      u32x4 w = ring[u];
      const bool edge = sb == 0 || sb + 1024 > span;  // wave-uniform
      if (edge) {  // run edge: keep words of [lead, span) only
        const int32_t lo = min(max(static_cast<int32_t>(lead) - static_cast<int32_t>(c), 0), 16);
        const int32_t hi = min(max(static_cast<int32_t>(span) - static_cast<int32_t>(c), 0), 16);
        w = dev::apply_mask(w, dev::word_mask(lo, hi));
      }
      if constexpr (OP == kFill) {  // zero the checksum field if this chunk holds one
        if (S >= 30) {
          const uint32_t f = m <= 28 ? 28 - m : 28 + S - m;  // field offset from the chunk start
          if (f < 16) {
            const uint32_t keep = (f & 2u) ? 0x0000FFFFu : 0xFFFF0000u;
            const uint32_t di = f >> 2;
            w.x &= di == 0 ? keep : ~0u;
            w.y &= di == 1 ? keep : ~0u;
            w.z &= di == 2 ? keep : ~0u;
            w.w &= di == 3 ? keep : ~0u;
          }
        }
      }
      // chunk sum with its partial sums (words before dword 1, 2, 3)
      const uint32_t q1 = dev::dot2_u16(w.x, 0u);
      const uint32_t q2 = dev::dot2_u16(w.y, q1);
      const uint32_t q3 = dev::dot2_u16(w.z, q2);
      const uint32_t tot = dev::dot2_u16(w.w, q3);
      const uint32_t incl = dev::wave_inclusive_scan(tot);
      // boundary in this chunk?  r = its offset from the chunk start
      const uint32_t r = m == 0 ? 0u : S - m;
      bool has = r < 16;
      if (edge) {  // only image ends in (lead, span] count
        const uint32_t p = c + r;
        has = has && p > lead && p <= span;
      }
      const uint32_t di = r >> 2;
      const uint32_t qd = di == 0 ? 0u : (di == 1 ? q1 : (di == 2 ? q2 : q3));
      const uint32_t dw = di == 0 ? w.x : (di == 1 ? w.y : (di == 2 ? w.z : w.w));
      const uint32_t head = qd + ((r & 2u) ? (dw & 0xFFFFu) : 0u);
      const uint32_t pb = carry + incl - tot + head;  // P(boundary)
      // previous boundary: S bytes back, in this step or the last one of the step before
      const uint32_t prev_rel = c + r - S - sb;  // wraps (huge) when before this step
      const bool prev_here = c + r >= sb + S;
      const uint32_t pprev_lane = lane_bpermute(pb, prev_here ? (prev_rel >> 4) : lane);
      const uint32_t pprev = prev_here ? pprev_lane : p_last;
      const uint64_t bal = __ballot(has);
      if (bal) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u));
        if (has) {
          const uint64_t k = kb + done + rank;
          const uint16_t cs = static_cast<uint16_t>(~(pb - pprev));
          if constexpr (OP == kVerify) {
            static_cast<uint8_t *>(a.out)[k] = (cs == 0) ? 1 : 0;
          } else {
            if (a.out) static_cast<uint16_t *>(a.out)[k] = cs;
            if (OP == kFill && S >= 30) *reinterpret_cast<uint16_t *>(base + (c + r - S) + 28) = cs;
          }
        }
        done += static_cast<uint32_t>(__popcll(bal));
        p_last = dev::read_lane(pb, 63u - static_cast<uint32_t>(__clzll(bal)));
      }
      carry += dev::read_lane(incl, 63);
      m = m + delta;
      m = min(m, m - S);  // unsigned: m - S wraps above m unless m >= S
      ring[u] = load_step(st + U);
    }
  }
  // an image ending exactly at the last step's end has its boundary in the
  // (absent) next step: P there is the final carry
  if (done < nimg && lane == 0) {
    const uint64_t k = kb + done;
    const uint16_t cs = static_cast<uint16_t>(~(carry - p_last));
    if constexpr (OP == kVerify) {
      static_cast<uint8_t *>(a.out)[k] = (cs == 0) ? 1 : 0;
    } else {
      if (a.out) static_cast<uint16_t *>(a.out)[k] = cs;
      if (OP == kFill && S >= 30) *reinterpret_cast<uint16_t *>(base + (span - S) + 28) = cs;
    }
  }
}

template <int U, int OP>
hipError_t launch_one(const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(vstream_kernel<U, OP>);
  const uint32_t cap = (a.blocks_per_cu && a.blocks_per_cu < per_cu) ? a.blocks_per_cu : per_cu;
  const uint64_t resident = static_cast<uint64_t>(cap) * num_cus;
  uint64_t blocks = resident * dev::oversub_for(a.oversub, a.count * a.stride, resident * kWavesPerBlock, 32);
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  FixedStreamArgs b = a;
  b.per_wave = a.count / (blocks * kWavesPerBlock);
  b.rem = a.count % (blocks * kWavesPerBlock);
  hipLaunchKernelGGL((vstream_kernel<U, OP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, b);
  return hipGetLastError();
}

template <int U>
hipError_t dispatch(int op, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum>(a, num_cus, s);
    case kFill: return launch_one<U, kFill>(a, num_cus, s);
    case kVerify: return launch_one<U, kVerify>(a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_vstream(int op, int variant, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  // 16 <= S (one boundary per chunk at most); per-wave run below 2^31 bytes;
  // 128 S + 16 l must not overflow u32 in the lane offset set-up
  if (a.stride < 16 || a.stride > (1u << 22) || a.count == 0) return hipErrorInvalidValue;
  const uint64_t max_run = ((a.count + 2047) / 2048 + 1) * a.stride + 128;
  if (max_run >= (uint64_t{1} << 31)) return hipErrorInvalidValue;
  switch (variant) {
    case 0: return dispatch<4>(op, a, num_cus, stream);
    case 1: return dispatch<2>(op, a, num_cus, stream);
    case 2: return dispatch<8>(op, a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
