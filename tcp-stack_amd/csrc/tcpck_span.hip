// tcpck_span.hip -- the packed-layout ("span") kernel: one wave streams a run
// of whole, back-to-back images with fully coalesced 1 KiB loads.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263,
// sum of LE u16 words mod 2^16 (the reference's u32 accumulator truncated by
// `~` to u16; no carry fold).  Because that arithmetic is a plain modular
// sum, the checksum of an image is a difference of prefix sums:
//
//     sum(image k) = P(end_k) - P(start_k)   (mod 2^16)
//
// where P(x) is the word sum of the wave's span up to byte x.  This kernel
// therefore never splits work by image:
//   * a tile = T consecutive images whose bytes are contiguous
//     (offsets[k+1] == offsets[k] + lengths[k]); wave w streams tiles
//     w, w + W, ... where W = waves in the grid;
//   * the tile's byte span is read as a flat stream: step s covers bytes
//     [A0 + 1024 s, A0 + 1024 (s+1)), lane l reads the 16 B at 1024 s + 16 l
//     (one global_load_dwordx4 ... nt per lane per step, U steps in flight);
//     only the first and last step of a span mask words (span edges);
//   * per step the 64 lane sums are prefix-scanned across the wave with DPP
//     (row_shr 1/2/4/8 + row_bcast 15/31), plus a running carry (readlane 63);
//   * image boundaries are at least 16 B apart (lengths >= 16, checked per
//     tile), so a 16-byte chunk holds at most one.  The lane holding boundary
//     j's byte posts (j, offset in chunk) into its wave's LDS slot for the
//     chunk; the chunk's lane reads it and records P(boundary) = carry +
//     exclusive scan + the words of its chunk before the boundary in the
//     wave's LDS array pb[j];
//   * at the end of the tile lane j < T computes ~(pb[j+1] - pb[j]) and the
//     T results are stored as one contiguous run.
// Tiles that are not packed, or hold an image shorter than 16 B, fall back to
// whole-wave-per-image summation inside the same launch (results identical).
// kFill subtracts the (pre-read) field word instead of masking it in the
// stream, then writes the checksum into bytes 28-29 (tcp-header.h:177).
// RFC 1071 mode is not served here (one's-complement prefix differences lose
// the +0 / -0 distinction); the host routes it to the seg kernel.
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

template <int OP>
__device__ __forceinline__ void emit(const SpanArgs &a, uint64_t k, uint32_t sum, uint64_t start,
                                     uint32_t len) {
  const uint16_t c = static_cast<uint16_t>(~sum);  // tcp-header.h:262
  if constexpr (OP == kVerify) {
    static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
  } else {
    if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
    if (OP == kFill && len >= 30) *reinterpret_cast<uint16_t *>(a.arena + start + 28) = c;
  }
}

template <int U, int OP, bool FIXED>
__global__ void __launch_bounds__(kBlock) span_kernel(SpanArgs a) {
  __shared__ uint32_t s_slot[kWavesPerBlock][64];
  __shared__ uint32_t s_pb[kWavesPerBlock][64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t *slot = s_slot[wv];
  uint32_t *pb = s_pb[wv];
  slot[lane] = 0;
  const uint32_t T = a.tile;
  const uint64_t ntiles = (a.count + T - 1) / T;
  const uint64_t nwaves = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  uint64_t t = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + wv;

  // descriptors of the first tile (variable layout); later tiles are
  // prefetched one tile ahead so the stream never waits on them
  uint64_t nbj = 0;
  uint32_t nlj = 0;
  if (!FIXED && t < ntiles) {
    const uint64_t k = t * T + lane;
    if (lane < T && k < a.count) {
      nbj = a.offsets[k] - a.base;
      nlj = a.lengths[k];
    }
  }
  for (; t < ntiles; t += nwaves) {
    const uint64_t k0 = t * T;
    const uint32_t n = static_cast<uint32_t>(min(static_cast<uint64_t>(T), a.count - k0));
    uint64_t bj;
    uint32_t lj;
    if (FIXED) {
      bj = (k0 + lane) * a.stride;
      lj = static_cast<uint32_t>(a.stride);
    } else {
      bj = nbj;
      lj = nlj;
      const uint64_t k = (t + nwaves) * T + lane;
      nbj = 0;
      nlj = 0;
      if (lane < T && k < a.count) {
        nbj = a.offsets[k] - a.base;
        nlj = a.lengths[k];
      }
    }
    const uint64_t s0 = dev::read_lane64(bj, 0);
    const uint64_t s1 = dev::read_lane64(bj, n - 1) + dev::read_lane(lj, n - 1);
    const uint64_t A0 = dev::align16_rel(a.arena, s0);
    bool packed = (s1 - A0) < (uint64_t{1} << 30);
    if (!FIXED) {
      const uint64_t nb = __shfl_down(static_cast<unsigned long long>(bj), 1, 64);
      const bool bad = lane < n && (lj < 16 || (lane + 1 < n && bj + lj != nb));
      packed = packed && __ballot(bad) == 0;
    }
    if (!packed) {  // wave-uniform: per-image fallback for this tile
      for (uint32_t j = 0; j < n; ++j) {
        const uint64_t st = dev::read_lane64(bj, j);
        const uint32_t ln = dev::read_lane(lj, j);
        const uint32_t sum = dev::wave_image_sum<2, kRef>(a.arena, st, ln, OP == kFill && ln >= 30);
        if (lane == 0) emit<OP>(a, k0 + j, sum, st, ln);
      }
      continue;
    }
    uint32_t field = 0;
    if (OP == kFill && lane < n && lj >= 30) field = *reinterpret_cast<const uint16_t *>(a.arena + bj + 28);

    const uint32_t lead = static_cast<uint32_t>(s0 - A0);
    const uint32_t span = static_cast<uint32_t>(s1 - A0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const uint32_t last_chunk = (span - 1) >> 4;
    const uint32_t rb = static_cast<uint32_t>(bj - A0);  // boundary j, relative to A0
    const bool router = lane >= 1 && lane < n;
    const uint8_t *base = a.arena + A0;
    uint32_t carry = 0;
    for (uint32_t s = 0; s < nsteps; s += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint32_t ci = ((s + u) << 6) + lane;
        ci = ci < last_chunk ? ci : last_chunk;  // clamp: always a legal address
        v[u] = dev::load16_nt(base + 16 * static_cast<uint64_t>(ci));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t st = s + u;
        if (st < nsteps) {  // wave-uniform
          const uint32_t sb = st << 10;
          if (router && rb - sb < 1024u) slot[(rb - sb) >> 4] = lane | ((rb & 15u) << 8) | 0x10000u;
          __builtin_amdgcn_wave_barrier();
          const uint32_t route = slot[lane];
          slot[lane] = 0;
          const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
          u32x4 w = v[u];
          int32_t lo = 0;
          if (sb == 0 || sb + 1024 > span) {  // span edge: mask words outside [lead, span)
            lo = min(max(static_cast<int32_t>(lead) - crel, 0), 16);
            const int32_t hi = min(max(static_cast<int32_t>(span) - crel, 0), 16);
            const uint32_t wm = dev::word_mask(lo, hi);
            if (wm != 0xFFu) w = dev::apply_mask(w, wm);
          }
          const uint32_t tot = dev::ref_chunk_sum(w);
          uint32_t head = 0;
          if (route) {
            const int32_t r = static_cast<int32_t>((route >> 8) & 15u);
            head = dev::ref_chunk_sum(dev::apply_mask(w, dev::word_mask(lo, r)));
          }
          const uint32_t incl = dev::wave_inclusive_scan(tot);
          if (route) pb[route & 63u] = carry + (incl - tot) + head;
          carry += dev::read_lane(incl, 63);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < n) {
      const uint32_t p_start = lane == 0 ? 0u : pb[lane];
      const uint32_t p_end = lane + 1 == n ? carry : pb[lane + 1];
      emit<OP>(a, k0 + lane, p_end - p_start - field, bj, lj);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int U, int OP, bool FIXED>
hipError_t launch_one(const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  const uint64_t ntiles = (a.count + a.tile - 1) / a.tile;
  uint64_t blocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
  static const uint32_t per_cu = dev::resident_blocks_per_cu(span_kernel<U, OP, FIXED>);
  const uint64_t max_blocks = static_cast<uint64_t>(per_cu) * num_cus;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((span_kernel<U, OP, FIXED>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                     stream, a);
  return hipGetLastError();
}

template <int OP>
hipError_t dispatch_fixed(bool fixed, const SpanArgs &a, uint32_t mb, hipStream_t s) {
  return fixed ? launch_one<4, OP, true>(a, mb, s) : launch_one<4, OP, false>(a, mb, s);
}

}  // namespace

uint32_t span_tile_for_len(uint64_t typical_len) {
  if (typical_len == 0) typical_len = 1;
  uint64_t t = (24u << 10) / typical_len;
  if (t < 1) t = 1;
  if (t > 63) t = 63;
  return static_cast<uint32_t>(t);
}

hipError_t launch_span(int op, bool fixed, const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.tile < 1 || a.tile > 63) return hipErrorInvalidValue;
  switch (op) {
    case kChecksum: return dispatch_fixed<kChecksum>(fixed, a, num_cus, stream);
    case kFill: return dispatch_fixed<kFill>(fixed, a, num_cus, stream);
    case kVerify: return dispatch_fixed<kVerify>(fixed, a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
