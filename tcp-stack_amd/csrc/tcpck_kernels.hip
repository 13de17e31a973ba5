// tcpck_kernels.hip -- the image-per-group ("seg") kernel: any layout.
//
// Semantics (parity mode, kRef): the reference's CalculateChecksum,
// filixi/TCP-stack include/tcp-header.h:252-263 -- little-endian u16 words
// summed into a u32 with no end-around carry, result ~sum truncated to u16,
// i.e. ~(sum mod 2^16).  kRfc1071 is the opt-in one's-complement sum.
//
// This kernel accepts every layout the C ABI allows (fixed stride with gaps,
// arbitrary even offsets/lengths in any order, zero-length images, both
// modes); the packed-layout fast paths are the run kernels (tcpck_rstream.hip,
// tcpck_vvstream.hip).
// Shape of the work: a pure HBM-read streaming reduction (~0.5 integer add per
// byte, no MFMA):
//   * G consecutive lanes own one image; lane l of the group reads the image's
//     16-byte chunks l, l+G, l+2G, ... so one wave-instruction reads 64/G
//     contiguous runs of G*16 bytes (1 KiB per wave-instruction in total);
//   * each lane issues U 16-byte nontemporal loads back to back before it
//     consumes any of them (U KiB in flight per wave, 32 waves per CU);
//   * chunk addresses past the image end are clamped to the image's last
//     chunk (always a legal address) and their words masked to zero, so the
//     loads are unconditional: no per-load branch, no per-load vmcnt(0);
//   * images start at arbitrary even offsets: the first chunk is the image
//     start rounded down to 16 B and its leading words are masked, the last
//     chunk's trailing words likewise (word-granular masks: even lengths that
//     are 2 mod 4 are exact);
//   * the G partial sums are combined with cross-lane xor shuffles, and lane 0
//     of the group stores the 2-byte result (kFill also writes it into bytes
//     28-29 of the image, tcp-header.h:177; kVerify stores checksum == 0).
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::u32x4;

template <int G, int U, int MODE, int OP, bool FIXED>
__global__ void __launch_bounds__(kBlock) seg_kernel(SegArgs a) {
  static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two <= 64");
  const uint32_t gl = threadIdx.x & (G - 1);
  const uint64_t groups_per_grid = static_cast<uint64_t>(gridDim.x) * (kBlock / G);
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  for (uint64_t k = (static_cast<uint64_t>(bid) * kBlock + threadIdx.x) / G; k < a.count;
       k += groups_per_grid) {
    const uint64_t start = FIXED ? k * a.stride : a.offsets[k] - a.base;
    const uint32_t len = FIXED ? a.len : a.lengths[k];
    const uint64_t a0 = dev::align16_rel(a.arena, start);     // 16-B aligned in absolute terms
    const uint8_t *p0 = a.arena + a0;
    const int64_t lead = static_cast<int64_t>(start - a0);    // masked bytes before the image
    const int64_t span = lead + static_cast<int64_t>(len);    // bytes from p0 to the image end
    const uint32_t nch = static_cast<uint32_t>((span + 15) >> 4);  // 16-byte chunks touched
    const int64_t field = (OP == kFill) ? lead + 28 : -64;    // checksum field counts as 0

    uint32_t acc = 0;
    for (uint32_t i0 = gl; i0 < nch; i0 += G * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * G;
        const uint32_t ic = i < nch ? i : nch - 1;  // clamp: always a legal address
        v[u] = dev::load16_nt(p0 + 16 * static_cast<uint64_t>(ic));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rel = 16 * static_cast<int64_t>(i0 + u * G);
        const int32_t lo = static_cast<int32_t>(min(max(lead - rel, int64_t{0}), int64_t{16}));
        const int32_t hi = static_cast<int32_t>(min(max(span - rel, int64_t{0}), int64_t{16}));
        uint32_t wm = dev::word_mask(lo, hi);
        if (OP == kFill) {
          const int64_t fb = field - rel;
          if (fb >= 0 && fb < 16) wm &= ~(1u << (fb >> 1));
        }
        u32x4 w = v[u];
        if (wm != 0xFFu) w = dev::apply_mask(w, wm);
        acc = dev::accumulate<MODE>(acc, w.x);
        acc = dev::accumulate<MODE>(acc, w.y);
        acc = dev::accumulate<MODE>(acc, w.z);
        acc = dev::accumulate<MODE>(acc, w.w);
      }
      if (MODE == kRfc1071) acc = dev::fold_lane<MODE>(acc);
    }
    const uint32_t sum = dev::group_sum<G>(dev::fold_lane<MODE>(acc));
    if (gl == 0) {
      const uint16_t c = dev::finish<MODE>(sum);
      if constexpr (OP == kVerify) {
        static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
      } else {
        if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
        if (OP == kFill && len >= 30)
          *reinterpret_cast<uint16_t *>(a.arena + start + 28) = c;  // stored raw, tcp-header.h:177
      }
    }
  }
}

// Jumbo images, W waves per image: the block owns one image at a time and
// thread t reads the image's 16-B chunks t, t + 64W, t + 128W, ... (each wave
// instruction still reads 1 KiB contiguous; the block 64W x 16 B).  The W
// wave sums meet in LDS.  With one image per block the dispatcher balances
// blocks of 64 KiB / W per wave instead of whole 64-KiB images per wave.
template <int W, int U, int MODE, int OP, bool FIXED>
__global__ void __launch_bounds__(64 * W) jumbo_kernel(SegArgs a) {
  constexpr uint32_t T = 64 * W;
  __shared__ uint32_t s_part[W];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  for (uint64_t k = bid; k < a.count; k += gridDim.x) {
    const uint64_t start = FIXED ? k * a.stride : a.offsets[k] - a.base;
    const uint32_t len = FIXED ? a.len : a.lengths[k];
    const uint64_t a0 = dev::align16_rel(a.arena, start);
    const uint8_t *p0 = a.arena + a0;
    const int64_t lead = static_cast<int64_t>(start - a0);
    const int64_t span = lead + static_cast<int64_t>(len);
    const uint32_t nch = static_cast<uint32_t>((span + 15) >> 4);
    const int64_t field = (OP == kFill) ? lead + 28 : -64;
    // a.rot: this image's chunks are read from chunk rot on, wrapping -- the
    // blocks in flight (consecutive images at the same 64-KiB phase for C4)
    // then read different offsets at the same time; whole 1 KiB wave steps stay
    // contiguous (rot a multiple of 64 chunks)
    const uint32_t rot = (a.rot && nch >= 128) ? ((static_cast<uint32_t>(k) * a.rot) % (nch >> 6)) << 6 : 0u;
    uint32_t acc = 0;
    for (uint32_t i0 = t; i0 < nch; i0 += T * U) {
      u32x4 v[U];
      uint32_t ie[U];  // the chunk read, after the rotation
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * T;
        const uint32_t r = i + rot;
        ie[u] = i < nch ? (r >= nch ? r - nch : r) : nch + i;  // past the image: masked below
        const uint32_t ic = i < nch ? ie[u] : nch - 1;  // clamp: always a legal address
        v[u] = dev::load16_nt(p0 + 16 * static_cast<uint64_t>(ic));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rel = 16 * static_cast<int64_t>(ie[u]);
        const int32_t lo = static_cast<int32_t>(min(max(lead - rel, int64_t{0}), int64_t{16}));
        const int32_t hi = static_cast<int32_t>(min(max(span - rel, int64_t{0}), int64_t{16}));
        uint32_t wm = dev::word_mask(lo, hi);
        if (OP == kFill) {
          const int64_t fb = field - rel;
          if (fb >= 0 && fb < 16) wm &= ~(1u << (fb >> 1));
        }
        u32x4 w = v[u];
        if (wm != 0xFFu) w = dev::apply_mask(w, wm);
        acc = dev::accumulate<MODE>(acc, w.x);
        acc = dev::accumulate<MODE>(acc, w.y);
        acc = dev::accumulate<MODE>(acc, w.z);
        acc = dev::accumulate<MODE>(acc, w.w);
      }
      if (MODE == kRfc1071) acc = dev::fold_lane<MODE>(acc);
    }
    const uint32_t ws = dev::group_sum<64>(dev::fold_lane<MODE>(acc));
    if (lane == 0) s_part[wv] = ws;
    __syncthreads();
    if (t == 0) {
      uint32_t sum = 0;
#pragma unroll
      for (int i = 0; i < W; ++i) sum += s_part[i];  // W x < 2^22: no overflow; finish folds
      const uint16_t c = dev::finish<MODE>(sum);
      if constexpr (OP == kVerify) {
        static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
      } else {
        if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
        if (OP == kFill && len >= 30) *reinterpret_cast<uint16_t *>(a.arena + start + 28) = c;
      }
    }
    __syncthreads();  // s_part is rewritten for the next image
  }
}

template <int W, int U, int MODE, int OP, bool FIXED>
hipError_t launch_jumbo(const SegArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = [] {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jumbo_kernel<W, U, MODE, OP, FIXED>, 64 * W, 0) !=
            hipSuccess || nb < 1)
      nb = 1;
    return static_cast<uint32_t>(nb);
  }();
  // one image per block (oversub 0) or at most oversub x the resident blocks (grid-stride)
  uint64_t blocks = a.count;
  const uint64_t cap = a.oversub ? static_cast<uint64_t>(per_cu) * num_cus * a.oversub : uint64_t{0x7FFFFFFF};
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((jumbo_kernel<W, U, MODE, OP, FIXED>), dim3(static_cast<uint32_t>(blocks)), dim3(64 * W), 0,
                     stream, a);
  return hipGetLastError();
}

template <int G, int U, int MODE, int OP, bool FIXED>
hipError_t launch_one(const SegArgs &a, uint32_t num_cus, hipStream_t stream) {
  const uint64_t groups_per_block = kBlock / G;
  uint64_t blocks = (a.count + groups_per_block - 1) / groups_per_block;
  // grid-stride kernel: launch exactly the resident blocks, never a second wave of them
  static const uint32_t per_cu = dev::resident_blocks_per_cu(seg_kernel<G, U, MODE, OP, FIXED>);
  const uint64_t max_blocks = static_cast<uint64_t>(per_cu) * num_cus * (a.oversub > 1 ? a.oversub : 1u);
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((seg_kernel<G, U, MODE, OP, FIXED>), dim3(static_cast<uint32_t>(blocks)),
                     dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int G, int U, int MODE, int OP>
hipError_t dispatch_fixed(bool fixed, const SegArgs &a, uint32_t mb, hipStream_t s) {
  if constexpr (G > 64) {  // G = 64 W: W waves per image
    return fixed ? launch_jumbo<G / 64, U, MODE, OP, true>(a, mb, s)
                 : launch_jumbo<G / 64, U, MODE, OP, false>(a, mb, s);
  } else {
    return fixed ? launch_one<G, U, MODE, OP, true>(a, mb, s)
                 : launch_one<G, U, MODE, OP, false>(a, mb, s);
  }
}

template <int G, int U, int MODE>
hipError_t dispatch_op(int op, bool fixed, const SegArgs &a, uint32_t mb, hipStream_t s) {
  switch (op) {
    case kChecksum: return dispatch_fixed<G, U, MODE, kChecksum>(fixed, a, mb, s);
    case kFill: return dispatch_fixed<G, U, MODE, kFill>(fixed, a, mb, s);
    case kVerify: return dispatch_fixed<G, U, MODE, kVerify>(fixed, a, mb, s);
    default: return hipErrorInvalidValue;
  }
}

template <int G, int U>
hipError_t dispatch_mode(int mode, int op, bool fixed, const SegArgs &a, uint32_t mb,
                         hipStream_t s) {
  return mode == kRef ? dispatch_op<G, U, kRef>(op, fixed, a, mb, s)
                      : dispatch_op<G, U, kRfc1071>(op, fixed, a, mb, s);
}

}  // namespace

// Images above 4 KiB: W waves per image, one block round (W x 4 KiB) just
// covering the image (scripts/xcd_probe.py --what jumbo,
// profiles/r01/jumbo_probe.log: 6 KiB W2 90.6%, 12 KiB W4 91.2%, 32 KiB W8
// 90.9%, 64 KiB W16 91.1%, against 80-85% for one wave per image).
SegShape shape_for_len(uint64_t typical_len) {
  if (typical_len <= 256) return kShapeSmall;
  if (typical_len <= 4096) return kShapeMss;
  if (typical_len <= 8192) return kShapeW2;
  if (typical_len <= 16384) return kShapeW4;
  if (typical_len <= 32768) return kShapeW8;
  return kShapeW16;
}

hipError_t launch_seg(int op, int mode, bool fixed, SegShape shape, const SegArgs &a,
                      uint32_t num_cus, hipStream_t stream) {
  switch (shape) {
    // the shapes AUTO picks (shape_for_len)
    case kShapeSmall: return dispatch_mode<8, 2>(mode, op, fixed, a, num_cus, stream);
    case kShapeMss: return dispatch_mode<16, 6>(mode, op, fixed, a, num_cus, stream);
    case kShapeW2: return dispatch_mode<128, 4>(mode, op, fixed, a, num_cus, stream);
    case kShapeW4: return dispatch_mode<256, 4>(mode, op, fixed, a, num_cus, stream);
    case kShapeW8: return dispatch_mode<512, 4>(mode, op, fixed, a, num_cus, stream);
    case kShapeW16: return dispatch_mode<1024, 2>(mode, op, fixed, a, num_cus, stream);
#ifdef TCPCK_PROBE
    // measurement-only shapes (libtcpck_probe.so)
    case kShapeJumbo: return dispatch_mode<64, 4>(mode, op, fixed, a, num_cus, stream);
    case kShapeWave2: return dispatch_mode<64, 2>(mode, op, fixed, a, num_cus, stream);
    case kShapeG32: return dispatch_mode<32, 3>(mode, op, fixed, a, num_cus, stream);
    case kShapeG4: return dispatch_mode<4, 8>(mode, op, fixed, a, num_cus, stream);
    case kShapeW16U4: return dispatch_mode<1024, 4>(mode, op, fixed, a, num_cus, stream);
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
