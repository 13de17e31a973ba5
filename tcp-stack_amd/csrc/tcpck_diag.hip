// tcpck_diag.hip -- streaming micro-kernels for timing experiments only (their
// outputs are not checksums).  Each wave reads one contiguous, 128-B aligned
// run of the buffer, LPB 16-byte chunks per lane per step (a lane's chunks are
// adjacent: lane l covers bytes [16 LPB l, 16 LPB (l+1)) of the step), U steps
// in flight, optionally with the per-step 64-lane DPP scan the checksum
// kernels need.  Answers: how much does per-step (scalar + scan) overhead cost,
// and what does a wider per-lane stride do to the memory pipeline?
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

template <int LPB, int U, bool SCAN>
__global__ void __launch_bounds__(kBlock) diag_stream_kernel(const uint8_t *buf, uint64_t bytes, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  const uint64_t lines = bytes >> 7;
  const uint64_t b0 = (wid * lines / W) << 7;
  const uint64_t b1 = ((wid + 1) * lines / W) << 7;
  if (b0 >= b1) return;
  constexpr uint32_t kStep = 1024u * LPB;
  const uint32_t nsteps = static_cast<uint32_t>((b1 - b0 + kStep - 1) / kStep);
  const uint32_t last_chunk = static_cast<uint32_t>((b1 - b0) >> 4) - 1;
  const uint8_t *base = buf + b0;
  auto ld = [&](uint32_t st, int i) -> u32x4 {
    const uint32_t ci = min(st * (64u * LPB) + lane * LPB + static_cast<uint32_t>(i), last_chunk);
    return dev::load16_nt(base + 16 * static_cast<uint64_t>(ci));
  };
  u32x4 ring[U][LPB];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < LPB; ++i) ring[u][i] = ld(static_cast<uint32_t>(u), i);
  uint32_t carry = 0;
  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t t = 0;
#pragma unroll
      for (int i = 0; i < LPB; ++i) t += dev::ref_chunk_sum(ring[u][i]);
      if constexpr (SCAN) {
        const uint32_t incl = dev::wave_inclusive_scan(t);
        carry += dev::read_lane(incl, 63);
      } else {
        carry += t;
      }
#pragma unroll
      for (int i = 0; i < LPB; ++i) ring[u][i] = ld(g + u + U, i);
    }
  }
  if (lane == 0) out[wid] = carry;
}

// Block-shared dynamic units: a 1024-thread block (16 waves, 4 per SIMD, of
// different ages) owns an equal static byte range, cut into units of UNIT KiB
// that its waves take from an LDS counter (ds_add_rtn: lgkmcnt, no interplay
// with the load ring's vmcnt).  The ring rolls from one unit into the next
// (the next unit is taken one unit ahead), so waves the SIMD favours simply
// take more units and all waves of the block finish together.
template <int U, int UNIT>
__global__ void __launch_bounds__(1024) diag_dyn_kernel(const uint8_t *buf, uint64_t bytes, uint32_t *out) {
  __shared__ uint32_t s_next;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lines = bytes >> 7;
  const uint64_t b0 = (static_cast<uint64_t>(blockIdx.x) * lines / gridDim.x) << 7;
  const uint64_t b1 = (static_cast<uint64_t>(blockIdx.x + 1) * lines / gridDim.x) << 7;
  constexpr uint32_t kUnit = UNIT * 1024u;
  const uint32_t range = static_cast<uint32_t>(b1 - b0);
  const uint32_t nunits = (range + kUnit - 1) / kUnit;
  if (threadIdx.x == 0) s_next = 0;
  __syncthreads();
  const uint8_t *base = buf + b0;
  auto grab = [&]() -> uint32_t {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&s_next, 1u);
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(t)));
  };
  uint32_t cur = grab();
  if (cur >= nunits) return;
  uint32_t nxt = grab();
  const uint32_t last_chunk = (range >> 4) - 1;
  // virtual step v of the wave: steps of unit cur are v in [vcur, vcur + kSteps)
  constexpr uint32_t kSteps = UNIT;
  uint32_t vcur = 0;
  auto addr_of = [&](uint32_t v) -> uint32_t {  // chunk index of lane for virtual step v
    const uint32_t t = v - vcur;
    const uint32_t u = t < kSteps ? cur : nxt;  // units are >= U steps: at most one ahead
    const uint32_t tt = t < kSteps ? t : t - kSteps;
    const uint32_t ci = u * (kUnit >> 4) + (tt << 6) + lane;
    return min(ci, last_chunk);  // invalid next unit / range end: clamp (masked below)
  };
  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = dev::load16_nt(base + 16 * static_cast<uint64_t>(addr_of(u)));
  uint32_t carry = 0;
  uint32_t v = 0;
  while (true) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cbyte = (cur * (kUnit >> 4) + ((v + u - vcur) << 6) + lane) << 4;
      u32x4 w = ring[u];
      if (cbyte >= range) w = u32x4{0, 0, 0, 0};
      const uint32_t t = dev::ref_chunk_sum(w);
      const uint32_t incl = dev::wave_inclusive_scan(t);
      carry += dev::read_lane(incl, 63);
      ring[u] = dev::load16_nt(base + 16 * static_cast<uint64_t>(addr_of(v + u + U)));
    }
    v += U;
    if (v - vcur >= kSteps) {  // unit done (kSteps multiple of U)
      if (nxt >= nunits) break;
      cur = nxt;
      vcur += kSteps;
      nxt = grab();
    }
  }
  if (lane == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = carry;
}

template <int U, int UNIT>
hipError_t launch_dyn(const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, diag_dyn_kernel<U, UNIT>, 1024, 0) != hipSuccess || nb < 1)
    nb = 1;
  hipLaunchKernelGGL((diag_dyn_kernel<U, UNIT>), dim3(static_cast<uint32_t>(nb) * num_cus), dim3(1024), 0, s, buf,
                     bytes, out);
  return hipGetLastError();
}

// Cache-policy bits of the stream's loads: the bare stream (1x16 B, U4, scan,
// one run per wave, grid oversubscribed 8x) with raw buffer loads whose aux
// operand is AUX (bit 0 sc0, bit 1 nt, bit 4 sc1 on gfx950).
// XCD: blocks that share an XCD take consecutive runs (dev::xcd_block).
template <int AUX, bool XCD = false>
__global__ void __launch_bounds__(kBlock) diag_cpol_kernel(const uint8_t *buf, uint64_t bytes, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t NW = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(XCD ? dev::xcd_block(blockIdx.x, gridDim.x) : blockIdx.x) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint64_t lines = bytes >> 7;
  const uint64_t b0 = (wid * lines / NW) << 7;
  const uint64_t b1 = ((wid + 1) * lines / NW) << 7;
  if (b0 >= b1) return;
  const uint32_t nsteps = static_cast<uint32_t>((b1 - b0 + 1023) >> 10);
  const auto rsrc = dev::make_rsrc(buf + b0, static_cast<uint32_t>(b1 - b0));
  auto ld = [&](uint32_t st) -> u32x4 {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), static_cast<int>(st << 10), AUX);
    return u32x4{v.x, v.y, v.z, v.w};
  };
  u32x4 ring[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ring[u] = ld(static_cast<uint32_t>(u));
  uint32_t carry = 0;
  for (uint32_t g = 0; g < nsteps; g += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t t = dev::ref_chunk_sum(ring[u]);
      const uint32_t incl = dev::wave_inclusive_scan(t);
      carry += dev::read_lane(incl, 63);
      ring[u] = ld(g + u + 4);
    }
  }
  if (lane == 0) out[wid] = carry;
}

template <int AUX, bool XCD = false>
hipError_t launch_cpol(const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s,
                       uint32_t m = 8) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(diag_cpol_kernel<AUX, XCD>);
  hipLaunchKernelGGL((diag_cpol_kernel<AUX, XCD>), dim3(per_cu * num_cus * m), dim3(kBlock), 0, s, buf, bytes, out);
  return hipGetLastError();
}

// In-place FILL write cost: the bare stream (1x16 B, U4, scan) over a buffer
// of 1492-B images, plus one store per image at its checksum field (byte 28):
// W bytes aligned down to W (W = 2, 4: the field's lane; W >= 16: every lane
// whose 16-B chunk lies in the W-byte block, writing back the data it read).
// Answers: is the cost of FILL the sub-line write itself, and does a wider,
// aligned write-back of data already in registers avoid it?
// SAUX >= 0: the field stores are raw buffer stores with cache-policy bits SAUX
// (bit 0 sc0, bit 1 nt, bit 4 sc1): does a write-through / streaming store
// reach HBM while the image's DRAM row is still open, instead of as a later
// write-back of a partially dirty line?
template <int W, int SAUX = -1>
__global__ void __launch_bounds__(kBlock) diag_fill_kernel(uint8_t *buf, uint64_t bytes, uint32_t *out) {
  constexpr uint32_t kS = 1492;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t NW = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint64_t lines = bytes >> 7;
  const uint64_t b0 = (wid * lines / NW) << 7;
  const uint64_t b1 = ((wid + 1) * lines / NW) << 7;
  if (b0 >= b1) return;
  const uint32_t nsteps = static_cast<uint32_t>((b1 - b0 + 1023) >> 10);
  const uint32_t last_chunk = static_cast<uint32_t>((b1 - b0) >> 4) - 1;
  uint8_t *base = buf + b0;
  auto ld = [&](uint32_t st) -> u32x4 {
    return dev::load16_nt(base + 16 * static_cast<uint64_t>(min((st << 6) + lane, last_chunk)));
  };
  const auto wrsrc = dev::make_rsrc(base, static_cast<uint32_t>(b1 - b0));
  // first field at or after b0 (absolute), then every kS bytes
  uint64_t nf = ((b0 + kS - 1 - 28) / kS) * kS + 28;
  if (nf < b0) nf += kS;
  u32x4 ring[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ring[u] = ld(static_cast<uint32_t>(u));
  uint32_t carry = 0;
  for (uint32_t g = 0; g < nsteps; g += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t st = g + u;
      const uint64_t sb = b0 + (static_cast<uint64_t>(st) << 10);
      const u32x4 w = ring[u];
      const uint32_t t = dev::ref_chunk_sum(w);
      const uint32_t incl = dev::wave_inclusive_scan(t);
      carry += dev::read_lane(incl, 63);
      if (W > 0) {
        while (nf < sb + 1024 && nf < b1) {
          const uint64_t c = sb + 16 * lane;  // this lane's chunk (absolute)
          if constexpr (W < 16) {
            const uint64_t blk = nf & ~static_cast<uint64_t>(W - 1);
            if (c <= blk && blk < c + 16) {
              if constexpr (SAUX >= 0) {
                __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(t), wrsrc, static_cast<int>(blk - b0), 0, SAUX);
              } else {
                if (W == 2) *reinterpret_cast<uint16_t *>(buf + blk) = static_cast<uint16_t>(t);
                if (W == 4) *reinterpret_cast<uint32_t *>(buf + blk) = t;
              }
            }
          } else {
            const uint64_t blk = nf & ~static_cast<uint64_t>(W - 1);
            if (c >= blk && c + 16 <= blk + W && c + 16 <= b1) {
              if constexpr (SAUX >= 0) {
                typedef unsigned v4u __attribute__((ext_vector_type(4)));
                __builtin_amdgcn_raw_buffer_store_b128(v4u{w.x, w.y, w.z, w.w}, wrsrc, static_cast<int>(c - b0), 0, SAUX);
              } else {
                *reinterpret_cast<u32x4 *>(buf + c) = w;
              }
            }
          }
          nf += kS;
        }
      }
      ring[u] = ld(st + 4);
    }
  }
  if (lane == 0) out[wid] = carry;
}

// The same field writes as a separate write-only pass: one thread per image.
template <int W>
__global__ void __launch_bounds__(kBlock) diag_scatter_kernel(uint8_t *buf, uint64_t n, uint32_t v) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n) return;
  if (W == 2) *reinterpret_cast<uint16_t *>(buf + k * 1492 + 28) = static_cast<uint16_t>(v + k);
  if (W == 4) *reinterpret_cast<uint32_t *>(buf + k * 1492 + 28) = static_cast<uint32_t>(v + k);
}

template <int W, int SAUX = -1>
hipError_t launch_fill(uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(diag_fill_kernel<W, SAUX>);
  hipLaunchKernelGGL((diag_fill_kernel<W, SAUX>), dim3(per_cu * num_cus * 8), dim3(kBlock), 0, s, buf, bytes, out);
  return hipGetLastError();
}

template <int W>
hipError_t launch_fill_aux(int aux, uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s) {
  switch (aux) {
    case 0: return launch_fill<W, 0>(buf, bytes, out, num_cus, s);
    case 1: return launch_fill<W, 1>(buf, bytes, out, num_cus, s);
    case 2: return launch_fill<W, 2>(buf, bytes, out, num_cus, s);
    case 3: return launch_fill<W, 3>(buf, bytes, out, num_cus, s);
    case 16: return launch_fill<W, 16>(buf, bytes, out, num_cus, s);
    case 17: return launch_fill<W, 17>(buf, bytes, out, num_cus, s);
    case 18: return launch_fill<W, 18>(buf, bytes, out, num_cus, s);
    case 19: return launch_fill<W, 19>(buf, bytes, out, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

template <int LPB, int U, bool SCAN>
hipError_t launch_one(const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s,
                      uint32_t oversub = 1) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(diag_stream_kernel<LPB, U, SCAN>);
  hipLaunchKernelGGL((diag_stream_kernel<LPB, U, SCAN>), dim3(per_cu * num_cus * (oversub ? oversub : 1)),
                     dim3(kBlock), 0, s, buf, bytes, out);
  return hipGetLastError();
}

// Device copy ceiling (timing only): the first half of buf copied to the
// second half.  RUN: wave w copies one contiguous run in 1 KiB steps (lane l:
// 16 B at 1024 t + 16 l), U steps in flight, nt loads; else a grid-stride float4
// copy, U loads issued before their U stores.  SPOL: store aux bits (0
// default, 2 nt, 16 sc1).  The measure segmentation's read + write rate is
// judged against (profiles/DESIGN_history_r01-r04.md section 6).
template <int U, int SPOL, bool RUN>
__global__ void __launch_bounds__(kBlock) diag_copy_kernel(uint8_t *buf, uint64_t bytes) {
  const uint64_t half = (bytes >> 1) & ~uint64_t{127};
  const uint8_t *src = buf;
  uint8_t *dst = buf + half;
  const uint64_t n16 = half >> 4;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  if constexpr (RUN) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
    const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
    const uint64_t lines = half >> 7;
    const uint64_t b0 = (wid * lines / W) << 7, b1 = ((wid + 1) * lines / W) << 7;
    if (b0 >= b1) return;
    const uint32_t span = static_cast<uint32_t>(b1 - b0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const auto rs = dev::make_rsrc(src + b0, span);
    const auto rd = dev::make_rsrc(dst + b0, span);
    v4u ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      ring[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(lane << 4), static_cast<int>(u << 10), 2);
    for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t st = g + u;
        if (st < nsteps)
          __builtin_amdgcn_raw_buffer_store_b128(ring[u], rd, static_cast<int>(lane << 4), static_cast<int>(st << 10), SPOL);
        ring[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(lane << 4), static_cast<int>((st + U) << 10), 2);
      }
    }
  } else {
    const uint64_t T = static_cast<uint64_t>(gridDim.x) * kBlock;
    const v4u *s4 = reinterpret_cast<const v4u *>(src);
    v4u *d4 = reinterpret_cast<v4u *>(dst);
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n16; i += U * T) {
      v4u r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = i + u * T < n16 ? __builtin_nontemporal_load(s4 + i + u * T) : v4u{};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i + u * T < n16) {
          if constexpr (SPOL == 2)
            __builtin_nontemporal_store(r[u], d4 + i + u * T);
          else
            d4[i + u * T] = r[u];
        }
      }
    }
  }
}

template <int U, int SPOL, bool RUN>
hipError_t launch_copy(uint8_t *buf, uint64_t bytes, uint32_t num_cus, hipStream_t s, uint32_t m) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(diag_copy_kernel<U, SPOL, RUN>);
  hipLaunchKernelGGL((diag_copy_kernel<U, SPOL, RUN>), dim3(per_cu * num_cus * m), dim3(kBlock), 0, s, buf, bytes);
  return hipGetLastError();
}

}  // namespace

// variant: LPB x U x scan: 0 = 1x4 scan, 1 = 1x4 no scan, 2 = 2x2 scan, 3 = 2x2 no scan,
// 4 = 4x1 scan, 5 = 2x4 scan, 6 = 4x2 scan, 7 = 1x2 scan;
// block-shared dynamic units (1x16 B, scan): 8 = U4 16 KiB units, 9 = U4 32 KiB,
// 10 = U4 8 KiB, 11 = U8 32 KiB; 0x1000 | w: in-place FILL write cost per 1492-B
// image (w = 0 none, 1 2 B, 2 4 B, 3 16 B, 4 32 B, 5 64 B, 6 128 B)
hipError_t launch_diag_stream(int variant, const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus,
                              hipStream_t s) {
  if (variant >= 0x5000) {  // copy ceiling: bits 0-1 U (2/4/8), 2-3 store policy (default/nt/sc1), 4 grid-stride,
                            // 8-11 grid multiple (x resident, 0 = 1)
    uint8_t *wb = const_cast<uint8_t *>(buf);
    const uint32_t m = (variant >> 8) & 0xFu ? static_cast<uint32_t>((variant >> 8) & 0xFu) : 1u;
    const int u = variant & 3, sp = (variant >> 2) & 3;
    const bool gs = (variant & 16) != 0;
#define TCPCK_COPY(UU, SS) (gs ? launch_copy<UU, SS, false>(wb, bytes, num_cus, s, m) : launch_copy<UU, SS, true>(wb, bytes, num_cus, s, m))
    if (u == 0) return sp == 0 ? TCPCK_COPY(2, 0) : (sp == 1 ? TCPCK_COPY(2, 2) : TCPCK_COPY(2, 16));
    if (u == 1) return sp == 0 ? TCPCK_COPY(4, 0) : (sp == 1 ? TCPCK_COPY(4, 2) : TCPCK_COPY(4, 16));
    return sp == 0 ? TCPCK_COPY(8, 0) : (sp == 1 ? TCPCK_COPY(8, 2) : TCPCK_COPY(8, 16));
#undef TCPCK_COPY
  }
  if (variant >= 0x4000) {  // in-place FILL write cost with store cache-policy bits: 0x4000 | aux (2 B), 0x4100 | aux (64 B)
    uint8_t *wb = const_cast<uint8_t *>(buf);
    return (variant & 0x100) ? launch_fill_aux<64>(variant & 0xFF, wb, bytes, out, num_cus, s)
                             : launch_fill_aux<2>(variant & 0xFF, wb, bytes, out, num_cus, s);
  }
  if (variant >= 0x3000) {  // nt stream, run order by XCD (bit 0) and grid multiple (bits 8..15)
    const uint32_t m = (variant >> 8) & 0xFu ? static_cast<uint32_t>((variant >> 8) & 0xFu) * 4u : 8u;
    return (variant & 1) ? launch_cpol<2, true>(buf, bytes, out, num_cus, s, m)
                         : launch_cpol<2, false>(buf, bytes, out, num_cus, s, m);
  }
  if (variant >= 0x2000) {  // load cache-policy bits
    switch (variant & 0xFF) {
      case 0: return launch_cpol<0>(buf, bytes, out, num_cus, s);
      case 1: return launch_cpol<1>(buf, bytes, out, num_cus, s);
      case 2: return launch_cpol<2>(buf, bytes, out, num_cus, s);
      case 3: return launch_cpol<3>(buf, bytes, out, num_cus, s);
      case 16: return launch_cpol<16>(buf, bytes, out, num_cus, s);
      case 17: return launch_cpol<17>(buf, bytes, out, num_cus, s);
      case 18: return launch_cpol<18>(buf, bytes, out, num_cus, s);
      case 19: return launch_cpol<19>(buf, bytes, out, num_cus, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (variant >= 0x1000) {  // in-place FILL write cost (timing only; writes into buf)
    uint8_t *wb = const_cast<uint8_t *>(buf);
    switch (variant & 0xFF) {
      case 0: return launch_fill<0>(wb, bytes, out, num_cus, s);
      case 1: return launch_fill<2>(wb, bytes, out, num_cus, s);
      case 2: return launch_fill<4>(wb, bytes, out, num_cus, s);
      case 3: return launch_fill<16>(wb, bytes, out, num_cus, s);
      case 4: return launch_fill<32>(wb, bytes, out, num_cus, s);
      case 5: return launch_fill<64>(wb, bytes, out, num_cus, s);
      case 6: return launch_fill<128>(wb, bytes, out, num_cus, s);
      case 7: {  // write-only pass, 2 B per image
        const uint64_t n = bytes / 1492;
        hipLaunchKernelGGL((diag_scatter_kernel<2>), dim3(static_cast<uint32_t>((n + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, s, wb, n, 7u);
        return hipGetLastError();
      }
      case 8: {  // the stream without writes, then the write-only pass
        hipError_t e = launch_fill<0>(wb, bytes, out, num_cus, s);
        if (e != hipSuccess) return e;
        const uint64_t n = bytes / 1492;
        hipLaunchKernelGGL((diag_scatter_kernel<2>), dim3(static_cast<uint32_t>((n + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, s, wb, n, 7u);
        return hipGetLastError();
      }
      default: return hipErrorInvalidValue;
    }
  }
  if (variant >> 8)  // 1x16 B, U4, scan, grid = (variant >> 8) x resident
    return launch_one<1, 4, true>(buf, bytes, out, num_cus, s, static_cast<uint32_t>(variant >> 8) & 0xFFu);
  switch (variant) {
    case 0: return launch_one<1, 4, true>(buf, bytes, out, num_cus, s);
    case 1: return launch_one<1, 4, false>(buf, bytes, out, num_cus, s);
    case 2: return launch_one<2, 2, true>(buf, bytes, out, num_cus, s);
    case 3: return launch_one<2, 2, false>(buf, bytes, out, num_cus, s);
    case 4: return launch_one<4, 1, true>(buf, bytes, out, num_cus, s);
    case 5: return launch_one<2, 4, true>(buf, bytes, out, num_cus, s);
    case 6: return launch_one<4, 2, true>(buf, bytes, out, num_cus, s);
    case 7: return launch_one<1, 2, true>(buf, bytes, out, num_cus, s);
    case 8: return launch_dyn<4, 16>(buf, bytes, out, num_cus, s);
    case 9: return launch_dyn<4, 32>(buf, bytes, out, num_cus, s);
    case 10: return launch_dyn<4, 8>(buf, bytes, out, num_cus, s);
    case 11: return launch_dyn<8, 32>(buf, bytes, out, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
