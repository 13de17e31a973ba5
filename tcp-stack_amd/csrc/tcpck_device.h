// tcpck_device.h -- device helpers shared by the gfx950 checksum kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcpck_internal.h"

namespace tcpck {
namespace dev {

using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / 64;

// 256-thread blocks of `kernel` resident per CU (occupancy query, >= 1).  The
// grid-stride kernels launch exactly num_cus x this many blocks, so every block
// starts at once and none waits for a slot (no second, tail wave of blocks).
template <typename Kernel>
inline uint32_t resident_blocks_per_cu(Kernel kernel) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
  return static_cast<uint32_t>(nb);
}

// Grid oversubscription for the run-per-wave kernels.  With one run per
// resident wave, the SIMD's age-ordered issue arbitration finishes the oldest
// slot ~2x before the youngest and the last runs stream alone; launching M x
// the resident grid lets the dispatcher refill freed slots with fresh, smaller
// runs.  requested: 0 = by size -- the largest power of two <= max_m that keeps
// runs >= min_run bytes (M = 12/16/24/40 measured 1-4% below M = 8/32 on the
// run kernels; C2 rstream 82.8% at M = 7, 87.9% at M = 32 back to back,
// profiles/r01/oversub_c2c3.log, b2b_c2c3.log) -- else explicit.
inline uint32_t oversub_for(uint32_t requested, uint64_t bytes, uint64_t resident_waves, uint32_t max_m,
                            uint32_t min_run = 4u << 10) {
  if (requested) return requested;
  const uint64_t q = bytes / (resident_waves * min_run + 1);
  uint32_t m = 1;
  while (2 * m <= max_m && 2 * m <= q) m *= 2;
  return m;
}

// Offset (relative to `arena`, wrapping) of the 16-byte-aligned ADDRESS at or
// below arena + off: loads stay naturally aligned even when the caller's arena
// pointer is not (the few bytes read before an image are masked, and they lie
// in the same 16-byte block -- hence the same page -- as a byte of the image).
__device__ __forceinline__ uint64_t align16_rel(const uint8_t *arena, uint64_t off) {
  const uint64_t mis = reinterpret_cast<uint64_t>(arena) & 15u;
  return ((off + mis) & ~uint64_t{15}) - mis;
}

// Same for the 128-byte (cache line) aligned address at or below arena + off.
__device__ __forceinline__ uint64_t align128_rel(const uint8_t *arena, uint64_t off) {
  const uint64_t mis = reinterpret_cast<uint64_t>(arena) & 127u;
  return ((off + mis) & ~uint64_t{127}) - mis;
}

// 16-byte streaming load, nontemporal (global_load_dwordx4 ... nt): the batch
// is read exactly once, so keep it from displacing other lines.
__device__ __forceinline__ u32x4 load16_nt(const uint8_t *p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

// Word-validity mask of a 16-byte chunk for the byte range [lo, hi) (both even,
// clamped to [0, 16]) -> 8-bit mask, bit i = u16 word i valid.
__device__ __forceinline__ uint32_t word_mask(int32_t lo, int32_t hi) {
  return ((1u << (hi >> 1)) - 1u) & ~((1u << (lo >> 1)) - 1u);
}

// 8-bit word mask -> AND mask for dword j of the chunk.
__device__ __forceinline__ uint32_t dword_mask(uint32_t wm, int j) {
  const uint32_t t = (wm >> (2 * j)) & 3u;
  return ((t & 1u) ? 0x0000FFFFu : 0u) | ((t & 2u) ? 0xFFFF0000u : 0u);
}

__device__ __forceinline__ u32x4 apply_mask(u32x4 w, uint32_t wm) {
  w.x &= dword_mask(wm, 0);
  w.y &= dword_mask(wm, 1);
  w.z &= dword_mask(wm, 2);
  w.w &= dword_mask(wm, 3);
  return w;
}

// Reference arithmetic (tcp-header.h:257-258): only the low 16 bits of the
// accumulator matter, so each dword adds both of its u16 halves as w + (w >> 16)
// (the high half's own carries land above bit 15).  Wrapping u32 adds keep the
// low 16 bits exact for any number of terms.
__device__ __forceinline__ uint32_t ref_add(uint32_t acc, uint32_t w) { return acc + w + (w >> 16); }

__device__ __forceinline__ uint32_t ref_chunk_sum(u32x4 w) {
  return ref_add(ref_add(ref_add(w.x + (w.x >> 16), w.y), w.z), w.w);
}

// Same sum with v_dot2_u32_u16 (both u16 halves times 1, plus the
// accumulator): 4 VALU per chunk instead of 8.
// (inline asm: hipcc 7.2 miscompiles the builtin on halves of a <4 x i32>
// load -- every dot read the first dword)
__device__ __forceinline__ uint32_t dot2_u16(uint32_t w, uint32_t acc) {
  uint32_t r;
  asm("v_dot2_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(w), "s"(0x00010001u), "v"(acc));
  return r;
}
__device__ __forceinline__ uint32_t ref_chunk_sum_dot(u32x4 w) {
  return dot2_u16(w.w, dot2_u16(w.z, dot2_u16(w.y, dot2_u16(w.x, 0u))));
}

// Raw buffer (SRSRC) loads: 32-bit lane offset + SGPR step offset, hardware
// range check (bytes past `bytes` read as 0, no fault), nontemporal (aux 2).
// Every caller passes wave-uniform values; readfirstlane says so to the
// compiler, which otherwise wraps each load of a descriptor built from a
// cross-lane result (a wave_max, a ds_swizzle) in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a)));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a >> 32)));
  const int n = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  void *u = reinterpret_cast<void *>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(u, 0, n, 0x00020000);
}
// In-place 2-B store of a FILL result into the image's checksum field, with
// the sc1 cache-policy bit: 4 % less time than a default-policy store for the
// scattered field writes (scripts/fill_write_probe.py --store-policy,
// profiles/r01/fill_store_policy.log; nt is worse).
__device__ __forceinline__ void store16_field(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, static_cast<int>(voff), 0, 16);
}

// ---- TcpHeaderN2H == TcpHeaderH2N on the 32 header bytes (tcp-header.h:193-221) ----
// v_perm_b32 selector for header dword j (header bytes 4j..4j+3): j = 0, 1, 4, 5
// hold a u32 field (addresses, seq, ack): byte reverse; j = 3 the two u16
// ports: swap within each half; j = 2, 6, 7: bytes 8-9 / 24-25 / 28-29 stay,
// the upper u16 (TcpLength, window, urgent pointer) swaps.
__device__ __forceinline__ uint32_t n2h_selector(uint32_t j) {
  return j == 3 ? 0x02030001u : ((j == 2 || j >= 6) ? 0x02030100u : 0x00010203u);
}
__device__ __forceinline__ uint32_t n2h_dword(uint32_t h, uint32_t sel) {
  return __builtin_amdgcn_perm(h, h, sel);
}

__device__ __forceinline__ u32x4 load16_buf_nt(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(voff), static_cast<int>(soff), 2);
  return u32x4{v.x, v.y, v.z, v.w};
}

// RFC 1071: 32-bit one's-complement add (2^32 == 1 mod 0xFFFF).
__device__ __forceinline__ uint32_t rfc_add(uint32_t acc, uint32_t w) {
  const uint32_t s = acc + w;
  return s + (s < w ? 1u : 0u);
}

template <int MODE>
__device__ __forceinline__ uint32_t accumulate(uint32_t acc, uint32_t w) {
  if constexpr (MODE == kRef) {
    return ref_add(acc, w);
  } else {
    return rfc_add(acc, w);
  }
}

// Folds an accumulator to 16 significant bits: unchanged mod 2^16 (REF), or
// mod 0xFFFF keeping zero-ness (RFC 1071).
template <int MODE>
__device__ __forceinline__ uint32_t fold_lane(uint32_t acc) {
  if constexpr (MODE == kRef) {
    return acc & 0xFFFFu;
  } else {
    acc = (acc & 0xFFFFu) + (acc >> 16);
    return (acc & 0xFFFFu) + (acc >> 16);
  }
}

template <int MODE>
__device__ __forceinline__ uint16_t finish(uint32_t sum) {
  if constexpr (MODE == kRef) {
    return static_cast<uint16_t>(~sum);  // tcp-header.h:262: ~ truncated to u16, no fold
  } else {
    sum = (sum & 0xFFFFu) + (sum >> 16);
    sum = (sum & 0xFFFFu) + (sum >> 16);
    return static_cast<uint16_t>(~sum);
  }
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

// 64-lane inclusive prefix sum with DPP (gfx9 family): row_shr 1,2,4,8 builds
// 16-lane scans, row_bcast:15 / row_bcast:31 carry rows into the rows above.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

__device__ __forceinline__ uint32_t read_lane(uint32_t x, uint32_t lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), static_cast<int>(lane)));
}

__device__ __forceinline__ uint64_t read_lane64(uint64_t x, uint32_t lane) {
  const uint32_t lo = read_lane(static_cast<uint32_t>(x), lane);
  const uint32_t hi = read_lane(static_cast<uint32_t>(x >> 32), lane);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Sum of the first r/2 words of a 16-byte chunk given as four dwords; r even
// in [0, 16).  REF arithmetic (low 16 bits meaningful) unless EXACT (the exact
// u32 word sum, for RFC 1071).  Used by the scalar boundary walks with
// wave-uniform inputs (readlane'd dwords): scalar code.
template <bool EXACT = false>
__device__ __forceinline__ uint32_t words_before(uint32_t r, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
  const uint32_t nw = r >> 1;
  uint32_t h = 0;
  auto both = [](uint32_t d) -> uint32_t { return EXACT ? (d & 0xFFFFu) + (d >> 16) : d + (d >> 16); };
  if (nw >= 2) h += both(x);
  if (nw >= 4) h += both(y);
  if (nw >= 6) h += both(z);
  if (nw & 1) {
    const uint32_t d = nw == 1 ? x : (nw == 3 ? y : (nw == 5 ? z : w));
    h += d & 0xFFFFu;
  }
  return h;
}

// Sum (REF arithmetic, low 16 bits meaningful) of the image [start, start+len)
// computed by one whole wave (64 lanes x U loads of 16 B in flight); the word at
// byte `start + 28` is excluded when exclude_field (send-side fill).  Result is
// the same in every lane.
template <int U, int MODE>
__device__ __forceinline__ uint32_t wave_image_sum(const uint8_t *arena, uint64_t start, uint32_t len,
                                                   bool exclude_field) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t a0 = align16_rel(arena, start);
  const uint8_t *p0 = arena + a0;
  const int32_t lead = static_cast<int32_t>(start - a0);
  const int64_t span64 = lead + static_cast<int64_t>(len);
  const uint32_t nch = static_cast<uint32_t>((span64 + 15) >> 4);
  const int64_t field = exclude_field ? lead + 28 : -64;
  uint32_t acc = 0;
  for (uint32_t i0 = lane; i0 < nch; i0 += 64 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * 64;
      v[u] = load16_nt(p0 + 16 * static_cast<uint64_t>(i < nch ? i : nch - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rel = 16 * static_cast<int64_t>(i0 + u * 64);
      const int32_t lo = static_cast<int32_t>(min(max(lead - rel, int64_t{0}), int64_t{16}));
      const int32_t hi = static_cast<int32_t>(min(max(span64 - rel, int64_t{0}), int64_t{16}));
      uint32_t wm = word_mask(lo, hi);
      const int64_t fb = field - rel;
      if (fb >= 0 && fb < 16) wm &= ~(1u << (fb >> 1));
      u32x4 w = v[u];
      if (wm != 0xFFu) w = apply_mask(w, wm);
      acc = accumulate<MODE>(acc, w.x);
      acc = accumulate<MODE>(acc, w.y);
      acc = accumulate<MODE>(acc, w.z);
      acc = accumulate<MODE>(acc, w.w);
    }
    if (MODE == kRfc1071) acc = fold_lane<MODE>(acc);
  }
  return group_sum<64>(fold_lane<MODE>(acc));
}

// First k in [0, count) with offsets[k] - base >= target (count if none);
// offsets ascending.  64-ary search: one probe per lane per level.
__device__ __forceinline__ uint64_t find_first_ge(const uint64_t *offsets, uint64_t base, uint64_t count, uint64_t target) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t lo = 0, hi = count;  // answer in [lo, hi]
  while (hi - lo > 64) {
    const uint64_t step = (hi - lo + 63) / 64;
    const uint64_t idx = lo + lane * step;
    const bool below = idx < hi && offsets[idx] - base < target;
    const uint32_t c = __popcll(__ballot(below));  // probes are sorted: lanes [0, c) are below
    const uint64_t nlo = c ? lo + (c - 1) * step + 1 : lo;
    const uint64_t nhi = min(hi, lo + c * step);
    lo = nlo;
    hi = nhi;
  }
  const uint64_t idx = lo + lane;
  const bool below = idx < hi && offsets[idx] - base < target;
  return lo + __popcll(__ballot(below));
}

// Both of first k with offsets[k] - base >= t0 / t1, searched in lockstep so
// the two dependent probe chains overlap (see dev::find_first_ge).
__device__ __forceinline__ void find_two(const uint64_t *offsets, uint64_t base, uint64_t count, uint64_t t0,
                                         uint64_t t1, uint64_t &r0, uint64_t &r1) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t lo[2] = {0, 0}, hi[2] = {count, count};
  const uint64_t t[2] = {t0, t1};
  while (hi[0] - lo[0] > 64 || hi[1] - lo[1] > 64) {
    uint64_t step[2], idx[2], v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      step[i] = hi[i] - lo[i] > 64 ? (hi[i] - lo[i] + 63) / 64 : 1;
      idx[i] = lo[i] + lane * step[i];
      v[i] = idx[i] < hi[i] ? offsets[idx[i]] : 0;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (hi[i] - lo[i] <= 64) continue;
      const bool below = idx[i] < hi[i] && v[i] - base < t[i];
      const uint32_t c = __popcll(__ballot(below));
      const uint64_t nlo = c ? lo[i] + (c - 1) * step[i] + 1 : lo[i];
      hi[i] = min(hi[i], lo[i] + c * step[i]);
      lo[i] = nlo;
    }
  }
  uint64_t v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint64_t idx = lo[i] + lane;
    v[i] = idx < hi[i] ? offsets[idx] : 0;
  }
  const bool b0 = lo[0] + lane < hi[0] && v[0] - base < t0;
  const bool b1 = lo[1] + lane < hi[1] && v[1] - base < t1;
  r0 = lo[0] + __popcll(__ballot(b0));
  r1 = lo[1] + __popcll(__ballot(b1));
}

// Equal-count run split without a device division: count = q * waves + r,
// wave w owns [w q + min(w, r), +q + (w < r)); q and r come from the launcher.
__device__ __forceinline__ void count_split(uint64_t wid, uint64_t q, uint64_t r, uint64_t &kb, uint64_t &ke) {
  kb = wid * q + (wid < r ? wid : r);
  ke = kb + q + (wid < r ? 1u : 0u);
}

// XCD-aware block order (bijective for any grid): blocks b and b + 8 share an
// XCD (round-robin dispatch; MI355X_MICROARCH.md, Workgroup dispatch), so
// the blocks labelled x = b % 8 get one contiguous range of logical ids.
// Speed only: correctness never depends on where a block runs.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// XCD-chunked block order: the blocks of one XCD take groups of 2^lc
// consecutive ids, the groups of the 8 XCDs interleaved -- neighbouring runs
// share an XCD (and its L2) while the 8 XCDs still stream nearby addresses.
// Bijective on the largest multiple of 8 * 2^lc blocks; the rest keep their id.
__device__ __forceinline__ uint32_t xcd_chunk_block(uint32_t b, uint32_t nb, uint32_t lc) {
  const uint32_t full = (nb >> (3 + lc)) << (3 + lc);
  if (b >= full) return b;
  const uint32_t i = b >> 3;  // the block's index among its XCD's blocks
  return ((((i >> lc) << 3) + (b & 7u)) << lc) + (i & ((1u << lc) - 1u));
}

// Block order selector for the run kernels' runtime argument: kOrderDefault
// keeps blockIdx, kOrderXcd is xcd_block, anything else the chunked order
// with groups of 2^lc blocks.
constexpr uint32_t kOrderDefault = 0xFFu;
constexpr uint32_t kOrderXcd = 0xFEu;
__device__ __forceinline__ uint32_t ordered_block(uint32_t b, uint32_t nb, uint32_t lc) {
  if (lc == kOrderDefault) return b;
  if (lc == kOrderXcd) return xcd_block(b, nb);
  return xcd_chunk_block(b, nb, lc);
}

// SPLIT 0: byte-balanced runs (two 64-ary searches over the offsets);
// SPLIT 1: equal image counts (no search; balance only statistical) -- tuning.

}  // namespace dev
}  // namespace tcpck
