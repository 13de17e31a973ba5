// tcpck_gstream.hip -- fixed-stride packed batches of small power-of-two images
// (stride == length == S, S = 32 .. 1024 B, e.g. 32-B pure-ACK images):
// G = S / 16 lanes per image, no boundary resolution at all.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).
//
// When S divides the 1 KiB a wave reads per step and the arena is 16-B
// aligned, every 16-B chunk belongs to exactly one image and every step holds
// 1024 / S whole images in aligned groups of G lanes.  So a step is:
//   * lane l loads the 16 B at 1024 s + 16 l (one fully coalesced 1 KiB
//     request per wave-instruction, buffer load, nt), U steps in flight in a
//     register ring as in rstream;
//   * the lane's 8 words summed with v_dot2_u32_u16;
//   * a G-lane butterfly inside a DPP row (quad_perm xor 1 / xor 2,
//     row_half_mirror, row_mirror: after each stage every lane holds the sum of
//     its 2 / 4 / 8 / 16-lane group; G = 32, 64 add xor shuffles across rows);
//   * lane 0 of each group stores out[k]; kFill: lane 1 of the group holds the
//     checksum field (image bytes 28-29 = chunk 1, dword 3, low half), zeroes it
//     before the sum and stores the result there (tcp-header.h:177).
// No prefix scan, no LDS, no scalar walk: the vector work per step is ~10
// VALU, against ~30 for vvstream's FIXED mode that AUTO used for these sizes.
//
// Runs are contiguous ranges of whole steps (equal counts, split by the
// launcher); with a 128-B aligned arena no line is shared by two runs.
//
// Other multiples of 16 B up to 240 B (48, 80, 96 (64-B payloads), ... B;
// G = 3 .. 15 not a power of two): a step is the P = 64 / G whole images that
// fit one wave, B = P * S bytes (96 B: 10 images, 960 B, 60 lanes); the idle
// lanes load and store out of the buffer range (nothing moves).  Group sums
// come from a wave-wide inclusive scan (6 shuffles) and two reads of it at the
// group's edges.  Variants 0-2, 4, 0x80 and the FILL write-back 0x400 / 0x401.
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

// sum over aligned groups of G lanes; every lane of a group gets the group sum
template <int G>
__device__ __forceinline__ uint32_t lane_group_sum(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]: xor 1
  if constexpr (G >= 4) x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]: xor 2
  if constexpr (G >= 8) x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (G >= 16) x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false); // row_mirror
  if constexpr (G >= 32) x += __shfl_xor(x, 16, 64);
  if constexpr (G >= 64) x += __shfl_xor(x, 32, 64);
  return x;
}

// SPOL: results stored through a buffer resource over the run's out[] slice
// with these cache-policy bits (-1: plain global stores); LPOL: load policy
// bits (2 = nt).  Tuning (variant bits 8-11, 12, scripts/gstream_probe.py).
// WB >= 0 (kFill): every lane writes its whole 16-B chunk back, the field
// patched, with store policy WB: the image's lines leave as full-line writes
// instead of one masked partial write per image (twice the traffic).
// any G in [2, 64]: aligned groups of G lanes from lane 0 (the idle lanes past
// the last whole group get garbage)
template <int G>
__device__ __forceinline__ uint32_t lane_group_sum_any(uint32_t x, uint32_t lane) {
  if constexpr ((G & (G - 1)) == 0) {
    return lane_group_sum<G>(x);
  } else {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= static_cast<uint32_t>(d)) x += y;
    }
    const uint32_t base = (lane / G) * G;
    const uint32_t hi = __shfl(x, static_cast<int>(base + G - 1) & 63, 64);
    const uint32_t lo = __shfl(x, static_cast<int>(base + 63) & 63, 64);  // lane base - 1
    return base ? hi - lo : hi;
  }
}

template <int U, int G, int OP, int SPOL = -1, int LPOL = 2, bool FLINE = false, int WB = -1>
__global__ void __launch_bounds__(kBlock) gstream_kernel(GroupStreamArgs a) {
  constexpr uint32_t S = 16 * G;     // image bytes
  constexpr uint32_t P = 64 / G;     // images per step
  constexpr uint32_t B = P * S;      // step bytes (1024 for a power-of-two G)
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  uint64_t sb, se;  // the wave's steps [sb, se)
  dev::count_split(wid, a.per_wave, a.rem, sb, se);
  if (sb >= se) return;
  const uint64_t byte0 = sb * B;
  const uint64_t left = a.count * S - byte0;  // > 0: sb < steps
  const uint32_t nsteps = static_cast<uint32_t>(se - sb);
  const uint64_t run = static_cast<uint64_t>(nsteps) * B;
  // records cover the run's image bytes; loads past them (the batch tail, the
  // ring's look-ahead past the run) read 0 without a memory access
  const auto rsrc = dev::make_rsrc(a.arena + byte0, static_cast<uint32_t>(run < left ? run : left));
  const uint64_t k0 = sb * P + lane / G;  // image of this lane's chunk in the run's first step
  // lanes past the step's last whole image: offsets past any buffer range
  const bool live = lane < P * G;
  const uint32_t loff = live ? lane << 4 : 0x80000000u;
  const bool leader = live && (lane % G) == 0;
  constexpr uint32_t kOutBytes = OP == kVerify ? 1u : 2u;
  const uint64_t kend = (se * P < a.count) ? se * P : a.count;
  const auto orsrc = dev::make_rsrc(static_cast<uint8_t *>(a.out) + kOutBytes * sb * P,
                                    a.out ? static_cast<uint32_t>(kOutBytes * (kend - sb * P)) : 0u);
  // FLINE (kFill): lanes whose chunk lies in an image's first 128-B line (the
  // line holding the checksum field) load with the default cache policy, so
  // the line is still in L2 when the field store lands and leaves as a whole
  // line instead of a masked partial write
  const bool fline = FLINE && ((lane * 16u) % S) < 128u;
  auto load = [&](uint32_t voff) -> u32x4 {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    v4u v;
    if (fline) {
      v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(voff), 0, 0);
    } else {
      v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(voff), 0, LPOL);
    }
    return u32x4{v.x, v.y, v.z, v.w};
  };
  const bool field_lane = live && (lane % G) == 1;

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = load(static_cast<uint32_t>(u) * B + loff);

  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = g + u;
      if (st < nsteps) {  // wave-uniform
        u32x4 w = ring[u];
        if constexpr (OP == kFill) {
          if (field_lane) w.w &= 0xFFFF0000u;  // bytes 28-29 of the image read as 0
        }
        const uint32_t sum = lane_group_sum_any<G>(dev::ref_chunk_sum_dot(w), lane);
        const uint16_t c = static_cast<uint16_t>(~sum);  // tcp-header.h:262
        const uint64_t k = k0 + static_cast<uint64_t>(st) * P;
        if constexpr (SPOL >= 0) {
          const uint32_t vo = (st * P + lane / G) * kOutBytes;  // range-checked: images past the batch drop
          if constexpr (OP == kVerify) {
            if (leader) __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(c == 0), orsrc, static_cast<int>(vo), 0, SPOL);
          } else {
            if (leader) __builtin_amdgcn_raw_buffer_store_b16(c, orsrc, static_cast<int>(vo), 0, SPOL);
            if (OP == kFill && field_lane && k < a.count) dev::store16_field(rsrc, st * B + loff + 12, c);
          }
        } else if (OP == kFill && WB >= 0) {
          if (leader && a.out && k < a.count) static_cast<uint16_t *>(a.out)[k] = c;
          if (field_lane) w.w |= c;  // the field was zeroed above
          typedef unsigned v4u __attribute__((ext_vector_type(4)));
          // range-checked: chunks past the batch drop
          __builtin_amdgcn_raw_buffer_store_b128(v4u{w.x, w.y, w.z, w.w}, rsrc, static_cast<int>(st * B + loff), 0,
                                                 WB < 0 ? 0 : WB);
        } else if (k < a.count) {
          if constexpr (OP == kVerify) {
            if (leader) static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
          } else {
            if (leader && a.out) static_cast<uint16_t *>(a.out)[k] = c;
            if (OP == kFill && field_lane) dev::store16_field(rsrc, st * B + loff + 12, c);
          }
        }
      }
      // the slot's data is dead: refill in place (the step offset in the VGPR
      // offset, which the range check always covers)
      ring[u] = load((st + U) * B + loff);
    }
  }
}

template <int U, int G, int OP, int SPOL, int LPOL, bool FLINE, int WB = -1>
hipError_t launch_one(const GroupStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(gstream_kernel<U, G, OP, SPOL, LPOL, FLINE, WB>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  const uint64_t bytes = a.count * (16u * G);
  constexpr uint32_t B = (64 / G) * 16u * G;
  const uint64_t steps = (bytes + B - 1) / B;
  // runs of >= 4 KiB, up to 1024 x the resident grid (the rstream rule)
  uint64_t blocks = resident * dev::oversub_for(a.oversub, bytes, resident * kWavesPerBlock, 1024);
  const uint64_t need = (steps + kWavesPerBlock - 1) / kWavesPerBlock;  // >= 1 step per wave
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  GroupStreamArgs b = a;
  b.per_wave = steps / (blocks * kWavesPerBlock);
  b.rem = steps % (blocks * kWavesPerBlock);
  if ((b.per_wave + 1 + U) * B >= (uint64_t{1} << 31)) return hipErrorInvalidValue;  // u32 run offsets
  hipLaunchKernelGGL((gstream_kernel<U, G, OP, SPOL, LPOL, FLINE, WB>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, b);
  return hipGetLastError();
}

template <int U, int G, int SPOL, int LPOL, bool FLINE, int WB>
hipError_t by_op(int op, const GroupStreamArgs &a, uint32_t num_cus, hipStream_t s) {
#ifndef TCPCK_PROBE
  // AUTO sends only FILL here: vvstream / rstream CHECKSUM and VERIFY these
  // layouts equally fast or faster (profiles/DESIGN_history_r01-r04.md section 4, gstream)
  if (op != kFill) return hipErrorInvalidValue;
#endif
  switch (op) {
    case kFill: return launch_one<U, G, kFill, SPOL, LPOL, FLINE, WB>(a, num_cus, s);
#ifdef TCPCK_PROBE
    case kChecksum: return launch_one<U, G, kChecksum, SPOL, LPOL, false>(a, num_cus, s);
    case kVerify: return launch_one<U, G, kVerify, SPOL, LPOL, false>(a, num_cus, s);
#endif
    default: return hipErrorInvalidValue;
  }
}

template <int U, int SPOL = -1, int LPOL = 2, bool FLINE = false, int WB = -1>
hipError_t by_len(int op, const GroupStreamArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (a.len) {
    case 32: return by_op<U, 2, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    case 64: return by_op<U, 4, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    case 128: return by_op<U, 8, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    case 256: return by_op<U, 16, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    case 512: return by_op<U, 32, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    case 1024: return by_op<U, 64, SPOL, LPOL, FLINE, WB>(op, a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

// the other multiples of 16 B up to 240 B (scan-based group sums)
template <int U, int LPOL = 2, int WB = -1>
hipError_t by_len_np(int op, const GroupStreamArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (a.len) {
    case 48: return by_op<U, 3, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 80: return by_op<U, 5, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 96: return by_op<U, 6, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 112: return by_op<U, 7, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 144: return by_op<U, 9, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 160: return by_op<U, 10, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 176: return by_op<U, 11, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 192: return by_op<U, 12, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 208: return by_op<U, 13, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 224: return by_op<U, 14, -1, LPOL, false, WB>(op, a, num_cus, s);
    case 240: return by_op<U, 15, -1, LPOL, false, WB>(op, a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_np(int op, int variant, const GroupStreamArgs &b, uint32_t num_cus, hipStream_t stream) {
  switch (variant & ~4) {
    // AUTO's variants (tcpck_api.hip run_fixed_impl: FILL of 48-240 B)
    case 0: return by_len_np<4>(op, b, num_cus, stream);
    case 0x80: return by_len_np<4, 0>(op, b, num_cus, stream);
    case 0x401: return op == kFill ? by_len_np<8, 2, 2>(op, b, num_cus, stream) : hipErrorInvalidValue;
#ifdef TCPCK_PROBE
    case 1: return by_len_np<8>(op, b, num_cus, stream);
    case 2: return by_len_np<2>(op, b, num_cus, stream);
    case 0x400: return op == kFill ? by_len_np<4, 2, 2>(op, b, num_cus, stream) : hipErrorInvalidValue;
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool gstream_applies(const uint8_t *arena, uint64_t stride, uint32_t len) {
  const bool pow2 = (len & (len - 1)) == 0;
  return stride == len && len >= 32 && len <= 1024 && (len & 15u) == 0 && (pow2 || len <= 240) &&
         (reinterpret_cast<uintptr_t>(arena) & 15u) == 0;
}

hipError_t launch_gstream(int op, int variant, const GroupStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (!gstream_applies(a.arena, a.len, a.len)) return hipErrorInvalidValue;
  if (a.count == 0) return hipSuccess;
  GroupStreamArgs b = a;
  b.order = (variant & 4) ? dev::kOrderDefault : 4u;  // XCD-chunked order, groups of 16 blocks
  if (variant & ~0xFF7) return hipErrorInvalidValue;
  if (a.len & (a.len - 1)) return launch_np(op, variant, b, num_cus, stream);
  // AUTO's variants (tcpck_api.hip run_fixed_impl): 0 (FILL of 512 B-1 KiB),
  // kGstreamDefaultLoads (FILL <= 256 B), kGstreamWriteBack (FILL <= 128 B)
  switch (variant & ~4) {
    case 0: return by_len<4>(op, b, num_cus, stream);
    case kGstreamDefaultLoads: return by_len<4, -1, 0>(op, b, num_cus, stream);  // default-policy loads
    case kGstreamWriteBack:  // every chunk written back whole, nt stores, U8
      return op == kFill ? by_len<8, -1, 2, false, 2>(op, b, num_cus, stream) : hipErrorInvalidValue;
    default: break;
  }
#ifdef TCPCK_PROBE
  // measurement-only variants (libtcpck_probe.so)
  if (variant & 0xC00) {  // FILL: whole-chunk write-back (bit 10: nt stores, bit 11: default policy)
    if (op != kFill) return hipErrorInvalidValue;
    switch (variant & 0xDF3) {
      case 0x400: return by_len<4, -1, 2, false, 2>(op, b, num_cus, stream);
      case 0x800: return by_len<4, -1, 2, false, 0>(op, b, num_cus, stream);
      case 0xC00: return by_len<4, -1, 2, false, 16>(op, b, num_cus, stream);  // sc1
      case 0x801: return by_len<8, -1, 2, false, 18>(op, b, num_cus, stream);  // sc1 nt (write-through)
      case 0xC01: return by_len<8, -1, 2, false, 19>(op, b, num_cus, stream);  // sc0 sc1 nt
      default: return hipErrorInvalidValue;
    }
  }
  if (variant & 0x200) {  // FILL field lines with the default load policy
    switch (variant & 0x1F3) {
      case 0: return by_len<4, -1, 2, true>(op, b, num_cus, stream);
      case 1: return by_len<8, -1, 2, true>(op, b, num_cus, stream);
      case 2: return by_len<2, -1, 2, true>(op, b, num_cus, stream);
      default: return hipErrorInvalidValue;
    }
  }
  if (variant & 0x1F0) {  // tuning: U4 with the store / load policy (bits 4-8)
    switch (variant & 0x1F3) {
      case 0x10: return by_len<4, 0>(op, b, num_cus, stream);    // buffer stores, default policy
      case 0x20: return by_len<4, 2>(op, b, num_cus, stream);    // buffer stores, nt
      case 0x40: return by_len<4, 16>(op, b, num_cus, stream);   // buffer stores, sc1
      case 0x100: return by_len<4, 0, 0>(op, b, num_cus, stream);   // both
      case 0x22: return by_len<2, 2>(op, b, num_cus, stream);    // U2, nt buffer stores
      default: return hipErrorInvalidValue;
    }
  }
  switch (variant & 3) {
    case 1: return by_len<8>(op, b, num_cus, stream);
    case 2: return by_len<2>(op, b, num_cus, stream);
    default: break;
  }
#endif
  return hipErrorInvalidValue;
}

}  // namespace tcpck
