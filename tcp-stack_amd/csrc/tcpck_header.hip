// tcpck_header.hip -- batched header byte-order conversion (in place or into
// a dense header array), and FILL's deferred field stores.
//
// The receive path verifies a packet on its network-order bytes and only then
// converts the header to host order (ReceivePacket, include/socket-manager.h:
// 182-184: CalculateChecksum(*packet) == 0, then TcpHeaderN2H); the send path
// converts before its checksum (TcpHeaderH2N, socket-internal.h:196).  The two
// conversions are the same byte permutation (tcp-header.h:193-221): u32 byte
// swaps of SourceAddress (bytes 0-3), DestinationAddress (4-7), SequenceNumber
// (16-19) and AcknowledgementNumber (20-23); u16 swaps of TcpLength (10-11),
// SourcePort (12-13), DestinationPort (14-15), Window (26-27) and
// UrgentPointer (30-31).  Bytes 8-9 (zero, PTCL), 24-25 (offset, flags) and
// 28-29 (checksum) stay as they are.
//
// Layout: 8 lanes per image, lane j owns header bytes 4j..4j+3, so a wave
// covers 8 images and each image's 32 bytes are one contiguous 8-lane group.
// Images are only 2-B aligned (even offsets), hence two u16 accesses per lane.
// Per image 32 bytes read and at most 28 written; like the ACK rewrite the pass
// is bound by the scattered lines it touches (one or two per image), not by
// streaming bandwidth.  EXTRACT (tcpck_batch_receive with a header array):
// the arena stays as it is and header k goes to out[32k, 32k + 32) instead --
// the writes are dense whole lines, not one partial line per image.
#include <algorithm>

#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;

__device__ __forceinline__ uint16_t bswap16(uint16_t v) { return static_cast<uint16_t>((v >> 8) | (v << 8)); }

template <bool FIXED, bool EXTRACT, bool WT = false>
__global__ void __launch_bounds__(kBlock) header_swap_kernel(HeaderArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t total = a.count * 8;
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; t < total; t += step) {
    const uint64_t k = t >> 3;
    const uint32_t j = static_cast<uint32_t>(t & 7);
    const uint64_t start = FIXED ? k * a.stride : a.offsets[k];
    uint16_t *w = reinterpret_cast<uint16_t *>(a.arena + start) + 2 * j;
    const uint16_t lo = w[0], hi = w[1];
    if constexpr (EXTRACT) {
      // dense output: lane group k writes the 32 B of header k, whole lines
      const uint32_t h = static_cast<uint32_t>(lo) | (static_cast<uint32_t>(hi) << 16);
      const uint32_t v = dev::n2h_dword(h, dev::n2h_selector(j));
      if constexpr (WT) {  // probe: write-through streaming stores
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.out) + t;
        asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(v) : "memory");
      } else {
        reinterpret_cast<uint32_t *>(a.out)[t] = v;
      }
    } else if (j == 0 || j == 1 || j == 4 || j == 5) {
      // j = 0, 1, 4, 5: a u32 field (its two u16 halves trade places, each swapped)
      w[0] = bswap16(hi);
      w[1] = bswap16(lo);
    } else {
      // j = 3: two u16 ports;  j = 2, 6, 7: only the upper u16 is a swapped field
      if (j == 3) w[0] = bswap16(lo);
      w[1] = bswap16(hi);
    }
  }
}

#ifdef TCPCK_PROBE
// Probe: the array form with two lanes per image, each one 16-B buffer load of
// header bytes 16h..16h+15 and one 16-B store (images 16-B aligned, arena
// < 4 GiB; the launcher checks), loads with cache bits LP (0 default, 1 nt,
// 2 sc0 sc1, 3 sc1): how many bytes a 32-B header costs to fetch.
template <bool FIXED, int LP>
__global__ void __launch_bounds__(kBlock) header_wide_kernel(HeaderArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const auto rsrc = dev::make_rsrc(a.arena, 0xFFFFFFF0u);
  constexpr int aux = LP == 0 ? 0 : (LP == 1 ? 2 : (LP == 2 ? 17 : 16));
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; t < a.count * 2; t += step) {
    const uint64_t k = t >> 1;
    const uint32_t h = static_cast<uint32_t>(t & 1);
    const uint64_t start = FIXED ? k * a.stride : a.offsets[k];
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(start + 16 * h), 0, aux);
    const dev::u32x4 o{dev::n2h_dword(v.x, 0x00010203u), dev::n2h_dword(v.y, 0x00010203u),
                       dev::n2h_dword(v.z, 0x02030100u), dev::n2h_dword(v.w, h ? 0x02030100u : 0x02030001u)};
    reinterpret_cast<dev::u32x4 *>(a.out)[t] = o;
  }
}

template <bool FIXED, int LP>
hipError_t launch_wide(const HeaderArgs &a, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(header_wide_kernel<FIXED, LP>);
  uint64_t blocks = (a.count * 2 + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((header_wide_kernel<FIXED, LP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <bool FIXED>
hipError_t wide_by_policy(const HeaderArgs &a, uint32_t num_cus, hipStream_t s) {
  switch ((a.store_bits >> 4) & 3u) {
    case 0: return launch_wide<FIXED, 0>(a, num_cus, s);
    case 1: return launch_wide<FIXED, 1>(a, num_cus, s);
    case 2: return launch_wide<FIXED, 2>(a, num_cus, s);
    default: return launch_wide<FIXED, 3>(a, num_cus, s);
  }
}
#endif

// The array form (tcpck_batch_receive with a header array): two lanes per
// image, lane h converting header bytes 16h..16h+15 -- one 16-B load when the
// image is 16-B aligned (every receive-ring slot), else eight u16 loads -- and
// one 16-B store (four 4-B stores into a 4-B aligned array).  2 us faster than
// eight lanes of u16 accesses on the 1M-datagram ring (29.2 vs 31.1 us; the
// pass fetches the same 128-B line per image either way, whatever the load's
// cache bits: scripts/receive_fused_probe.py --wide, profiles/r03/
// receive_header_wide.log).
//
// ORDER (probe builds, tcpck_probe_receive_ex's ORDER field; 0 = the
// product's): which images a block reads together, i.e. which header lines are
// in flight at once -- 1: XCD-chunked block order (groups of 16 blocks per
// XCD), 2: multiplicative block scatter (the blocks in flight spread over the
// whole batch), 3: each block's 128 images 1/128 of the batch apart.
template <bool FIXED, int ORDER = 0>
__global__ void __launch_bounds__(kBlock) header_extract_kernel(HeaderArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const bool out16 = (reinterpret_cast<uintptr_t>(a.out) & 15u) == 0;
  uint32_t bid = blockIdx.x;
  if constexpr (ORDER == 1) bid = dev::ordered_block(blockIdx.x, gridDim.x, 4u);
  if constexpr (ORDER == 2) bid = static_cast<uint32_t>((uint64_t{blockIdx.x} * 2654435761ull) % gridDim.x);
  const uint64_t n2 = a.count * 2;
  for (uint64_t t = static_cast<uint64_t>(bid) * kBlock + threadIdx.x; t < n2; t += step) {
    uint64_t k = t >> 1;
    const uint32_t h = static_cast<uint32_t>(t & 1);
    if constexpr (ORDER == 3) {
      // t's image as a 128 x (count / 128) transpose: lane pair i of block
      // group g reads image i * (count / 128) + g; the tail stays in order
      const uint64_t rows = a.count >> 7, body = rows << 7;
      if (k < body) k = (k & 127u) * rows + (k >> 7);
    }
    const uint8_t *p = a.arena + (FIXED ? k * a.stride : a.offsets[k]) + 16 * h;
    dev::u32x4 v;
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
      v = *reinterpret_cast<const dev::u32x4 *>(p);
    } else {  // images are 2-B aligned
      const uint16_t *q = reinterpret_cast<const uint16_t *>(p);
      v = dev::u32x4{q[0] | (static_cast<uint32_t>(q[1]) << 16), q[2] | (static_cast<uint32_t>(q[3]) << 16),
                     q[4] | (static_cast<uint32_t>(q[5]) << 16), q[6] | (static_cast<uint32_t>(q[7]) << 16)};
    }
    // dwords 4h..4h+3 of TcpHeaderN2H (dev::n2h_selector): 0/4, 1/5 byte
    // reversed, 2/6 the upper u16 swapped, 3 the two ports, 7 the urgent pointer
    const dev::u32x4 o{dev::n2h_dword(v.x, 0x00010203u), dev::n2h_dword(v.y, 0x00010203u),
                       dev::n2h_dword(v.z, 0x02030100u), dev::n2h_dword(v.w, h ? 0x02030100u : 0x02030001u)};
    const uint64_t r = (k << 1) | h;  // header k's half h (== t in order)
    if (out16) {
      reinterpret_cast<dev::u32x4 *>(a.out)[r] = o;
    } else {
      uint32_t *d = reinterpret_cast<uint32_t *>(a.out) + 4 * r;
      d[0] = o.x, d[1] = o.y, d[2] = o.z, d[3] = o.w;
    }
  }
}

template <bool FIXED, int ORDER = 0>
hipError_t launch_extract(const HeaderArgs &a, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(header_extract_kernel<FIXED, ORDER>);
  uint64_t blocks = (a.count * 2 + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((header_extract_kernel<FIXED, ORDER>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <bool FIXED, bool EXTRACT, bool WT = false>
hipError_t launch_one(const HeaderArgs &a, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(header_swap_kernel<FIXED, EXTRACT, WT>);
  uint64_t blocks = (a.count * 8 + kBlock - 1) / kBlock;
  // grid-stride beyond 8 resident grids (4 loads in flight per lane measured no faster:
  // profiles/r02/receive_probe.log)
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((header_swap_kernel<FIXED, EXTRACT, WT>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, s,
                     a);
  return hipGetLastError();
}

// ---- FILL's field stores after the stream (PatchArgs) ----------------------
//
// One lane per image stores the 2-B checksum into bytes 28-29 as a
// write-through streaming store (global_store_short sc0 sc1 nt): nothing but
// the field is read or written.  The store policy is what matters here
// (scripts/fill_drain_probe.py, profiles/r03/fill_store_policy.log): a plain,
// sc0, sc1 or nt store leaves its line dirty in the memory-side Infinity Cache
// (MALL) and the next read stream pays for the 1M scattered write-backs -- C2's
// stream then ran 244 us instead of 209 us, even with 100 us of idle GPU
// between the passes; with sc1 nt / sc0 sc1 nt the pass writes HBM itself (38
// us for 1M 2-B stores, 44 us for 64-B blocks) and the next stream runs at
// 209 us: AUTO's C2 FILL 280 -> 248 us.
__device__ __forceinline__ void store16_through(uint8_t *p, uint16_t c) {
  const uint32_t v = c;
  asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// UPDATE: sums[k] is image k's CHECKSUM with its field in; the zero-field
// checksum follows from the old field f, c = ~(~C - f) mod 2^16, and goes to
// the field and back to sums[k].  Images < 30 B keep their plain checksum and
// are not written (seg's FILL does the same).
template <bool VAR, bool UPDATE>
__global__ void __launch_bounds__(kBlock) patch_fields_kernel(PatchArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  for (uint64_t kf = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; kf < a.count; kf += step) {
    const uint64_t k = a.reverse ? a.count - 1 - kf : kf;
    uint64_t f;  // the field, relative to arena
    if constexpr (VAR) {
      if (a.lengths[k] < 30) continue;  // no field
      f = a.offsets[k] - a.base + 28;
    } else {
      f = k * a.stride + 28;
    }
    uint16_t c = a.sums[k];
    if constexpr (UPDATE) {
      const uint16_t old = *reinterpret_cast<const uint16_t *>(a.arena + f);
      c = static_cast<uint16_t>(~static_cast<uint16_t>(static_cast<uint16_t>(~c) - old));
      a.sums[k] = c;
    }
    store16_through(a.arena + f, c);  // raw host order, tcp-header.h:177
  }
}

template <bool VAR, bool UPDATE>
hipError_t launch_patch(const PatchArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(patch_fields_kernel<VAR, UPDATE>);
  uint64_t blocks = (a.count + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((patch_fields_kernel<VAR, UPDATE>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream,
                     a);
  return hipGetLastError();
}

#ifdef TCPCK_PROBE
// Timing only (fixed strides, no update): the field pass at other
// granularities and store policies.  GRAN 0: four lanes per image, the field's
// 64-B block read and written back whole (AUTO's form in round 2); 1: one lane,
// the 16-B chunk holding the field; 2: the 2-B field alone (no read); 3: eight
// lanes, the field's 128-B line; 4: two lanes, the field's 32-B block.  BLIND:
// the block written without reading it (zeros around the field: destroys the
// images, timing of whole-block writes only).  BITS: store cache bits sc0 1 |
// nt 2 | sc1 4, -1 a plain C++ store.
template <int BITS>
__device__ __forceinline__ void store_block(dev::u32x4 *p, dev::u32x4 v) {
  if constexpr (BITS < 0) {
    *p = v;
  } else if constexpr (BITS == 0) {
    asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 1) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 4) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 5) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (BITS == 6) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  }
}

template <int G, bool BLIND, int BITS>
__global__ void __launch_bounds__(kBlock) patch_probe_kernel(PatchArgs a) {
  constexpr int LPI = G == 3 ? 8 : (G == 0 ? 4 : (G == 4 ? 2 : 1));  // lanes per image
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t total = a.count * LPI;
  const uint64_t base = reinterpret_cast<uint64_t>(a.arena);
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; t < total; t += step) {
    const uint64_t k = t / LPI;
    const uint32_t j = static_cast<uint32_t>(t % LPI);
    const uint64_t f = k * a.stride + 28;
    const uint16_t c = a.sums[k];
    if constexpr (G == 2) {
      uint16_t *p = reinterpret_cast<uint16_t *>(a.arena + f);
      const uint32_t v = c;
      if constexpr (BITS == 7)
        asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
      else if constexpr (BITS == 6)
        asm volatile("global_store_short %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
      else
        *p = c;
    } else {
      const uint64_t gm = G == 3 ? 127 : (G == 0 ? 63 : (G == 4 ? 31 : 15));
      const uint64_t blk = ((base + f) & ~gm) - base;
      if (G != 1 && (blk < a.lo || blk + gm + 1 > a.hi)) {  // the block would leave the batch
        if (j == 0) *reinterpret_cast<uint16_t *>(a.arena + f) = c;
        continue;
      }
      dev::u32x4 *p = reinterpret_cast<dev::u32x4 *>(a.arena + blk) + j;
      dev::u32x4 v = BLIND ? dev::u32x4{0u, 0u, 0u, 0u} : *p;
      const uint32_t r = static_cast<uint32_t>(f - blk) - 16 * j;
      if (r < 16) {
        const uint32_t sh = 16 * ((r >> 1) & 1);
        const uint32_t di = r >> 2;
        const uint32_t m = ~(0xFFFFu << sh), x = static_cast<uint32_t>(c) << sh;
        v.x = di == 0 ? (v.x & m) | x : v.x;
        v.y = di == 1 ? (v.y & m) | x : v.y;
        v.z = di == 2 ? (v.z & m) | x : v.z;
        v.w = di == 3 ? (v.w & m) | x : v.w;
      }
      store_block<BITS>(p, v);
    }
  }
}

// Timing only: the 2-B write-through field pass with other image -> thread
// maps.  MAP 0: four consecutive images per thread; 1: four per thread, a
// quarter of the batch apart; 2: the resident grid only, grid-stride; 3: each
// 256-thread block writes its 256 images in a stride-8 interleaved order.
template <int MAP>
__global__ void __launch_bounds__(kBlock) patch_map_kernel(PatchArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  auto put = [&](uint64_t k) {
    if (k < a.count) store16_through(a.arena + k * a.stride + 28, a.sums[k]);
  };
  if constexpr (MAP == 0) {
    for (uint64_t t = t0; 4 * t < a.count; t += step)
      for (int i = 0; i < 4; ++i) put(4 * t + i);
  } else if constexpr (MAP == 1) {
    const uint64_t q = (a.count + 3) / 4;
    for (uint64_t t = t0; t < q; t += step)
      for (int i = 0; i < 4; ++i) put(t + i * q);
  } else if constexpr (MAP == 2) {
    for (uint64_t t = t0; t < a.count; t += step) put(t);
  } else {
    for (uint64_t b = static_cast<uint64_t>(blockIdx.x) * kBlock; b < a.count; b += step) {
      const uint32_t x = threadIdx.x;
      put(b + (x & 31u) * 8u + (x >> 5));
    }
  }
}

template <int G, bool BLIND, int BITS>
hipError_t launch_patch_probe(const PatchArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(patch_probe_kernel<G, BLIND, BITS>);
  const uint64_t lpi = G == 3 ? 8 : (G == 0 ? 4 : (G == 4 ? 2 : 1));
  uint64_t blocks = (a.count * lpi + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((patch_probe_kernel<G, BLIND, BITS>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream,
                     a);
  return hipGetLastError();
}

// store_bits = 1 + BITS (0: plain) | GRAN << 4
template <int G, bool BLIND = false>
hipError_t probe_by_bits(const PatchArgs &a, uint32_t num_cus, hipStream_t stream) {
  switch (static_cast<int>(a.store_bits & 15) - 1) {
    case -1: return launch_patch_probe<G, BLIND, -1>(a, num_cus, stream);
    case 0: return launch_patch_probe<G, BLIND, 0>(a, num_cus, stream);
    case 1: return launch_patch_probe<G, BLIND, 1>(a, num_cus, stream);
    case 2: return launch_patch_probe<G, BLIND, 2>(a, num_cus, stream);
    case 3: return launch_patch_probe<G, BLIND, 3>(a, num_cus, stream);
    case 4: return launch_patch_probe<G, BLIND, 4>(a, num_cus, stream);
    case 5: return launch_patch_probe<G, BLIND, 5>(a, num_cus, stream);
    case 6: return launch_patch_probe<G, BLIND, 6>(a, num_cus, stream);
    case 7: return launch_patch_probe<G, BLIND, 7>(a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}
#endif

}  // namespace

hipError_t launch_patch_fields(const PatchArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  if (!a.sums) return hipErrorInvalidValue;
#ifdef TCPCK_PROBE
  if (a.probe_form) {  // timing forms (TCPCK_KERNEL_PATCH param)
    if (a.update || a.offsets) return hipErrorInvalidValue;
    if ((a.store_bits >> 4) >= 4 && (a.store_bits >> 4) < 8) {  // the 2-B write-through pass with other maps
      static const uint32_t per_cu = 8;
      const int map = static_cast<int>(a.store_bits >> 4) - 4;
      uint64_t blocks = (a.count + kBlock - 1) / kBlock;
      if (map == 0 || map == 1) blocks = (blocks + 3) / 4;
      if (map == 2) blocks = std::min<uint64_t>(blocks, static_cast<uint64_t>(per_cu) * num_cus);
      const dim3 g(static_cast<uint32_t>(blocks)), b(kBlock);
      switch (map) {
        case 0: hipLaunchKernelGGL(patch_map_kernel<0>, g, b, 0, stream, a); break;
        case 1: hipLaunchKernelGGL(patch_map_kernel<1>, g, b, 0, stream, a); break;
        case 2: hipLaunchKernelGGL(patch_map_kernel<2>, g, b, 0, stream, a); break;
        case 3: hipLaunchKernelGGL(patch_map_kernel<3>, g, b, 0, stream, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    switch (a.store_bits >> 4) {
      case 0: return a.stride >= 64 ? probe_by_bits<0>(a, num_cus, stream) : hipErrorInvalidValue;
      case 1: return probe_by_bits<1>(a, num_cus, stream);
      case 2: return probe_by_bits<2>(a, num_cus, stream);
      case 3: return a.stride >= 128 ? probe_by_bits<3>(a, num_cus, stream) : hipErrorInvalidValue;
      case 8: return a.stride >= 64 ? probe_by_bits<0, true>(a, num_cus, stream) : hipErrorInvalidValue;
      case 9: return a.stride >= 128 ? probe_by_bits<3, true>(a, num_cus, stream) : hipErrorInvalidValue;
      case 10: return probe_by_bits<1, true>(a, num_cus, stream);
      case 11: return a.stride >= 32 ? probe_by_bits<4, true>(a, num_cus, stream) : hipErrorInvalidValue;
      case 12: return a.stride >= 32 ? probe_by_bits<4>(a, num_cus, stream) : hipErrorInvalidValue;
      default: return hipErrorInvalidValue;
    }
  }
#endif
  if (a.offsets) {
    if (!a.lengths) return hipErrorInvalidValue;
    return a.update ? launch_patch<true, true>(a, num_cus, stream) : launch_patch<true, false>(a, num_cus, stream);
  }
  if (a.stride < 30) return hipErrorInvalidValue;  // every image holds a field
  return a.update ? launch_patch<false, true>(a, num_cus, stream) : launch_patch<false, false>(a, num_cus, stream);
}

hipError_t launch_header_swap(const HeaderArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
#ifdef TCPCK_PROBE
  if (a.out && (a.store_bits & 2)) {  // the wide form: 16-B aligned images and array, arena < 4 GiB
    if ((reinterpret_cast<uintptr_t>(a.arena) & 15u) || (reinterpret_cast<uintptr_t>(a.out) & 15u) ||
        (!a.offsets && (a.stride & 15u)))
      return hipErrorInvalidValue;
    return a.offsets ? wide_by_policy<false>(a, num_cus, stream) : wide_by_policy<true>(a, num_cus, stream);
  }
  if (a.out && (a.store_bits >> 8) & 3u) {  // the array form in another image order
    switch ((a.store_bits >> 8) & 3u) {
      case 1: return a.offsets ? launch_extract<false, 1>(a, num_cus, stream) : launch_extract<true, 1>(a, num_cus, stream);
      case 2: return a.offsets ? launch_extract<false, 2>(a, num_cus, stream) : launch_extract<true, 2>(a, num_cus, stream);
      default: return a.offsets ? launch_extract<false, 3>(a, num_cus, stream) : launch_extract<true, 3>(a, num_cus, stream);
    }
  }
  if (a.out && a.store_bits)
    return a.offsets ? launch_one<false, true, true>(a, num_cus, stream) : launch_one<true, true, true>(a, num_cus, stream);
#endif
  if (a.out) return a.offsets ? launch_extract<false>(a, num_cus, stream) : launch_extract<true>(a, num_cus, stream);
  return a.offsets ? launch_one<false, false>(a, num_cus, stream) : launch_one<true, false>(a, num_cus, stream);
}

#ifdef TCPCK_PROBE
// ---- FILL's field blocks from the side buffer (probe, round 6) --------------
// Four lanes per image: lane c copies bytes [16c, 16c + 16) of image k's block
// from side[64 k] to the block's place with a write-through 16-B store (sc0
// sc1 nt): a whole 64-B block needs no merge read at the memory side, where a
// 2-B store does (profiles/r03/fill_blind.log: blind 64-B blocks 20 us per 1M
// fields after the stream, 2-B stores 41-42 us).  The side buffer holds the
// bytes the stream read, checksum in place, so nothing else changes.
__global__ void __launch_bounds__(kBlock) side_copy_kernel(uint8_t *arena, uint64_t stride, uint64_t count,
                                                           const uint8_t *side, const uint16_t *sums) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  for (uint64_t q = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; q < 4 * count; q += step) {
    const uint64_t k = q >> 2;
    const uint32_t c = static_cast<uint32_t>(q & 3u);
    const uintptr_t f = reinterpret_cast<uintptr_t>(arena) + k * stride + 28;
    const uintptr_t blk = f & ~uintptr_t{63};
    if (blk >= reinterpret_cast<uintptr_t>(arena)) {
      const dev::u32x4 v = dev::load16_nt(side + 64 * k + 16 * c);
      uint8_t *dst = reinterpret_cast<uint8_t *>(blk + 16 * c);
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(v) : "memory");
    } else if (c == ((f & 63u) >> 4)) {  // the block starts before the arena: the field alone
      store16_through(reinterpret_cast<uint8_t *>(f), sums[k]);
    }
  }
}

hipError_t launch_side_copy(uint8_t *arena, uint64_t stride, uint64_t count, const uint8_t *side,
                            const uint16_t *sums, uint32_t num_cus, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  if (stride < 128 || !side || !sums) return hipErrorInvalidValue;
  static const uint32_t per_cu = dev::resident_blocks_per_cu(side_copy_kernel);
  uint64_t blocks = (4 * count + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(side_copy_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, arena, stride,
                     count, side, sums);
  return hipGetLastError();
}
#endif

}  // namespace tcpck
