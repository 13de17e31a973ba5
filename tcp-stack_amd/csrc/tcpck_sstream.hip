// tcpck_sstream.hip -- slotted layouts: images anywhere in the arena (fixed
// slots with large gaps, variable-length images in fixed receive slots, any
// offset list), streamed as one COMPACTED run per wave.  CHECKSUM, VERIFY, FILL.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  The receive arena this serves
// is the batched form of NetworkService::Run's recvfrom buffer
// (src/network-service.cc:39,49-56) feeding ReceivePacket's verify
// (include/socket-manager.h:182): datagrams land in fixed slots, each image
// shorter than its slot.
//
// The run's images are read as one stream with the gaps left out: image i
// (run-relative) owns n_i = chunks of 16 B from its 16-B aligned start to its
// rounded-up end (at least 1), at compacted chunks [C_i, C_i + n_i), C the
// prefix sum of n.  Lane l of step t loads compacted chunk q = 64 t + l from
// the arena address of image i(q): d_i + 16 q, d_i = (16-B start of image i) -
// 16 C_i.  In compacted byte coordinates image i is [16 C_i + h_i, + len_i)
// (h_i its offset inside its first chunk), and the bytes between two images
// (the rest of the previous image's last chunk, the start of this one's
// first chunk) form a virtual gap image.  So the compacted run is a packed
// sequence of 2 n virtual images -- gap i ending at 16 C_i + h_i, image i at
// + len_i -- and every image sum is a prefix difference P(end) - P(start),
// resolved per step from an LDS prefix table exactly as tcpck_vvstream.hip's
// gapped mode does; only the odd (image) differences are stored.  Lines that
// lie wholly in a gap are never read.
//
//   * fixed slots (stride % 16 == 0): n and h are the same for every image,
//     i(q) = q / n by a multiply-high with a launcher-computed magic number,
//     the ends are arithmetic -- no descriptors at all;
//   * variable (offsets + lengths): runs of <= 128 images, so every descriptor
//     of the run is read once, 2 per lane, before the stream: C and d per
//     image and the 2 n virtual ends go to per-wave LDS tables.  The step's
//     chunk -> image map: the images that start inside the step post a flag at
//     their first chunk, and lane l's image is the run's current image + the
//     number of flags at or below l (ballot + mbcnt) -- one LDS write, one
//     read and a table lookup per step, done when the step's loads are issued
//     (U steps ahead of its sums);
//   * images need not be in order or apart: an image that starts before the
//     run's first image, or a run whose compacted bytes or buffer range pass
//     2^31, is recomputed image by image (exact, slow);
//   * kFill zeroes each field (compacted 16 C_i + h_i + 28) in the stream and
//     stores the result at the image's arena address (d_i + 16 C_i + h_i +
//     28); images < 30 B send the run to the per-image pass, which skips
//     them (the C ABI rejects them).
//   * HDR (kVerify, tcpck_batch_receive with a header array): the run's
//     headers in host order (TcpHeaderN2H, include/socket-manager.h:184;
//     tcp-header.h:208-221) into the dense array.  HDR >= 2 (AUTO): from the
//     stream's own registers -- an image that starts on a 16-B boundary has
//     its 32 header bytes in compacted chunks C_i and C_i + 1, so the two lanes
//     holding them permute their dwords and store 16 B each at hdr + 32 k
//     (+ 16) as the step is consumed: the header bytes are read once, by the
//     stream (3: write-through sc0 sc1 nt stores).  A run with a misaligned or < 32-B image (or a
//     misaligned array) and HDR 1 instead convert after the verdicts, one
//     image per lane, re-reading the header lines (KEEPL: the stream read
//     with the default cache policy so they are still in L2).
#include <algorithm>
#include <type_traits>

#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

constexpr uint32_t kMaxRun = 128;             // images per run, variable layouts
constexpr int kPer = kMaxRun / 64;            // descriptors per lane
constexpr uint32_t kOrderScatter = 0xFDu;     // block order: multiplicative scatter
constexpr uint32_t kEnds = 2 * kMaxRun + 64;  // virtual ends (gap, image) + 64 read past the run
// results staged in LDS and stored 64 at a time: a store inside the stream
// loop counts in vmcnt beside the ring's loads, so every wait that follows it
// also waits for a younger load.  <= 63 pending + <= 65 ends per step.
constexpr uint32_t kResRing = 128;
// HDR >= 2: header records staged the same way when every image of the run
// is >= 64 B (>= 4 chunks: <= 17 images have header chunks in a step), 8
// images (256 B) per flush: <= 7 complete + 1 partial pending + 17 < 32.
// Runs with shorter images store each record as its chunk passes.
constexpr uint32_t kHdrRing = 32;
constexpr uint32_t kHdrFlush = 8;
constexpr uint32_t kHdrStageMin = 64;

struct SSArgs {
  uint8_t *arena;
  const uint64_t *offsets;  // variable layouts
  const uint32_t *lengths;
  uint64_t base;
  uint64_t count;
  void *out;                // u16 (CHECKSUM, FILL; may be null for FILL) or u8 (VERIFY)
  uint64_t per_wave, rem;   // equal-count split: count = per_wave * waves + rem
  uint32_t stride;          // fixed slots: image k at k * stride, stride % 16 == 0
  uint32_t len;
  uint32_t nchunk;          // fixed: 16-B chunks per image (the same for all: stride % 16 == 0)
  uint32_t lead;            // fixed: offset of every image inside its first chunk
  uint32_t magic, shift;    // fixed: q / nchunk == mulhi(q, magic) >> shift (magic 0: q >> shift)
  uint32_t order;           // block order (dev::ordered_block)
  int mode;                 // kRef or kRfc1071
  uint8_t *hdr;             // HDR: host-order header k at hdr + 32 k
  uint32_t defer_field;     // kFill: results to out only, the fields left for launch_patch_fields
};

__device__ __forceinline__ u32x4 zero_word(u32x4 w, uint32_t wi) {
  const uint32_t keep = (wi & 1u) ? 0x0000FFFFu : 0xFFFF0000u;
  const uint32_t di = wi >> 1;
  w.x &= di == 0 ? keep : 0xFFFFFFFFu;
  w.y &= di == 1 ? keep : 0xFFFFFFFFu;
  w.z &= di == 2 ? keep : 0xFFFFFFFFu;
  w.w &= di == 3 ? keep : 0xFFFFFFFFu;
  return w;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = max(x, static_cast<uint32_t>(__shfl_xor(static_cast<int>(x), m, 64)));
  return x;
}

// MODE kRfc1071: exact u32 prefix tables (as tcpck_vvstream.hip), the
// differences folded
template <int U, int OP, bool FIXED, int MODE = kRef, int HDR = 0, bool KEEPL = false>
__global__ void __launch_bounds__(kBlock) sstream_kernel(SSArgs a) {
  __shared__ uint32_t s_end[kWavesPerBlock][FIXED ? 1 : kEnds];         // virtual ends, compacted bytes
  __shared__ uint32_t s_c[kWavesPerBlock][FIXED ? 1 : kMaxRun + 64];    // first compacted chunk, ~0 past the run
  __shared__ uint32_t s_d[kWavesPerBlock][FIXED ? 1 : kMaxRun];         // chunk q of image i at d_i + 16 q
  __shared__ uint32_t s_flag[kWavesPerBlock][FIXED ? 1 : 64];           // images starting at chunk q0 + l
  __shared__ __attribute__((aligned(16))) uint32_t s_pre[kWavesPerBlock][MODE == kRef ? 256 : 512];  // the step's prefix table
  __shared__ uint32_t s_fld[kWavesPerBlock][OP == kFill ? 64 : 1];      // kFill: field word + 1 per chunk
  __shared__ uint16_t s_res[kWavesPerBlock][kResRing];                  // finished checksums awaiting their flush
  __shared__ u32x4 s_hdr[kWavesPerBlock][HDR >= 2 ? 2 * kHdrRing : 1];  // HDR >= 2: host-order header halves
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  // kOrderScatter: block b takes run group (b P) mod nb, P prime > nb -- the
  // runs in flight at any time spread over the whole batch (tuning)
  const uint32_t bid = a.order == kOrderScatter
                           ? static_cast<uint32_t>((uint64_t{blockIdx.x} * 2654435761ull) % gridDim.x)
                           : dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock + wv;
  uint64_t kb, ke;
  dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  if (kb >= ke) return;
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  uint8_t *const arena = a.arena;

  auto store = [&](uint64_t k, uint32_t sum, uint64_t start) {
    const uint16_t c = dev::finish<MODE>(sum);  // tcp-header.h:262 (REF)
    if constexpr (OP == kVerify) {
      static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
    } else {
      if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
      if (OP == kFill) *reinterpret_cast<uint16_t *>(arena + start + 28) = c;  // raw, as the reference
    }
  };

  // ---- the run's base, its compacted size and the descriptor tables --------
  bool bad = false;
  uint64_t B;        // run base (relative to arena; arena + B is 16-B aligned)
  uint32_t T = 0;    // compacted chunks of the run
  uint32_t R = 0;    // buffer range from B (bytes, whole chunks)
  bool al4;          // every virtual end 4-B aligned: u32 prefix table
  bool hs = false;   // HDR >= 2: every header in its image's first two chunks (the stream emits them)
  bool hst = false;  // HDR >= 2: and every image >= kHdrStageMin (the records staged in LDS)
  const uint32_t S = a.stride;
  const uint32_t L = FIXED ? a.len : 0u;
  const uint32_t n16 = FIXED ? a.nchunk << 4 : 0u;  // fixed: compacted bytes per image
  const uint32_t h = FIXED ? a.lead : 0u;
  if constexpr (FIXED) {
    B = dev::align16_rel(arena, kb * S);
    T = nimg * a.nchunk;  // the launcher keeps runs below 2^27 chunks and 2^31 bytes
    R = ((nimg - 1) * S + h + L + 15) & ~15u;
    al4 = ((h | L) & 3u) == 0;
    if (OP == kFill) bad = L < 30;
    hs = h == 0 && L >= 32;
    hst = L >= kHdrStageMin;
  } else {
    uint64_t o[kPer];
    uint32_t l[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {  // image kPer lane + i
      const uint32_t j = kPer * lane + i;
      o[i] = j < nimg ? a.offsets[kb + j] - a.base : 0;
      l[i] = j < nimg ? a.lengths[kb + j] : 0u;
    }
    B = dev::align16_rel(arena, dev::read_lane64(o[0], 0));
    uint32_t n[kPer], hh[kPer], r16[kPer], hi = 0;
    bool ok = true, odd = false, shrt = false, hmis = false, hsmall = false;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t j = kPer * lane + i;
      const uint64_t r = o[i] - B;  // from the run base; an image before it wraps high
      const bool in = j < nimg;
      // RFC 1071: the u32 prefix differences are exact only for images below
      // 128 KiB (2^16 words of <= 0xFFFF); a longer image (an understated
      // max_len hint, or the kernel named explicitly) sends the run to the
      // exact per-image pass
      ok = ok && (!in || (r < (uint64_t{1} << 30) && l[i] <= (1u << 23) &&
                          (MODE == kRef || l[i] < (1u << 17))));
      const uint32_t rr = static_cast<uint32_t>(r);
      hh[i] = in ? rr & 15u : 0u;
      r16[i] = rr & ~15u;
      n[i] = in ? max((hh[i] + l[i] + 15u) >> 4, 1u) : 0u;
      hi = in ? max(hi, rr + l[i]) : hi;
      odd = odd || (in && ((hh[i] | l[i]) & 3u) != 0);
      shrt = shrt || (in && l[i] < 30);
      hmis = hmis || (in && (hh[i] != 0 || l[i] < 32));  // HDR >= 2: header not in chunks C_i, C_i + 1
      hsmall = hsmall || (in && l[i] < kHdrStageMin);
    }
    bad = __ballot(!ok) != 0;
    al4 = __ballot(odd) == 0;
    hs = __ballot(hmis) == 0;
    hst = __ballot(hsmall) == 0;
    if (OP == kFill) bad = bad || __ballot(shrt) != 0;
    uint32_t c[kPer];  // exclusive prefix of n inside the lane, then across the wave
    uint32_t lsum = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      c[i] = lsum;
      lsum += n[i];
    }
    const uint32_t incl = dev::wave_inclusive_scan(lsum);  // <= 128 x (2^19 + 1): no wrap
    const uint32_t ex = incl - lsum;
    T = dev::read_lane(incl, 63);
    R = (wave_max(hi) + 15u) & ~15u;
    bad = bad || T >= (1u << 27);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t j = kPer * lane + i;
      const bool in = j < nimg;
      const uint32_t ci = ex + c[i];
      const uint32_t eg = 16u * ci + hh[i];
      s_c[wv][j] = in ? ci : ~0u;
      s_d[wv][j] = r16[i] - 16u * ci;  // u32 wrap: d_i + 16 q lands in image i for its chunks
      s_end[wv][2 * j] = in ? eg : ~0u;
      s_end[wv][2 * j + 1] = in ? eg + l[i] : ~0u;
    }
    s_c[wv][kMaxRun + lane] = ~0u;
    s_end[wv][2 * kMaxRun + lane] = ~0u;
    s_flag[wv][lane] = 0u;
    __builtin_amdgcn_wave_barrier();
  }

  hs = HDR >= 2 && hs && !bad && (reinterpret_cast<uintptr_t>(a.hdr) & 15u) == 0;
  hst = hs && hst;
  if (!bad) {
    const uint32_t span = T << 4;  // compacted bytes; every end <= span
    const uint32_t nsteps = (T + 63) >> 6;
    const uint32_t nv = 2 * nimg;
    const auto rsrc = dev::make_rsrc(arena + B, R);
    const uint16_t *pre16 = reinterpret_cast<const uint16_t *>(s_pre[wv]);
    u32x4 *pre4 = reinterpret_cast<u32x4 *>(s_pre[wv]);
    uint32_t *fld = s_fld[wv];
    if constexpr (OP == kFill) {
      fld[lane] = 0;
      __builtin_amdgcn_wave_barrier();
    }

    // chunk -> arena offset (from B) of the lane's chunk of step t; steps are
    // mapped in order, U ahead of their sums
    uint32_t il = 0;  // variable: the image holding the first chunk of the next step mapped
    // HDR >= 2: the step's header chunks -- (run image << 1) | (0: bytes 0-15,
    // 1: bytes 16-31) of the lane's chunk, ~0 for any other chunk
    uint32_t hk_next = ~0u;
    uint32_t hf_prev = 0;  // variable: the previous step's lane 63 held a first chunk
    auto map_step = [&](uint32_t t) -> uint32_t {
      const uint32_t q0 = t << 6;
      const uint32_t q = q0 + lane;
      if constexpr (FIXED) {
        const uint32_t i = a.magic ? (__umulhi(q, a.magic) >> a.shift) : (q >> a.shift);
        const uint32_t c = q - i * a.nchunk;
        if constexpr (HDR >= 2 || HDR < 0) hk_next = (q < T && c < 2u) ? (i << 1) | c : ~0u;
        return i * S + (c << 4);
      } else {
        const uint32_t cj = s_c[wv][il + lane];  // image il + lane starts at chunk cj
        const uint32_t p = cj - q0;              // il itself may start before q0: wraps high
        if (p < 64u) s_flag[wv][p] = 1u;
        __builtin_amdgcn_wave_barrier();
        const uint32_t f = s_flag[wv][lane];
        s_flag[wv][lane] = 0u;
        const uint64_t M = __ballot(f != 0u);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(M >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(M), 0u));
        // flags at or below l, less il's own flag when il starts at q0
        const uint32_t idx = il + below + f - static_cast<uint32_t>(M & 1u);
        const uint32_t d = s_d[wv][idx];
        if constexpr (HDR >= 2 || HDR < 0) {
          // first chunk: the lane's own flag; second: the flag one lane down
          // (lane 0: the previous step's lane 63) -- every image here has >= 2 chunks
          const uint32_t second = lane ? static_cast<uint32_t>(M >> (lane - 1)) & 1u : hf_prev;
          hk_next = f ? idx << 1 : (second ? (idx << 1) | 1u : ~0u);
          hf_prev = static_cast<uint32_t>(M >> 63);
        }
        // the image holding chunk q0 + 64: one that starts there, else lane 63's
        const uint64_t b64 = __ballot(p == 64u);
        const uint32_t i63 = dev::read_lane(idx, 63);
        if (b64) {
          il += static_cast<uint32_t>(__builtin_ctzll(b64));
        } else if (i63 - il == 63u) {
          il = s_c[wv][il + 64] == q0 + 64 ? il + 64 : i63;
        } else {
          il = i63;
        }
        return d + (q << 4);
      }
    };
    auto load_step = [&](uint32_t t) -> u32x4 {
      if constexpr (HDR < 0) {
        // probe (HDR -1): each image's first two chunks read with the default
        // policy, the rest nt -- the header lines left cached for a header pass
        const uint32_t off = map_step(t);
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        if (hk_next != ~0u) {
          const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(off), 0, 0);
          return u32x4{v.x, v.y, v.z, v.w};
        }
        return dev::load16_buf_nt(rsrc, off, 0);
      } else if constexpr (KEEPL) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(map_step(t)), 0, 0);
        return u32x4{v.x, v.y, v.z, v.w};
      } else {
        return dev::load16_buf_nt(rsrc, map_step(t), 0);
      }
    };
    // arena offset (from B) of image i's checksum field
    auto field_at = [&](uint32_t i, uint32_t start) -> uint32_t {
      if constexpr (FIXED)
        return i * S + h + 28;
      else
        return s_d[wv][i] + start + 28;  // start = 16 C_i + h_i
    };
    // virtual end v (0 .. 2 nimg - 1), compacted bytes
    auto end_of = [&](uint32_t v) -> uint32_t {
      if constexpr (FIXED)
        return h + (v >> 1) * n16 + (v & 1u) * L;
      else
        return s_end[wv][v];
    };
    auto ends_at = [&](uint32_t jn0) -> uint32_t {  // end of virtual jn0 + lane, ~0 past the run
      if constexpr (FIXED) {
        const uint32_t v = jn0 + lane;
        return v < nv ? end_of(v) : ~0u;
      } else {
        return s_end[wv][jn0 + lane];  // jn0 <= 2 nimg: inside the table
      }
    };

    u32x4 ring[U];
    uint32_t hring[U];  // HDR >= 2: header keys of the ring's chunks
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ring[u] = load_step(static_cast<uint32_t>(u));
      hring[u] = hk_next;
    }

    uint32_t carry = 0, p_last = 0, jn = 0, fj = 0;
    uint32_t fl = 0;  // results stored: run images [0, fl)
    auto flush = [&](uint32_t n) {  // the staged results of run images fl .. fl + n - 1
      __builtin_amdgcn_wave_barrier();
      if (lane < n) {
        const uint16_t c = s_res[wv][(fl + lane) & (kResRing - 1)];
        if constexpr (OP == kVerify)
          static_cast<uint8_t *>(a.out)[kb + fl + lane] = c == 0 ? 1 : 0;
        else if (a.out)
          static_cast<uint16_t *>(a.out)[kb + fl + lane] = c;
      }
      fl += n;
    };
    uint32_t flh = 0;  // HDR >= 2: header records stored, run images [0, flh)
    auto flush_hdr = [&](uint32_t n) {  // records of run images flh .. flh + n - 1, 16 B per lane
      __builtin_amdgcn_wave_barrier();
      if (lane < 2 * n) {
        const u32x4 o = s_hdr[wv][(2 * flh + lane) & (2 * kHdrRing - 1)];
        u32x4 *dst = reinterpret_cast<u32x4 *>(a.hdr + 32 * (kb + flh) + 16 * lane);
        if constexpr (HDR == 3)  // write-through streaming store (probe)
          asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(o) : "memory");
        else
          *dst = o;
      }
      flh += n;
    };
    uint32_t e_last = 0;  // end of virtual jn - 1 (the stream start for jn = 0)
    auto stream_run = [&](auto al4_tag) {
      constexpr bool AL4 = decltype(al4_tag)::value;
      for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t st = g + u;
          const uint32_t sb = st << 10;
          u32x4 w = ring[u];
          if constexpr (HDR >= 2) {
            if (hs && hring[u] != ~0u) {  // this lane holds header bytes 0-15 or 16-31 of an image
              const uint32_t hk = hring[u];
              // TcpHeaderN2H per dword (dev::n2h_selector): dwords 0/4, 1/5 byte
              // reversed, 2/6 TcpLength/window swapped, 3 the ports, 7 urgent
              const u32x4 o{dev::n2h_dword(w.x, 0x00010203u), dev::n2h_dword(w.y, 0x00010203u),
                            dev::n2h_dword(w.z, 0x02030100u), dev::n2h_dword(w.w, (hk & 1u) ? 0x02030100u : 0x02030001u)};
              if (hst) {
                s_hdr[wv][hk & (2 * kHdrRing - 1)] = o;  // (image << 1 | half) mod the ring
              } else {
                u32x4 *dst = reinterpret_cast<u32x4 *>(a.hdr + 32 * (kb + (hk >> 1)) + 16 * (hk & 1u));
                if constexpr (HDR == 3)  // write-through streaming store (probe)
                  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(o) : "memory");
                else
                  *dst = o;
              }
            }
          }
          if (sb + 1024 > span && sb + (lane << 4) >= span) w = u32x4{0u, 0u, 0u, 0u};  // past the run
          const uint32_t j = jn + lane;
          uint32_t e = ends_at(jn);
          if constexpr (OP == kFill) {  // zero the checksum fields that lie in this step
            const uint32_t i = fj + lane;
            const uint32_t f = i < nimg ? end_of(2 * i) + 28 : ~0u;
            const bool inf = f < sb + 1024;
            const uint64_t bf = __ballot(inf);
            if (bf) {
              if (inf) fld[(f - sb) >> 4] = ((f & 15u) >> 1) + 1u;  // post the word to the chunk's lane
              __builtin_amdgcn_wave_barrier();
              const uint32_t qf = fld[lane];
              if (qf) {
                fld[lane] = 0u;
                w = zero_word(w, qf - 1u);
              }
              __builtin_amdgcn_wave_barrier();
              fj += static_cast<uint32_t>(__popcll(bf));
            }
          }
          const uint32_t q1 = dev::dot2_u16(w.x, 0u);
          const uint32_t q2 = dev::dot2_u16(w.y, q1);
          const uint32_t q3 = dev::dot2_u16(w.z, q2);
          const uint32_t tot = dev::dot2_u16(w.w, q3);
          const uint32_t incl = dev::wave_inclusive_scan(tot);
          bool table = false;
          uint32_t jj = j;
          for (;;) {  // once per step unless it holds more than 64 ends
            const bool inb = e < sb + 1024;
            const uint64_t bal = __ballot(inb);
            if (!bal) break;
            if (!table) {
              const uint32_t p0 = carry + incl - tot;
              const uint32_t b1 = p0 + q1, b2 = p0 + q2, b3 = p0 + q3;
              if constexpr (AL4)
                pre4[lane] = u32x4{p0, b1, b2, b3};
              else if constexpr (MODE == kRfc1071) {
                pre4[2 * lane] = u32x4{p0, p0 + (w.x & 0xFFFFu), b1, b1 + (w.y & 0xFFFFu)};
                pre4[2 * lane + 1] = u32x4{b2, b2 + (w.z & 0xFFFFu), b3, b3 + (w.w & 0xFFFFu)};
              } else
                pre4[lane] = u32x4{__builtin_amdgcn_perm(p0 + w.x, p0, 0x05040100u),
                                   __builtin_amdgcn_perm(b1 + w.y, b1, 0x05040100u),
                                   __builtin_amdgcn_perm(b2 + w.z, b2, 0x05040100u),
                                   __builtin_amdgcn_perm(b3 + w.w, b3, 0x05040100u)};
              __builtin_amdgcn_wave_barrier();
              table = true;
            }
            const uint32_t cnt = static_cast<uint32_t>(__popcll(bal));  // lanes 0..cnt-1 (ends ascend)
            const uint32_t off = min(e - sb, 1022u);
            const uint32_t P = AL4 ? s_pre[wv][off >> 2]
                                   : (MODE == kRfc1071 ? s_pre[wv][off >> 1] : static_cast<uint32_t>(pre16[off >> 1]));
            const uint32_t pprev = static_cast<uint32_t>(
                __builtin_amdgcn_update_dpp(static_cast<int>(p_last), static_cast<int>(P), 0x138, 0xF, 0xF, false));
            // the previous virtual end (= this image's start), read by DPP with
            // every lane active: a DPP source lane masked off by a branch reads
            // as the old value
            uint32_t el = 0;
            if constexpr (OP == kFill)
              el = static_cast<uint32_t>(
                  __builtin_amdgcn_update_dpp(static_cast<int>(e_last), static_cast<int>(e), 0x138, 0xF, 0xF, false));
            if (inb && (jj & 1u)) {  // an image end (odd virtual index)
              const uint32_t i = jj >> 1;
              const uint16_t cs = dev::finish<MODE>(P - pprev);  // tcp-header.h:262 (REF)
              s_res[wv][i & (kResRing - 1)] = cs;
              if constexpr (OP == kFill)
                if (!a.defer_field) dev::store16_field(rsrc, field_at(i, lane == 0 ? e_last : el), cs);  // raw, as the reference
            }
            p_last = dev::read_lane(P, cnt - 1);
            e_last = dev::read_lane(e, cnt - 1);
            jn += cnt;
            if (cnt < 64) break;
            jj = jn + lane;
            e = ends_at(jn);
          }
          __builtin_amdgcn_wave_barrier();  // the next step rewrites the table
          while ((jn >> 1) - fl >= 64u) flush(64u);  // wave-uniform
          if constexpr (HDR >= 2)
            if (hst)
              while ((jn >> 1) - flh >= kHdrFlush) flush_hdr(kHdrFlush);
          carry += dev::read_lane(incl, 63);
          ring[u] = load_step(st + U);
          hring[u] = hk_next;
        }
      }
    };
    if (al4)
      stream_run(std::true_type{});
    else
      stream_run(std::false_type{});
    while (fl < (jn >> 1)) flush(min((jn >> 1) - fl, 64u));
    if constexpr (HDR >= 2)  // every header chunk has passed: the rest of the records
      if (hst)
        while (flh < nimg) flush_hdr(min(nimg - flh, kHdrFlush));
    if (jn < nv) {  // ends exactly at the last step's end (= span): the first gets the rest
      const uint32_t rem = nv - jn;
      for (uint32_t i = lane; i < rem; i += 64) {
        const uint32_t v = jn + i;
        if (v & 1u) {
          const uint32_t sum = i == 0 ? carry - p_last : 0u;
          if constexpr (OP == kFill) {
            const uint16_t cs = dev::finish<MODE>(sum);
            if (a.out) static_cast<uint16_t *>(a.out)[kb + (v >> 1)] = cs;
            if (!a.defer_field) dev::store16_field(rsrc, field_at(v >> 1, i == 0 ? e_last : span), cs);
          } else {
            store(kb + (v >> 1), sum, 0);
          }
        }
      }
    }
  }
  if (bad) {  // wave-uniform: a layout the compacted walk does not take -> exact per-image pass
    for (uint64_t k = kb; k < ke; ++k) {
      const uint64_t start = FIXED ? k * S : a.offsets[k] - a.base;
      const uint32_t len = FIXED ? L : a.lengths[k];
      if (OP == kFill && len < 30) continue;  // precondition of kFill (the C ABI rejects these)
      const uint32_t sum = dev::wave_image_sum<2, MODE>(arena, start, len, OP == kFill);
      if (lane == 0) store(k, sum, start);
    }
  }
  if (HDR == 1 || (HDR >= 2 && !hs)) {
    // the run's headers in host order, image kb + i by lane i (mod 64): 32-B
    // records, consecutive lanes consecutive records -- whole lines out
    for (uint32_t i = lane; i < nimg; i += 64) {
      const uint64_t k = kb + i;
      const uint8_t *p = arena + (FIXED ? k * S : a.offsets[k] - a.base);
      uint32_t hd[8];
      const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
      if ((pa & 15u) == 0) {
        const u32x4 x = reinterpret_cast<const u32x4 *>(p)[0], y = reinterpret_cast<const u32x4 *>(p)[1];
        hd[0] = x.x, hd[1] = x.y, hd[2] = x.z, hd[3] = x.w, hd[4] = y.x, hd[5] = y.y, hd[6] = y.z, hd[7] = y.w;
      } else if ((pa & 3u) == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) hd[j] = reinterpret_cast<const uint32_t *>(p)[j];
      } else {  // images are 2-B aligned
        const uint16_t *q = reinterpret_cast<const uint16_t *>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) hd[j] = static_cast<uint32_t>(q[2 * j]) | (static_cast<uint32_t>(q[2 * j + 1]) << 16);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) hd[j] = dev::n2h_dword(hd[j], dev::n2h_selector(static_cast<uint32_t>(j)));
      uint8_t *o = a.hdr + 32 * k;
      if ((reinterpret_cast<uintptr_t>(o) & 15u) == 0) {
        reinterpret_cast<u32x4 *>(o)[0] = u32x4{hd[0], hd[1], hd[2], hd[3]};
        reinterpret_cast<u32x4 *>(o)[1] = u32x4{hd[4], hd[5], hd[6], hd[7]};
      } else {  // the API requires a 4-B aligned array
#pragma unroll
        for (int j = 0; j < 8; ++j) reinterpret_cast<uint32_t *>(o)[j] = hd[j];
      }
    }
  }
}

template <int U, int OP, bool FIXED, int MODE = kRef, int HDR = 0, bool KEEPL = false>
hipError_t launch_one(SSArgs a, uint32_t oversub, uint64_t min_waves, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(sstream_kernel<U, OP, FIXED, MODE, HDR, KEEPL>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  uint64_t blocks = resident * oversub;
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;  // >= 1 image per wave
  const uint64_t least = (min_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks < least) blocks = least;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
  a.per_wave = a.count / (blocks * kWavesPerBlock);
  a.rem = a.count % (blocks * kWavesPerBlock);
  hipLaunchKernelGGL((sstream_kernel<U, OP, FIXED, MODE, HDR, KEEPL>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                     stream, a);
  return hipGetLastError();
}

template <int U, bool FIXED>
hipError_t dispatch(int op, const SSArgs &a, uint32_t m, uint64_t min_waves, uint32_t num_cus, hipStream_t s,
                    bool keepl, int hdr_mode) {
#ifdef TCPCK_PROBE
  if (!a.hdr && keepl && op == kVerify && a.mode == kRef)  // + 16 without a header array: HDR -1
    return launch_one<U, kVerify, FIXED, kRef, -1>(a, m, min_waves, num_cus, s);
#endif
  if (a.hdr) {  // VERIFY + the run's headers into the array (tcpck_batch_receive)
    if (op != kVerify) return hipErrorInvalidValue;
    if (hdr_mode == 2 && !keepl)  // AUTO: the headers from the stream's registers
      return a.mode != kRef ? launch_one<U, kVerify, FIXED, kRfc1071, 2>(a, m, min_waves, num_cus, s)
                            : launch_one<U, kVerify, FIXED, kRef, 2>(a, m, min_waves, num_cus, s);
#ifdef TCPCK_PROBE
    if (a.mode != kRef)
      return keepl ? launch_one<U, kVerify, FIXED, kRfc1071, 1, true>(a, m, min_waves, num_cus, s)
                   : launch_one<U, kVerify, FIXED, kRfc1071, 1, false>(a, m, min_waves, num_cus, s);
    if (hdr_mode == 3) return launch_one<U, kVerify, FIXED, kRef, 3>(a, m, min_waves, num_cus, s);
    return keepl ? launch_one<U, kVerify, FIXED, kRef, 1, true>(a, m, min_waves, num_cus, s)
                 : launch_one<U, kVerify, FIXED, kRef, 1, false>(a, m, min_waves, num_cus, s);
#else
    return hipErrorInvalidValue;
#endif
  }
  if (a.mode != kRef) {
    switch (op) {
      case kChecksum: return launch_one<U, kChecksum, FIXED, kRfc1071>(a, m, min_waves, num_cus, s);
      case kVerify: return launch_one<U, kVerify, FIXED, kRfc1071>(a, m, min_waves, num_cus, s);
      case kFill: return launch_one<U, kFill, FIXED, kRfc1071>(a, m, min_waves, num_cus, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum, FIXED>(a, m, min_waves, num_cus, s);
    case kVerify: return launch_one<U, kVerify, FIXED>(a, m, min_waves, num_cus, s);
    case kFill: return launch_one<U, kFill, FIXED>(a, m, min_waves, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool sstream_fixed_applies(uint64_t stride, uint32_t len) {
  return stride >= len && len >= 2 && (stride & 15u) == 0 && stride <= (1u << 24);
}

hipError_t launch_sstream(int op, int variant, bool fixed, const RunArgs &r, uint32_t num_cus, hipStream_t stream) {
  if (r.count == 0) return hipSuccess;
  SSArgs a{};
  a.arena = r.arena;
  a.offsets = r.offsets;
  a.lengths = r.lengths;
  a.base = r.base;
  a.count = r.count;
  a.out = r.out;
  a.mode = r.mode;
  a.hdr = r.hdr;
  // + 128 (kFill with a results buffer): the results only, the caller runs the field pass
  a.defer_field = (variant & 128) ? 1u : 0u;
  if (a.defer_field && (op != kFill || !r.out)) return hipErrorInvalidValue;
  // + 4: default block order; + 8: scattered (the policy's); else groups of
  // 16 blocks per XCD
  a.order = (variant & 8) ? kOrderScatter : ((variant & 4) ? dev::kOrderDefault : 4u);
  uint64_t bytes = r.total_bytes;
  uint64_t min_waves = (r.count + kMaxRun - 1) / kMaxRun;  // variable: <= kMaxRun images per run
  if (fixed) {
    if (!sstream_fixed_applies(r.stride, r.len)) return hipErrorInvalidValue;
    a.stride = static_cast<uint32_t>(r.stride);
    a.len = r.len;
    a.lead = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(r.arena) & 15u);  // the same for every image
    a.nchunk = (a.lead + r.len + 15) >> 4;
    uint32_t sh = 0;
    while ((2u << sh) <= a.nchunk) ++sh;  // floor(log2 nchunk)
    a.shift = sh;
    a.magic = (a.nchunk & (a.nchunk - 1)) == 0
                  ? 0u
                  : static_cast<uint32_t>(((uint64_t{1} << (32 + sh)) + a.nchunk - 1) / a.nchunk);
    bytes = r.count * r.len;
    // runs below 2^31 arena bytes and 2^27 compacted chunks (u32 run arithmetic)
    const uint64_t per = std::min<uint64_t>((uint64_t{1} << 30) / r.stride, (uint64_t{1} << 26) / a.nchunk);
    min_waves = (r.count + per - 1) / std::max<uint64_t>(per, 1);
  }
  if (bytes == 0) bytes = r.count * 1024;
  // grid: M x the resident grid, M a power of two, blocks in the scattered
  // order (scripts/ss_sweep.py, scripts/sparse_probe.py; profiles/r02/
  // ss_sweep3_scatter.log, ss_sweep4_run128.log, sparse_probe2_orders.log).
  // Sparse reads are sensitive to which addresses are in flight together: with
  // the XCD-chunked order the same kernel ran 1492-B images in 4-KiB slots at
  // 59-74 % and 2-KiB images in 4-KiB slots at 64-80 % depending on M, while the
  // scattered order (the runs in flight spread over the whole batch) holds
  // 78-88 % at every density >= 1/4 and block size tried.  Offset lists pay a
  // descriptor round trip before a run's first data load, so their runs stay
  // longer: >= 16 KiB of image bytes (var 96/608/1492 in 2048-B slots 72.0 %
  // at M = 4 against 57 % at M = 16), fixed slots >= 8 KiB (1492 in 2048-B
  // slots 83.0 %, in 4-KiB slots 82.0 %, 9000 in 16 KiB 86.4 % at M = 16).
  // U4 throughout (U8 costs occupancy: 90 VGPRs against 58).
  if (!(variant & 12)) a.order = kOrderScatter;
  const uint32_t m = dev::oversub_for(r.oversub, bytes, static_cast<uint64_t>(num_cus) * 32, 1024,
                                      fixed ? 8u << 10 : 16u << 10);
  const int u = variant & 3;  // 0: policy, 1: U4, 2: U8
  const bool u8 = u == 2;
#ifndef TCPCK_PROBE
  // the product library runs the policy (0) and its RECEIVE form (+ 32) only
  if ((variant & ~(32 | 128)) != 0) return hipErrorInvalidValue;
#endif
  const bool keepl = (variant & 16) != 0;  // HDR 1: the stream read with the default cache policy
  // HDR: + 32 the headers from the stream's registers (kSstreamHdrStream), + 64 with write-through stores
  const int hdr_mode = (variant & 32) ? ((variant & 64) ? 3 : 2) : 1;
#ifdef TCPCK_PROBE
  if (u8) return fixed ? dispatch<8, true>(op, a, m, min_waves, num_cus, stream, keepl, hdr_mode)
                       : dispatch<8, false>(op, a, m, min_waves, num_cus, stream, keepl, hdr_mode);
#endif
  if (u8) return hipErrorInvalidValue;
  return fixed ? dispatch<4, true>(op, a, m, min_waves, num_cus, stream, keepl, hdr_mode)
               : dispatch<4, false>(op, a, m, min_waves, num_cus, stream, keepl, hdr_mode);
}

}  // namespace tcpck
