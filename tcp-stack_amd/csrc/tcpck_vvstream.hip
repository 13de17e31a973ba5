// tcpck_vvstream.hip -- packed batches streamed as one contiguous run of whole
// images per wave, every image end of a 1 KiB step resolved by the lanes in
// parallel from a per-wave prefix table in LDS.  Packed variable layouts (C3)
// and fixed strides (LAYOUT 1: packed, stride == length; LAYOUT 2: stride >
// length, the gaps streamed with the images); CHECKSUM, VERIFY and FILL.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  Packed images make the run one
// flat byte stream and sum(k) = P(end_k) - P(end_{k-1}) (mod 2^16), with P(x)
// the word sum of the run before byte x.
//
//   * run split: equal image counts (the launcher passes count = q W + r, no
//     device division) or, at low oversubscription, byte-balanced (two
//     lockstep 64-ary searches over the offsets);
//   * the run's first U data loads go out before anything else, so the
//     descriptor latency overlaps the stream's;
//   * image ends (variable layouts): 256 lengths at a time, one vector load
//     per lane (4 lengths, prefetched a round ahead), prefix-summed across the
//     wave into a 512-entry LDS ring per wave; fixed packed: end j = lead +
//     (j+1) S; fixed gapped: the run is a packed sequence of 2n virtual
//     images, gap i (ending where image i starts) and image i, end v = lead +
//     (v >> 1) S + (v & 1) L, and only the odd (image) differences are stored;
//   * per step: lane j holds end e(jn + j), read before the step's sums so the
//     LDS latency overlaps them.  If any end falls in the step, every lane
//     writes P at its chunk's 8 word positions as packed u16s (one
//     ds_write_b128: P matters mod 2^16 only; the table is laid out like the
//     step), and the lanes whose end is in the step read the u16 at the end's
//     byte offset: sum(jn + j) = P(j) - P(j - 1), P(j - 1) by DPP wave_shr:1
//     (lane 0: the last P of the batch before, an SGPR).  Any image length
//     works; a step with more than 64 ends loops;
//   * kFill (send path, socket-manager.cc:9-10): the checksum field (bytes
//     28-29 of each image, tcp-header.h:177) is zeroed in the stream -- the
//     lane whose image start + 28 falls in the step posts the word to the
//     chunk's lane through LDS (images >= 30 B: one field per chunk at most)
//     -- and the result is stored to out[k] and into the field;
//   * kFill + BLK (flag 128, images >= 64 B, reference mode, no gaps): each
//     field leaves as its whole 64-B block, written through from the step's
//     own registers (unmasked) with the checksum in place -- a whole-block
//     store needs no merge read at the memory side, a 2-B store does.  The
//     field lane's chunk gets the word; the block's 4 lanes store.  The one
//     image that can cross a step boundary with its field before the
//     boundary has its block staged in LDS (64 B per wave) until its end is
//     resolved.  Blocks reaching outside the batch's bytes take the 2-B store;
//   * a wave whose lengths disagree with the offsets (layout hint wrong)
//     recomputes its images one by one.  kFill checks this before it writes
//     anything into the arena.
#include <type_traits>

#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

constexpr uint32_t kRound = 256;  // ends loaded per round (4 per lane)
constexpr uint32_t kRing = 512;   // LDS ring entries per wave (two rounds)
constexpr uint32_t kMirror = 64;  // slots 0..63 repeated after the ring: a step's 64 reads never wrap

struct VVArgs {
  uint8_t *arena;
  const uint64_t *offsets;  // variable layouts
  const uint32_t *lengths;
  uint64_t base;
  uint64_t count;
  void *out;                // u16 (CHECKSUM, FILL; may be null for FILL) or u8 (VERIFY)
  uint64_t per_wave, rem;   // equal-count split: count = per_wave * waves + rem
  uint32_t stride;          // fixed layouts: image k at k * stride
  uint32_t len;             // fixed layouts: image length (<= stride)
  uint32_t order;           // block order (dev::ordered_block)
  uint32_t keep_first;      // 1: the run's first line read with the default cache policy (L2-kept edge
                            // line); 2 (probe): its whole first step, the policy before round 5
  uint32_t defer_field;     // kFill: results to out only, the fields left for launch_patch_fields
  uint64_t *dbg;            // probe library: 8 x u64 per wave {start, descriptors, first data, end, hw/xcc, images, span, 0}
};

#ifdef TCPCK_PROBE
// s_memrealtime (100 MHz) once `dep` exists: a stamp ordered after the value it names
__device__ __forceinline__ uint64_t stamp_after(uint32_t dep) {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
  return t;
}
#endif

// Word wi (0..7) of a 16-byte chunk set to zero.
__device__ __forceinline__ u32x4 zero_word(u32x4 w, uint32_t wi) {
  const uint32_t keep = (wi & 1u) ? 0x0000FFFFu : 0xFFFF0000u;
  const uint32_t di = wi >> 1;
  w.x &= di == 0 ? keep : 0xFFFFFFFFu;
  w.y &= di == 1 ? keep : 0xFFFFFFFFu;
  w.z &= di == 2 ? keep : 0xFFFFFFFFu;
  w.w &= di == 3 ? keep : 0xFFFFFFFFu;
  return w;
}

// Word wi (0..7) of a 16-byte chunk set to v.
[[maybe_unused]] __device__ __forceinline__ u32x4 put_word(u32x4 w, uint32_t wi, uint32_t v) {
  const uint32_t sh = (wi & 1u) << 4;
  const uint32_t m = ~(0xFFFFu << sh), x = (v & 0xFFFFu) << sh;
  const uint32_t di = wi >> 1;
  w.x = di == 0 ? (w.x & m) | x : w.x;
  w.y = di == 1 ? (w.y & m) | x : w.y;
  w.z = di == 2 ? (w.z & m) | x : w.z;
  w.w = di == 3 ? (w.w & m) | x : w.w;
  return w;
}

[[maybe_unused]] __device__ __forceinline__ void store16_chunk_wt(__amdgpu_buffer_rsrc_t r, uint32_t voff, u32x4 v) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, r, static_cast<int>(voff), 0, 19);  // sc0 sc1 nt
}

// LAYOUT: 0 packed variable, 1 fixed packed (stride == len), 2 fixed gapped
// MODE kRfc1071: the prefix table holds exact u32 sums -- u32 P at the dword
// positions when every end is 4-B aligned (as in REF), else u32 P at every
// word position (twice the LDS of REF's packed u16 table) -- so P(end) -
// P(start) is an image's exact word sum and folds
template <int U, int OP, int SPLIT, int LAYOUT, bool KEEP = false, int MODE = kRef, bool BLK = false>
__global__ void __launch_bounds__(kBlock) vvstream_kernel(VVArgs a) {
  constexpr bool FIXED = LAYOUT != 0;
  constexpr bool GAP = LAYOUT == 2;
  static_assert(!BLK || (OP == kFill && !GAP && MODE == kRef && !KEEP), "BLK: reference-mode FILL, no gaps");
  constexpr uint32_t kMinFill = BLK ? 64u : 30u;  // BLK: one field per 64-B block
  __shared__ u32x4 s_blk[kWavesPerBlock][BLK ? 4 : 1];  // BLK: the staged block of the image crossing the step
  __shared__ uint32_t s_end[kWavesPerBlock][FIXED ? 1 : kRing + kMirror];
  __shared__ __attribute__((aligned(16))) uint32_t s_pre[kWavesPerBlock][MODE == kRef ? 256 : 512];  // the step's prefixes
  __shared__ uint32_t s_fld[kWavesPerBlock][OP == kFill ? 64 : 1];              // kFill: field word + 1 per chunk
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock + wv;
  const uint64_t N = a.count;
#ifdef TCPCK_PROBE
  const uint64_t t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t t_desc = 0, t_first = 0;
#endif
  const uint32_t S = a.stride;
  const uint32_t L = FIXED ? a.len : 0u;
  uint64_t kb, ke;
  if (FIXED || SPLIT == 1) {
    dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  } else {
    const uint64_t first = a.offsets[0] - a.base;
    const uint64_t total = a.offsets[N - 1] - a.base + a.lengths[N - 1] - first;
    const uint64_t q = total / W, rm = total % W;
    dev::find_two(a.offsets, a.base, N, first + q * wid + rm * wid / W,
                  first + q * (wid + 1) + rm * (wid + 1) / W, kb, ke);
    if (wid == 0) kb = 0;
    if (wid + 1 == W) ke = N;
  }
  if (kb >= ke) return;

  uint64_t s0, s1;
  if constexpr (FIXED) {
    s0 = kb * S;
    s1 = (ke - 1) * S + L;
  } else {
    s0 = a.offsets[kb] - a.base;
    s1 = a.offsets[ke - 1] - a.base + a.lengths[ke - 1];
  }
  uint8_t *const arena = a.arena;
  const uint64_t A0 = dev::align128_rel(arena, s0);
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  const uint32_t nv = GAP ? 2 * nimg : nimg;  // (virtual) images whose ends the stream resolves
  bool bad = !(s1 >= s0 && s1 - A0 < (uint64_t{1} << 31));
#ifdef TCPCK_PROBE
  if (a.dbg) t_desc = stamp_after(static_cast<uint32_t>(s1 - A0));
#endif

  // k = batch image index, start = its offset in the arena
  auto store = [&](uint64_t k, uint32_t sum, uint64_t start) {
    const uint16_t c = dev::finish<MODE>(sum);  // tcp-header.h:262 (REF)
    if constexpr (OP == kVerify) {
      static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
    } else {
      if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
      if (OP == kFill) *reinterpret_cast<uint16_t *>(arena + start + 28) = c;  // raw, as the reference
    }
  };
  // the streaming path's form: start_rel run-relative (from A0), field store through the run's rsrc
  auto store_rel = [&](uint64_t k, uint32_t sum, uint32_t start_rel, __amdgpu_buffer_rsrc_t r) {
    const uint16_t c = dev::finish<MODE>(sum);  // tcp-header.h:262 (REF)
    if constexpr (OP == kVerify) {
      static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
    } else {
      if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
      if (OP == kFill && !a.defer_field) dev::store16_field(r, start_rel + 28, c);  // raw, as the reference
    }
  };

  if (!bad) {
    const uint32_t lead = static_cast<uint32_t>(s0 - A0);
    const uint32_t span = static_cast<uint32_t>(s1 - A0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const uint32_t last_chunk = span > 0 ? (span - 1) >> 4 : 0;
    // BLK: the batch's bytes, run-relative: a block is stored whole only inside
    // them, and the buffer covers the blocks of the run's fields that reach
    // past its span (their bytes belong to the next run's images, read here)
    int64_t blo = 0, bhi = 0;
    uint32_t extent = (last_chunk + 1) << 4;
    if constexpr (BLK) {
      const uint64_t b0 = FIXED ? 0 : a.offsets[0] - a.base;
      const uint64_t b1 = FIXED ? (N - 1) * S + L : a.offsets[N - 1] - a.base + a.lengths[N - 1];
      blo = static_cast<int64_t>(b0) - static_cast<int64_t>(A0);
      bhi = static_cast<int64_t>(b1) - static_cast<int64_t>(A0);
      const int64_t want = min(static_cast<int64_t>((span + 63u) & ~63u), bhi & ~int64_t{15});
      if (want > static_cast<int64_t>(extent)) extent = static_cast<uint32_t>(want);
    }
    const auto rsrc = dev::make_rsrc(arena + A0, extent);
    // BLK: the 64-B block at run-relative b lies inside the batch
    auto whole = [&](uint32_t b) { return static_cast<int64_t>(b) >= blo && static_cast<int64_t>(b) + 64 <= bhi; };
    uint32_t stage_f = 0;  // BLK: the staged field (run-relative), 0 = none
    // KEEP (kFill, small images): every line holds a checksum field, so read
    // it with the default policy -- still in L2 when the field store lands, it
    // leaves as a whole line instead of a masked partial write (gstream's
    // measurement, profiles/DESIGN_history_r01-r04.md section 4)
    auto load_step = [&](uint32_t st) -> u32x4 {
      if constexpr (KEEP) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), static_cast<int>(st << 10), 0);
        return u32x4{v.x, v.y, v.z, v.w};
      } else {
        return dev::load16_buf_nt(rsrc, lane << 4, st << 10);
      }
    };
    uint32_t *ring_end = s_end[wv];
    u32x4 *pre4 = reinterpret_cast<u32x4 *>(s_pre[wv]);
    const uint16_t *pre16 = reinterpret_cast<const uint16_t *>(s_pre[wv]);
    uint32_t *fld = s_fld[wv];
    if constexpr (OP == kFill) {
      fld[lane] = 0;
      __builtin_amdgcn_wave_barrier();
    }

    // the run's first data loads go out first
    uint32_t carry = 0, p_last = 0, jn = 0, fj = 0;
    uint32_t e_last = lead;  // end of image jn - 1 (= start of image jn), run-relative
    u32x4 ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u == 0 && a.keep_first && (lane < 8 || a.keep_first == 2)) {
        // the first line is the previous run's last: kept in L2 for its last
        // step (only that line: a whole first step with the default policy is
        // found in the Infinity Cache by the next launch over the same arena,
        // which cold batches never see; rstream's launcher has the numbers)
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), 0, 0);
        ring[0] = u32x4{v.x, v.y, v.z, v.w};
      } else {
        ring[u] = load_step(static_cast<uint32_t>(u));
      }
    }

    // descriptor rounds (variable layouts): lengths of run images [256 r, 256 r + 256), 4 per lane
    const uint32_t *lens = FIXED ? nullptr : a.lengths + kb;
    auto load_round = [&](uint32_t r, uint32_t (&d)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t j = r * kRound + 4 * lane + i;
        d[i] = j < nimg ? lens[j] : 0u;
      }
    };
    uint32_t loaded = FIXED ? nv : 0;  // ends available (run-relative image count)
    uint32_t pos = lead;                 // end of the last written image
    bool short_fill = false;             // kFill: an image < 30 B (two fields per chunk possible)
    // every end so far 4-B aligned: the step's prefix table then holds u32 P
    // at dword positions (no packing), else packed u16 P at word positions
    bool al4 = (lead & 3u) == 0 && (!FIXED || ((S & 3u) == 0 && (!GAP || (L & 3u) == 0)));
    // Round r's lengths are loaded when the round is written, not prefetched a
    // round ahead: a prefetch kept in registers across the step loop made the
    // compiler copy them on every step, behind a vmcnt(0) that drained the
    // data ring.  Runs of <= 256 images (C3 at 32x: ~16-25) write their one
    // round before the loop.
    auto fill_round = [&]() {            // load and write round (loaded / 256)
      const uint32_t r = loaded / kRound;
      uint32_t d[4];
      load_round(r, d);
      al4 = al4 && __ballot(((d[0] | d[1] | d[2] | d[3]) & 3u) != 0) == 0;  // lengths past nimg are 0
      if constexpr (MODE == kRfc1071) {
        // the u32 prefix differences are exact only below 128 KiB: a longer
        // image (an understated max_len hint, or the kernel named explicitly)
        // sends the run to the exact per-image pass, which rewrites every result
        bad = bad || __ballot((d[0] | d[1] | d[2] | d[3]) >= (1u << 17)) != 0;
      }
      const uint32_t e1 = d[0], e2 = e1 + d[1], e3 = e2 + d[2], e4 = e3 + d[3];
      const uint32_t incl = dev::wave_inclusive_scan(e4);
      const uint32_t ex = pos + incl - e4;
      if constexpr (OP == kFill) {
        const uint32_t jb = r * kRound + 4 * lane;
        bool sh = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) sh |= (jb + i < nimg) && d[i] < kMinFill;
        short_fill |= __ballot(sh) != 0;
      }
      // ends past the batch read as ~0 (never inside a step)
      const uint32_t jb = r * kRound + 4 * lane;
      const uint32_t v0 = jb < nimg ? ex + e1 : ~0u, v1 = jb + 1 < nimg ? ex + e2 : ~0u;
      const uint32_t v2 = jb + 2 < nimg ? ex + e3 : ~0u, v3 = jb + 3 < nimg ? ex + e4 : ~0u;
      const uint32_t si = (r * kRound) % kRing + 4 * lane;
      ring_end[si] = v0;
      ring_end[si + 1] = v1;
      ring_end[si + 2] = v2;
      ring_end[si + 3] = v3;
      if (si < kMirror) {
        ring_end[kRing + si] = v0;
        ring_end[kRing + si + 1] = v1;
        ring_end[kRing + si + 2] = v2;
        ring_end[kRing + si + 3] = v3;
      }
      pos = pos + dev::read_lane(incl, 63);
      loaded += kRound;
      if (loaded >= nimg) {
        // the last round: the 64 slots after it (consumed ends of the round
        // before) read as ~0 too, for the steps' reads past nimg
        const uint32_t sn = loaded % kRing + lane;
        ring_end[sn] = ~0u;
        if (sn < kMirror) ring_end[kRing + sn] = ~0u;
      }
      __builtin_amdgcn_wave_barrier();  // ends are read by other lanes
    };
    if constexpr (!FIXED) {
      fill_round();
      if constexpr (OP == kFill) {
        // nothing may be written into the arena before the layout is known to
        // be packed: check the whole run's lengths against its span first
        if (nimg > kRound) {
          uint32_t sum = 0;
          bool sh = false;
          for (uint32_t j = lane; j < nimg; j += 64) {
            const uint32_t l = lens[j];
            sum += l;
            sh |= l < kMinFill || (MODE == kRfc1071 && l >= (1u << 17));  // (RFC 1071: as fill_round)
          }
          short_fill = short_fill || __ballot(sh) != 0;
          bad = bad || short_fill || lead + dev::group_sum<64>(sum) != span;
        } else {
          bad = bad || short_fill || pos != span;
        }
      }
    } else {
      if constexpr (OP == kFill) bad = L < kMinFill;
    }
    auto end_of = [&](uint32_t j) -> uint32_t {  // run-relative end of run image j (j < nimg)
      if constexpr (GAP) {
        return lead + (j >> 1) * S + (j & 1u) * L;
      } else if constexpr (FIXED) {
        return lead + (j + 1) * S;
      } else {
        return ring_end[j % kRing];
      }
    };
    // the ends of images jn + lane, ~0 past the batch
    auto ends_at = [&](uint32_t jn0) -> uint32_t {
      if constexpr (FIXED) {
        const uint32_t j = jn0 + lane;
        return j < nv ? end_of(j) : ~0u;
      } else {
        return ring_end[jn0 % kRing + lane];  // mirrored: no wrap
      }
    };

    // AL4 (every end of the run 4-B aligned; decided once per run): the
    // prefix table holds u32 P at dword positions, no packing
    auto stream_run = [&](auto al4_tag) {
      constexpr bool AL4 = decltype(al4_tag)::value;
      for (uint32_t g = 0; g < nsteps && !bad; g += U) {
  #pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t st = g + u;
          const uint32_t sb = st << 10;
          const uint32_t c = sb + (lane << 4);
          u32x4 w = ring[u];
          const u32x4 raw = w;  // BLK: the block stores write the unmasked bytes
          if (sb == 0 || sb + 1024 > span) {
            const int32_t lo = min(max(static_cast<int32_t>(lead) - static_cast<int32_t>(c), 0), 16);
            const int32_t hi = min(max(static_cast<int32_t>(span) - static_cast<int32_t>(c), 0), 16);
            w = dev::apply_mask(w, dev::word_mask(lo, hi));
          }
          // the step's first ends, read before the sums (the LDS latency overlaps them)
          if (!FIXED && jn + 66 > loaded && loaded < nimg) fill_round();  // >= 64 ends (+ 1 field) ahead
          uint32_t j = jn + lane;
          uint32_t e = ends_at(jn);
          if constexpr (OP == kFill) {  // zero the checksum fields that lie in this step
            const uint32_t i = fj + lane;
            uint32_t f;
            if constexpr (FIXED)
              f = lead + i * S + 28;
            else
              f = (i == 0 ? lead : (i < nimg ? end_of(i - 1) : span)) + 28;
            const bool inf = i < nimg && f < sb + 1024;
            const uint64_t bf = __ballot(inf);
            if (bf) {
              if (inf) fld[(f - sb) >> 4] = ((f & 15u) >> 1) + 1u;  // post the word to the chunk's lane
              __builtin_amdgcn_wave_barrier();
              const uint32_t q = fld[lane];
              if (q) {
                fld[lane] = 0u;
                w = zero_word(w, q - 1u);
              }
              __builtin_amdgcn_wave_barrier();
              fj += static_cast<uint32_t>(__popcll(bf));
            }
          }
          const uint32_t q1 = dev::dot2_u16(w.x, 0u);
          const uint32_t q2 = dev::dot2_u16(w.y, q1);
          const uint32_t q3 = dev::dot2_u16(w.z, q2);
          const uint32_t tot = dev::dot2_u16(w.w, q3);
#ifdef TCPCK_PROBE
          if (a.dbg && st == 0) t_first = stamp_after(tot);
#endif
          const uint32_t incl = dev::wave_inclusive_scan(tot);
          bool table = false;
          for (;;) {  // once per step unless it holds more than 64 ends
            const bool inb = e < sb + 1024;
            const uint64_t bal = __ballot(inb);
            if (!bal) break;
            if (!table) {
              // P at the chunk start, then at word positions 2i (P = a + q_i) and
              // 2i + 1 (+ the low word of dword i): u32 at the dword positions
              // when every end is 4-B aligned, else packed low/high per dword
              const uint32_t p0 = carry + incl - tot;
              const uint32_t b1 = p0 + q1, b2 = p0 + q2, b3 = p0 + q3;
              if constexpr (AL4) {
                pre4[lane] = u32x4{p0, b1, b2, b3};
              } else if constexpr (MODE == kRfc1071) {  // exact u32 at all 8 word positions
                pre4[2 * lane] = u32x4{p0, p0 + (w.x & 0xFFFFu), b1, b1 + (w.y & 0xFFFFu)};
                pre4[2 * lane + 1] = u32x4{b2, b2 + (w.z & 0xFFFFu), b3, b3 + (w.w & 0xFFFFu)};
              } else
                pre4[lane] = u32x4{__builtin_amdgcn_perm(p0 + w.x, p0, 0x05040100u),
                                   __builtin_amdgcn_perm(b1 + w.y, b1, 0x05040100u),
                                   __builtin_amdgcn_perm(b2 + w.z, b2, 0x05040100u),
                                   __builtin_amdgcn_perm(b3 + w.w, b3, 0x05040100u)};
              __builtin_amdgcn_wave_barrier();  // cross-lane LDS reads below
              table = true;
            }
            const uint32_t cnt = static_cast<uint32_t>(__popcll(bal));  // lanes 0..cnt-1 (ends ascend)
            const uint32_t off = min(e - sb, 1022u);                    // the table is laid out like the step
            const uint32_t P = AL4 ? s_pre[wv][off >> 2]
                                   : (MODE == kRfc1071 ? s_pre[wv][off >> 1] : static_cast<uint32_t>(pre16[off >> 1]));
            // P of image jn + lane - 1: lane 0 keeps p_last (wave_shr:1, bound_ctrl off)
            const uint32_t pprev = static_cast<uint32_t>(
                __builtin_amdgcn_update_dpp(static_cast<int>(p_last), static_cast<int>(P), 0x138, 0xF, 0xF, false));
            if constexpr (OP == kFill) {
              const uint32_t el = static_cast<uint32_t>(
                  __builtin_amdgcn_update_dpp(static_cast<int>(e_last), static_cast<int>(e), 0x138, 0xF, 0xF, false));
              const uint32_t start = lane == 0 ? e_last : el;  // image jn + lane starts where jn + lane - 1 ends
              if constexpr (BLK) {
                if (inb) {
                  const uint16_t c = dev::finish<MODE>(P - pprev);  // tcp-header.h:262
                  if (a.out) static_cast<uint16_t *>(a.out)[kb + j] = c;
                  const uint32_t f = start + 28;  // tcp-header.h:177
                  if (f >= sb) {                  // the field's block is in this step's registers
                    fld[(f - sb) >> 4] = 0x80000000u | (((f & 15u) >> 1) << 16) | c;
                  } else if (whole(f & ~63u)) {   // the staged block (the image crossed the step start)
                    reinterpret_cast<uint16_t *>(s_blk[wv])[(f & 63u) >> 1] = c;
                  } else {
                    dev::store16_field(rsrc, f, c);
                  }
                }
              } else if (inb && (!GAP || (j & 1u))) {
                store_rel(kb + (GAP ? j >> 1 : j), P - pprev, start, rsrc);
              }
            } else {
              if (inb && (!GAP || (j & 1u))) store(kb + (GAP ? j >> 1 : j), P - pprev, 0);
            }
            p_last = dev::read_lane(P, cnt - 1);
            e_last = dev::read_lane(e, cnt - 1);
            jn += cnt;
            if (cnt < 64) break;
            if (!FIXED && jn + 66 > loaded && loaded < nimg) fill_round();  // never with AL4
            j = jn + lane;
            e = ends_at(jn);
          }
          if constexpr (BLK) {
            __builtin_amdgcn_wave_barrier();  // fld / s_blk written by other lanes
            // the staged block, its field resolved in this step: lanes 0-3 store it
            if (stage_f != 0 && stage_f < e_last) {
              if (lane < 4 && whole(stage_f & ~63u)) store16_chunk_wt(rsrc, (stage_f & ~63u) + 16 * lane, s_blk[wv][lane]);
              stage_f = 0;
            }
            // the fields resolved in this step: every lane of a field's 64-B block stores its chunk
            const uint32_t v = fld[lane];
            const uint64_t bv = __ballot(v != 0);
            if (bv) {
              const uint32_t cb = sb + ((lane & ~3u) << 4);  // the lane's block
              if ((bv >> (lane & ~3u)) & 0xFull) {
                if (whole(cb))
                  store16_chunk_wt(rsrc, sb + (lane << 4), v ? put_word(raw, (v >> 16) & 7u, v) : raw);
                else if (v)
                  dev::store16_field(rsrc, sb + (lane << 4) + (((v >> 16) & 7u) << 1), static_cast<uint16_t>(v));
              }
              if (v) fld[lane] = 0u;
            }
            // the image crossing this step's end, its field in this step: stage its block
            if (jn < nv) {
              const uint32_t f = e_last + 28;
              if (f >= sb && f < sb + 1024) {
                const uint32_t cb = f & ~63u;
                if (((sb + (lane << 4)) & ~63u) == cb) s_blk[wv][lane & 3u] = raw;
                stage_f = f;
              }
            }
          }
          __builtin_amdgcn_wave_barrier();  // the next step rewrites the table
          carry += dev::read_lane(incl, 63);
          ring[u] = load_step(st + U);
        }
      }
    };
    if (al4 && (FIXED || loaded >= nimg))
      stream_run(std::true_type{});
    else
      stream_run(std::false_type{});
    if constexpr (!FIXED) bad = bad || pos != span || loaded < nimg;
    if (BLK && !bad && jn < nv) {  // the image ending at the span: its block is staged
      const uint16_t c = dev::finish<MODE>(carry - p_last);
      if (lane == 0 && a.out) static_cast<uint16_t *>(a.out)[kb + jn] = c;
      const uint32_t f = e_last + 28;
      if (whole(f & ~63u)) {
        if (lane == 0) reinterpret_cast<uint16_t *>(s_blk[wv])[(f & 63u) >> 1] = c;
        __builtin_amdgcn_wave_barrier();
        if (lane < 4) store16_chunk_wt(rsrc, (f & ~63u) + 16 * lane, s_blk[wv][lane]);
      } else if (lane == 0) {
        dev::store16_field(rsrc, f, c);
      }
      jn = nv - 1 == jn ? nv : jn;  // (images >= 64 B: the last one only)
    }
    if (!bad && jn < nv) {  // ends exactly at the last step's end (= span): the first gets the rest
      const uint32_t rem = nv - jn;
      for (uint32_t i = lane; i < rem; i += 64) {
        const uint32_t v = jn + i;
        if (!GAP || (v & 1u)) store_rel(kb + (GAP ? v >> 1 : v), i == 0 ? carry - p_last : 0u, i == 0 ? e_last : span, rsrc);
      }
      jn = nv;
    }
    bad = bad || jn != nv;
  }
#ifdef TCPCK_PROBE
  if (a.dbg && lane == 0) {
    uint32_t hw_id, xcc_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    uint64_t *d = a.dbg + 8 * wid;
    d[0] = t_start;
    d[1] = t_desc;
    d[2] = t_first;
    d[3] = __builtin_amdgcn_s_memrealtime();
    d[4] = hw_id | (static_cast<uint64_t>(xcc_id) << 32);
    d[5] = ke - kb;
    d[6] = s1 - s0;
    d[7] = 0;
  }
#endif
  if (bad) {  // wave-uniform: the layout is not what the walk assumed -> exact per-image pass
    for (uint64_t k = kb; k < ke; ++k) {
      const uint64_t start = FIXED ? k * S : a.offsets[k] - a.base;
      const uint32_t len = FIXED ? L : a.lengths[k];
      if (OP == kFill && len < 30) continue;  // precondition of kFill (the C ABI rejects these)
      const uint32_t sum = dev::wave_image_sum<2, MODE>(arena, start, len, OP == kFill);
      if (lane == 0) store(k, sum, start);
    }
  }
}

template <int U, int OP, int SPLIT, int LAYOUT, bool KEEP = false, int MODE = kRef, bool BLK = false>
hipError_t launch_one(const RunArgs &s, uint32_t oversub, int flags, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(vvstream_kernel<U, OP, SPLIT, LAYOUT, KEEP, MODE, BLK>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  uint64_t blocks = resident * (oversub ? oversub : 1);
  const uint64_t need = (s.count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  VVArgs a{};
  a.arena = s.arena;
  a.offsets = s.offsets;
  a.lengths = s.lengths;
  a.base = s.base;
  a.count = s.count;
  a.out = s.out;
  a.per_wave = s.count / (blocks * kWavesPerBlock);
  a.rem = s.count % (blocks * kWavesPerBlock);
  a.stride = static_cast<uint32_t>(s.stride);
  a.len = s.len;
  a.order = (flags & 8) ? 4u : dev::kOrderDefault;  // groups of 16 blocks per XCD
  a.keep_first = (flags & 16) ? ((flags & 256) ? 2u : 1u) : 0u;
  a.defer_field = (flags & 64) ? 1u : 0u;
  a.dbg = s.dbg;
  hipLaunchKernelGGL((vvstream_kernel<U, OP, SPLIT, LAYOUT, KEEP, MODE, BLK>), dim3(static_cast<uint32_t>(blocks)),
                     dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int U, int SPLIT, int LAYOUT>
hipError_t dispatch(int op, const RunArgs &a, uint32_t oversub, int flags, uint32_t num_cus, hipStream_t s) {
  if (a.mode != kRef) {  // RFC 1071 (no KEEP variant)
    switch (op) {
      case kChecksum: return launch_one<U, kChecksum, SPLIT, LAYOUT, false, kRfc1071>(a, oversub, flags, num_cus, s);
      case kVerify: return launch_one<U, kVerify, SPLIT, LAYOUT, false, kRfc1071>(a, oversub, flags, num_cus, s);
      case kFill: return launch_one<U, kFill, SPLIT, LAYOUT, false, kRfc1071>(a, oversub, flags, num_cus, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum, SPLIT, LAYOUT>(a, oversub, flags, num_cus, s);
    case kVerify: return launch_one<U, kVerify, SPLIT, LAYOUT>(a, oversub, flags, num_cus, s);
    case kFill:
#ifdef TCPCK_PROBE
      // BLK: measured against AUTO's FILL forms and slower at every grid
      // (scripts/fill_block_probe.py, profiles/r05/): the probe library only
      if constexpr (LAYOUT != 2)
        if (flags & 128) return launch_one<U, kFill, SPLIT, LAYOUT, false, kRef, true>(a, oversub, flags, num_cus, s);
#endif
      return (flags & 32) ? launch_one<U, kFill, SPLIT, LAYOUT, true>(a, oversub, flags, num_cus, s)
                          : launch_one<U, kFill, SPLIT, LAYOUT>(a, oversub, flags, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_vvstream(int op, int variant, bool fixed, const RunArgs &a, uint32_t num_cus,
                           hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  if (fixed && (a.len == 0 || a.stride < a.len || a.stride > (1u << 24))) return hipErrorInvalidValue;
  const bool gap = fixed && a.stride != a.len;
  const uint64_t bytes = fixed ? a.count * a.stride : a.total_bytes;
  uint32_t m = a.oversub ? a.oversub : 1;
  // 8: XCD-chunked run order; 16: L2-kept first line; 32: kFill reads every
  // step with the default cache policy (small images); 64: kFill writes the
  // results only (the caller runs launch_patch_fields for the fields); 128:
  // kFill stores each field's whole 64-B block (BLK; reference mode, no gaps)
  int flags = variant & 248;
  if ((flags & 64) && (op != kFill || !a.out)) return hipErrorInvalidValue;
#ifdef TCPCK_PROBE
  if ((flags & 128) && (op != kFill || a.mode != kRef || gap || (flags & 96))) return hipErrorInvalidValue;
#else
  if (flags & 128) return hipErrorInvalidValue;  // BLK: the probe library only
#endif
  variant &= 7;
#ifdef TCPCK_PROBE
  if (variant == 5) {  // (probe) the policy with its whole first step L2-kept, as before round 5
    variant = 4;
    flags |= 256;
  }
#endif
  int u8 = (variant & 1);
  int split = variant >= 2 ? 1 : 0;
  if (variant == 4) {
    // library policy: oversubscribe by size, runs of >= 8 KiB, M a power of two
    // (M = 16/24/40 measured 2-4% below 32 on the run kernels,
    // profiles/r01/oversub_c2c3.log; C3: 32).  From M = 32, U8 (C3 85.0-86.3%
    // vs U4 82.7-84.2%); once M >= 4 the dispatcher balances the runs and
    // equal-count runs (no offset searches) win.  Larger batches keep the
    // runs short with larger M, as rstream does (C5: profiles/r01/split_probe.log).
    m = dev::oversub_for(a.oversub, bytes, static_cast<uint64_t>(num_cus) * 32, 1024, 8u << 10);
    u8 = m >= 32;
    if (op == kFill && !fixed && !(flags & 224)) {  // (deferred fields, + 64: the stream is CHECKSUM's; BLK too)
      // FILL of packed variable batches: runs of >= 4 KiB and U4 (C3: M = 64,
      // 53.7 % of the roof against 48.6 % at the checksum policy's U8 x 32;
      // M = 96-255 fall off fast, profiles/r01/c3_fill_sweep.log)
      m = dev::oversub_for(a.oversub, bytes, static_cast<uint64_t>(num_cus) * 32, 1024, 4u << 10);
      u8 = false;
    }
    split = m >= 4;
  } else {
#ifdef TCPCK_PROBE
    // measurement-only (libtcpck_probe.so): 0/1 byte split U4/U8, 2/3 equal counts, one run per resident wave
    if (variant > 4 || variant < 0) return hipErrorInvalidValue;
#else
    return hipErrorInvalidValue;  // the product library runs the policy only
#endif
  }
  if (gap) return u8 ? dispatch<8, 1, 2>(op, a, m, flags, num_cus, stream) : dispatch<4, 1, 2>(op, a, m, flags, num_cus, stream);
  if (fixed) return u8 ? dispatch<8, 1, 1>(op, a, m, flags, num_cus, stream) : dispatch<4, 1, 1>(op, a, m, flags, num_cus, stream);
  if (split) return u8 ? dispatch<8, 1, 0>(op, a, m, flags, num_cus, stream) : dispatch<4, 1, 0>(op, a, m, flags, num_cus, stream);
  return u8 ? dispatch<8, 0, 0>(op, a, m, flags, num_cus, stream) : dispatch<4, 0, 0>(op, a, m, flags, num_cus, stream);
}

}  // namespace tcpck
