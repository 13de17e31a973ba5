// tcpck_vvstream.hip -- packed variable-length batches (C3): one contiguous
// run of whole images per wave, the boundaries of each 1 KiB step resolved by
// the lanes in parallel from a per-wave LDS ring of image end positions.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  Packed images make the run one
// flat byte stream and sum(k) = P(end_k) - P(end_{k-1}) (mod 2^16), with P(x)
// the word sum of the run before byte x.
//
//   * run split as rvstream (byte-balanced, two lockstep 64-ary searches);
//   * image end positions: 256 lengths at a time are read with one vector
//     load per lane (4 lengths each, prefetched a round ahead, so the load
//     ring drains once per 256 images), prefix-summed across the wave and
//     written to a 512-entry LDS ring per wave;
//   * per step: lane j reads end e(jn + j) from LDS; the lanes whose end falls
//     in the step (a ballot, <= 64 since images are >= 16 B, at most one end
//     per chunk) post the end's byte offset into the LDS slot of the lane
//     holding that chunk; that lane forms P = carry + exclusive scan + its
//     words before the end (partial sums of its own v_dot2 chain) and clears
//     its slot; the boundary lane takes P back (ds_bpermute); sum(jn + j) =
//     P(j) - P(j - 1), P(-1) = the last P of the step before (one SGPR);
//   * results leave from lanes 0..cnt-1 as one contiguous store per step.
// A wave whose lengths are shorter than 16 B or disagree with the offsets
// (layout hint wrong) recomputes its images one by one.  kFill is served by
// the span kernel (the host routes it); kChecksum and kVerify here.
#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

constexpr uint32_t kRound = 256;   // ends loaded per round (4 per lane)
constexpr uint32_t kRing = 512;    // LDS ring entries per wave (two rounds)

__device__ __forceinline__ uint32_t lane_bpermute(uint32_t v, uint32_t src_lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src_lane << 2), static_cast<int>(v)));
}

// RES: how a step's boundaries are resolved.
//   0: slot hand-off -- the lane holding an end posts it to the LDS slot of the
//      chunk's lane, which forms P from its own v_dot2 partial sums; the
//      boundary lane pulls P back (ds_bpermute).  One end per chunk at most:
//      images < 16 B fall back to per-image sums.
//   1: prefix table -- every lane writes the run prefix P at each of its
//      chunk's 8 word positions as packed u16s (one ds_write_b128: P matters
//      mod 2^16 only), the boundary lane reads the u16 at its end's byte offset
//      in the step (the table is laid out like the step).  Any number of ends
//      per chunk (a step with more than 64 ends loops), 3 LDS ops per step
//      instead of 7, no cross-lane selects.
template <int U, int OP, int SPLIT, int RES = 0>
__global__ void __launch_bounds__(kBlock)
    vvstream_kernel(uint8_t *__restrict__ arena, const uint64_t *__restrict__ offsets,
                    const uint32_t *__restrict__ lengths, uint64_t base, uint64_t count, void *__restrict__ out,
                    uint64_t per_wave, uint64_t rem) {
  __shared__ uint32_t s_end[kWavesPerBlock][kRing];
  __shared__ uint32_t s_slot[kWavesPerBlock][RES == 0 ? 64 : 1];  // end offset in chunk + 1, posted to the chunk's lane
  __shared__ __attribute__((aligned(16))) uint32_t s_pre[kWavesPerBlock][RES == 1 ? 256 : 1];  // packed u16 prefixes
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + wv;
  const uint64_t N = count;
  uint64_t kb, ke;
  if (SPLIT == 1) {
    dev::count_split(wid, per_wave, rem, kb, ke);
  } else {
    const uint64_t first = offsets[0] - base;
    const uint64_t total = offsets[N - 1] - base + lengths[N - 1] - first;
    const uint64_t q = total / W, rm = total % W;
    dev::find_two(offsets, base, N, first + q * wid + rm * wid / W, first + q * (wid + 1) + rm * (wid + 1) / W, kb, ke);
    if (wid == 0) kb = 0;
    if (wid + 1 == W) ke = N;
  }
  if (kb >= ke) return;

  const uint64_t s0 = offsets[kb] - base;
  const uint64_t s1 = offsets[ke - 1] - base + lengths[ke - 1];
  const uint64_t A0 = dev::align128_rel(arena, s0);
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  bool bad = !(s1 >= s0 && s1 - A0 < (uint64_t{1} << 31));

  auto store = [&](uint64_t k, uint32_t sum) {
    const uint16_t c = static_cast<uint16_t>(~sum);  // tcp-header.h:262
    if constexpr (OP == kVerify)
      static_cast<uint8_t *>(out)[k] = (c == 0) ? 1 : 0;
    else
      static_cast<uint16_t *>(out)[k] = c;
  };

  if (!bad) {
    const uint32_t lead = static_cast<uint32_t>(s0 - A0);
    const uint32_t span = static_cast<uint32_t>(s1 - A0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const uint32_t last_chunk = span > 0 ? (span - 1) >> 4 : 0;
    const auto rsrc = dev::make_rsrc(arena + A0, (last_chunk + 1) << 4);
    auto load_step = [&](uint32_t st) -> u32x4 { return dev::load16_buf_nt(rsrc, lane << 4, st << 10); };
    uint32_t *ring_end = s_end[wv];
    uint32_t *slot = s_slot[wv];
    if constexpr (RES == 0) {
      slot[lane] = 0;
      __builtin_amdgcn_wave_barrier();
    }
    u32x4 *pre4 = reinterpret_cast<u32x4 *>(s_pre[wv]);
    const uint16_t *pre16 = reinterpret_cast<const uint16_t *>(s_pre[wv]);

    // descriptor rounds: lengths of run images [256 r, 256 r + 256), 4 per lane
    const uint32_t *lens = lengths + kb;
    auto load_round = [&](uint32_t r, uint32_t (&d)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t j = r * kRound + 4 * lane + i;
        d[i] = j < nimg ? lens[j] : 0u;
      }
    };
    uint32_t dnext[4];
    load_round(0, dnext);
    uint32_t loaded = 0;     // ends written to the ring (run-relative image count)
    uint32_t pos = lead;     // end of the last written image
    bool short_img = false;  // an image < 16 B: more than one end per chunk possible
    auto fill_round = [&]() {  // write round (loaded / 256) from dnext, prefetch the next
      uint32_t d[4] = {dnext[0], dnext[1], dnext[2], dnext[3]};
      const uint32_t r = loaded / kRound;
      load_round(r + 1, dnext);
      uint32_t e1 = d[0], e2 = e1 + d[1], e3 = e2 + d[2], e4 = e3 + d[3];
      const uint32_t incl = dev::wave_inclusive_scan(e4);
      const uint32_t ex = pos + incl - e4;
      const uint32_t jb = r * kRound + 4 * lane;
      bool sh = false;
#pragma unroll
      for (int i = 0; i < 4; ++i) sh |= (jb + i < nimg) && d[i] < 16;
      if (RES == 0) short_img |= __ballot(sh) != 0;
      const uint32_t si = (r * kRound) % kRing + 4 * lane;
      ring_end[si] = ex + e1;
      ring_end[si + 1] = ex + e2;
      ring_end[si + 2] = ex + e3;
      ring_end[si + 3] = ex + e4;
      pos = pos + dev::read_lane(incl, 63);
      loaded += kRound;
      __builtin_amdgcn_wave_barrier();  // ends are read by other lanes
    };
    uint32_t carry = 0, p_last = 0, jn = 0;
    u32x4 ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ring[u] = load_step(static_cast<uint32_t>(u));
    // the first ends after the data loads: the lengths' latency overlaps the
    // stream's instead of preceding it (straight-line code: vmcnt(U), no drain)
    fill_round();

    for (uint32_t g = 0; g < nsteps && !short_img; g += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t st = g + u;
        const uint32_t sb = st << 10;
        const uint32_t c = sb + (lane << 4);
        u32x4 w = ring[u];
        if (sb == 0 || sb + 1024 > span) {
          const int32_t lo = min(max(static_cast<int32_t>(lead) - static_cast<int32_t>(c), 0), 16);
          const int32_t hi = min(max(static_cast<int32_t>(span) - static_cast<int32_t>(c), 0), 16);
          w = dev::apply_mask(w, dev::word_mask(lo, hi));
        }
        uint32_t j = jn + lane;
        uint32_t e = ~0u;
        if constexpr (RES == 1) {  // the step's first ends, read before the sums (LDS latency overlaps)
          if (jn + 64 > loaded && loaded < nimg) fill_round();  // keep >= 64 ends ahead
          j = jn + lane;
          e = j < nimg ? ring_end[j % kRing] : ~0u;
        }
        const uint32_t q1 = dev::dot2_u16(w.x, 0u);
        const uint32_t q2 = dev::dot2_u16(w.y, q1);
        const uint32_t q3 = dev::dot2_u16(w.z, q2);
        const uint32_t tot = dev::dot2_u16(w.w, q3);
        const uint32_t incl = dev::wave_inclusive_scan(tot);
        if constexpr (RES == 1) {
          bool table = false;
          for (;;) {  // once per step unless it holds more than 64 ends
            const bool inb = e < sb + 1024;
            const uint64_t bal = __ballot(inb);
            if (!bal) break;
            if (!table) {
              // P at the chunk start, then at word positions 2i (P = a + q_i)
              // and 2i + 1 (+ low word of dword i), packed low/high per dword
              const uint32_t a = carry + incl - tot;
              const uint32_t b1 = a + q1, b2 = a + q2, b3 = a + q3;
              pre4[lane] = u32x4{__builtin_amdgcn_perm(a + w.x, a, 0x05040100u),
                                 __builtin_amdgcn_perm(b1 + w.y, b1, 0x05040100u),
                                 __builtin_amdgcn_perm(b2 + w.z, b2, 0x05040100u),
                                 __builtin_amdgcn_perm(b3 + w.w, b3, 0x05040100u)};
              __builtin_amdgcn_wave_barrier();  // cross-lane LDS reads below
              table = true;
            }
            const uint32_t cnt = static_cast<uint32_t>(__popcll(bal));  // lanes 0..cnt-1 (ends ascend)
            const uint32_t P = pre16[inb ? ((e - sb) >> 1) : 0u];     // the table is laid out like the step
            const uint32_t pl = static_cast<uint32_t>(
                __builtin_amdgcn_update_dpp(static_cast<int>(p_last), static_cast<int>(P), 0x138, 0xF, 0xF, false));
            const uint32_t pprev = lane == 0 ? p_last : pl;  // wave_shr:1
            if (inb) store(kb + j, P - pprev);
            p_last = dev::read_lane(P, cnt - 1);
            jn += cnt;
            if (cnt < 64) break;
            if (jn + 64 > loaded && loaded < nimg) fill_round();
            j = jn + lane;
            e = j < nimg ? ring_end[j % kRing] : ~0u;
          }
          __builtin_amdgcn_wave_barrier();  // the next step rewrites the table
        } else {
          if (jn + 64 > loaded && loaded < nimg) fill_round();  // keep >= 64 ends ahead
          j = jn + lane;
          e = j < nimg ? ring_end[j % kRing] : ~0u;
          const bool inb = e < sb + 1024;
          const uint64_t bal = __ballot(inb);
          if (bal) {
            const uint32_t cnt = static_cast<uint32_t>(__popcll(bal));  // lanes 0..cnt-1 (ends ascend)
            const uint32_t rel = e - sb;
            const uint32_t cl = rel >> 4;
            if (inb) slot[cl] = (rel & 15u) + 1u;  // tell the chunk's lane where the end lies
            __builtin_amdgcn_wave_barrier();        // cross-lane LDS hand-off: no per-lane forwarding
            const uint32_t rr = slot[lane];
            if (rr) slot[lane] = 0u;
            __builtin_amdgcn_wave_barrier();
            const uint32_t r = rr ? rr - 1 : 0u;
            const uint32_t di = r >> 2;
            const uint32_t qd = di == 0 ? 0u : (di == 1 ? q1 : (di == 2 ? q2 : q3));
            const uint32_t dw = di == 0 ? w.x : (di == 1 ? w.y : (di == 2 ? w.z : w.w));
            const uint32_t pb = carry + incl - tot + qd + ((r & 2u) ? (dw & 0xFFFFu) : 0u);
            const uint32_t pj = lane_bpermute(pb, inb ? cl : 0u);
            const uint32_t pl = lane_bpermute(pj, lane ? lane - 1 : 0u);
            const uint32_t pprev = lane == 0 ? p_last : pl;
            if (inb) store(kb + j, pj - pprev);
            p_last = dev::read_lane(pj, cnt - 1);
            jn += cnt;
          }
        }
        carry += dev::read_lane(incl, 63);
        ring[u] = load_step(st + U);
      }
    }
    bad = short_img || pos != span || loaded < nimg;
    if (!bad && jn < nimg) {  // ends exactly at the last step's end (= span): the first gets the rest
      const uint32_t rem = nimg - jn;
      for (uint32_t i = lane; i < rem; i += 64) store(kb + jn + i, i == 0 ? carry - p_last : 0u);
      jn = nimg;
    }
    bad = bad || jn != nimg;
  }
  if (bad) {  // wave-uniform: the layout is not what the walk assumed -> exact per-image pass
    for (uint64_t k = kb; k < ke; ++k) {
      const uint32_t sum = dev::wave_image_sum<2, kRef>(arena, offsets[k] - base, lengths[k], false);
      if (lane == 0) store(k, sum);
    }
  }
}

template <int U, int OP, int SPLIT, int RES>
hipError_t launch_one(const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(vvstream_kernel<U, OP, SPLIT, RES>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  uint64_t blocks = resident * dev::oversub_for(a.oversub, a.total_bytes, resident * kWavesPerBlock, 32, 8u << 10);
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((vvstream_kernel<U, OP, SPLIT, RES>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream,
                     a.arena, a.offsets, a.lengths, a.base, a.count, a.out, a.count / (blocks * kWavesPerBlock),
                     a.count % (blocks * kWavesPerBlock));
  return hipGetLastError();
}

template <int U, int SPLIT, int RES = 0>
hipError_t dispatch(int op, const SpanArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum, SPLIT, RES>(a, num_cus, s);
    case kVerify: return launch_one<U, kVerify, SPLIT, RES>(a, num_cus, s);
    default: return hipErrorInvalidValue;  // kFill: span kernel
  }
}

}  // namespace

hipError_t launch_vvstream(int op, int variant, const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  if (variant == 4 || variant == 9) {
    // library policy (prefix-table resolution): oversubscribe by size, runs of
    // >= 8 KiB, M a power of two <= 32 (M = 16/24/40 measured 2-4% below 32 on
    // both run kernels, profiles/r01/oversub_c2c3.log).  At M = 32, U8 (C3
    // 85.0-86.3% vs U4 82.7-84.2%); once M >= 4 the dispatcher balances the runs
    // and equal-count runs (no offset searches) win.
    SpanArgs b = a;
    uint32_t m = a.oversub;
    if (m == 0) {
      const uint64_t per = static_cast<uint64_t>(num_cus) * 32 * (8u << 10);
      const uint64_t q = a.total_bytes / per;
      m = 1;
      while (m < 32 && 2 * m <= q) m *= 2;
    }
    b.oversub = m;
    if (m >= 32) return dispatch<8, 1, 1>(op, b, num_cus, stream);
    return m >= 4 ? dispatch<4, 1, 1>(op, b, num_cus, stream) : dispatch<4, 0, 1>(op, b, num_cus, stream);
  }
  switch (variant) {
    case 0: return dispatch<4, 0>(op, a, num_cus, stream);
    case 1: return dispatch<8, 0>(op, a, num_cus, stream);
    case 2: return dispatch<4, 1>(op, a, num_cus, stream);
    case 3: return dispatch<8, 1>(op, a, num_cus, stream);
    case 5: return dispatch<4, 0, 1>(op, a, num_cus, stream);
    case 6: return dispatch<8, 0, 1>(op, a, num_cus, stream);
    case 7: return dispatch<4, 1, 1>(op, a, num_cus, stream);
    case 8: return dispatch<8, 1, 1>(op, a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
