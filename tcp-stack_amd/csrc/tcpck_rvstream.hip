// tcpck_rvstream.hip -- packed variable-length batches (C3): one contiguous,
// byte-balanced run of whole images per wave, image boundaries walked in
// scalar registers from the length array.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  Packed images (offsets[k+1] ==
// offsets[k] + lengths[k], TCPCK_LAYOUT_PACKED) make the batch one flat byte
// stream, and sum(k) = P(end_k) - P(start_k) (mod 2^16) with P(x) the word sum
// of the wave's run before byte x.  This is rstream (tcpck_rstream.hip) with
// the fixed stride replaced by the length array:
//
//   * wave w owns the images starting in bytes [w T / W, (w+1) T / W) of the
//     batch (T = batch bytes): kb and ke come from two 64-ary searches over the
//     offsets run in lockstep (one 64-lane probe per level, 4 levels for 4M
//     images), so runs are byte-balanced whatever the length mix;
//   * the run start is rounded down to a 128-B line; lane l reads the 16 B at
//     1024 s + 16 l of step s, U steps in flight in a register ring refilled in
//     place; per step a DPP inclusive scan and the step total (readlane 63);
//   * the boundary walk is wave-uniform: next boundary = current + lengths[k],
//     the length read by a scalar load issued one boundary ahead (lgkmcnt, so
//     it never waits on the vector load ring); any length works, including
//     images shorter than a 16-B chunk and empty images (several boundaries in
//     one chunk are just several scalar iterations);
//   * P(boundary) = carry + scan(lane) - sum(lane) + the lane's words before
//     the byte (v_readlane); results are staged one per lane and leave as 64-
//     wide coalesced stores;
//   * kFill subtracts each image's checksum word (bytes 28-29, read from the
//     stream when the walk passes it) and writes the result there
//     (tcp-header.h:177); kVerify stores checksum == 0.
// Layout check: a wave whose length walk does not end exactly at
// offsets[ke-1] + lengths[ke-1] (hint wrong: not packed) recomputes its images
// one by one from the offsets, so results stay exact.
#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

template <int U, int OP, int SPLIT = 0>
__global__ void __launch_bounds__(kBlock)
    rvstream_kernel(uint8_t *__restrict__ arena, const uint64_t *__restrict__ offsets,
                    const uint32_t *__restrict__ lengths, uint64_t base, uint64_t count, void *__restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint64_t N = count;
  // byte-balanced split of the batch's span [first, first + total)
  const uint64_t first = offsets[0] - base;
  const uint64_t total = offsets[N - 1] - base + lengths[N - 1] - first;
  const uint64_t q = total / W, rm = total % W;
  const uint64_t t0 = first + q * wid + rm * wid / W;
  const uint64_t t1 = first + q * (wid + 1) + rm * (wid + 1) / W;
  uint64_t kb, ke;
  if (SPLIT == 1) {
    kb = wid * N / W;
    ke = (wid + 1) * N / W;
  } else {
    dev::find_two(offsets, base, N, t0, t1, kb, ke);
  }
  if (wid == 0) kb = 0;
  if (wid + 1 == W) ke = N;
  if (kb >= ke) return;

  const uint64_t s0 = offsets[kb] - base;
  const uint64_t s1 = offsets[ke - 1] - base + lengths[ke - 1];
  const uint64_t A0 = dev::align128_rel(arena, s0);
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  // run must be ordered and below 2^31 bytes for the 32-bit walk
  bool bad = !(s1 >= s0 && s1 - A0 < (uint64_t{1} << 31));

  auto store = [&](uint64_t k, uint32_t sum, uint64_t field_pos) {
    const uint16_t c = static_cast<uint16_t>(~sum);  // tcp-header.h:262
    if constexpr (OP == kVerify) {
      static_cast<uint8_t *>(out)[k] = (c == 0) ? 1 : 0;
    } else {
      if (out) static_cast<uint16_t *>(out)[k] = c;
      if (OP == kFill && field_pos != ~uint64_t{0}) *reinterpret_cast<uint16_t *>(arena + field_pos) = c;
    }
  };

  if (!bad) {
    const uint32_t lead = static_cast<uint32_t>(s0 - A0);
    const uint32_t span = static_cast<uint32_t>(s1 - A0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const uint32_t last_chunk = span > 0 ? (span - 1) >> 4 : 0;
    const uint8_t *runp = arena + A0;
    const uint32_t *lens = lengths + kb;

    auto load_step = [&](uint32_t st) -> u32x4 {
      const uint32_t ci = min((st << 6) + lane, last_chunk);  // clamp: always a legal address
      return dev::load16_nt(runp + 16 * static_cast<uint64_t>(ci));
    };

    // wave-uniform walk (SGPRs), run-relative 32-bit positions:
    // image jn starts at nb; lnext = lengths of image jn (scalar load in flight)
    const uint32_t len0 = lens[0];
    uint32_t nb = lead + len0;
    uint32_t jn = 1;
    uint32_t lnext = lens[min(jn, nimg - 1)];
    uint32_t carry = 0;
    uint32_t p_last = 0;
    // kFill: checksum word of the current image (the one ending at nb)
    uint32_t fpos = len0 >= 30 ? lead + 28 : ~0u;  // pending field position, ~0 = none / read
    uint32_t fword = 0;
    uint32_t fstage = ~0u;  // staged field positions (kFill write-back)
    uint32_t stage = 0;
    uint32_t out_rel = 0;

    auto flush = [&](uint32_t n) {
      if (lane < n) {
        const uint64_t k = kb + out_rel + lane;
        const uint16_t c = static_cast<uint16_t>(stage);
        if constexpr (OP == kVerify) {
          static_cast<uint8_t *>(out)[k] = (c == 0) ? 1 : 0;
        } else {
          if (out) static_cast<uint16_t *>(out)[k] = c;
          if (OP == kFill && fstage != ~0u) *reinterpret_cast<uint16_t *>(arena + A0 + fstage) = c;
        }
      }
    };
    auto emit = [&](uint32_t jr, uint32_t sum, uint32_t fp) {
      const uint32_t j = jr - out_rel;
      stage = lane == j ? (~sum & 0xFFFFu) : stage;
      if (OP == kFill) fstage = lane == j ? fp : fstage;
      if (j == 63) {
        flush(64);
        out_rel += 64;
      }
    };
    // kFill: read the pending field word if it lies in step [sb, sb + 1024)
    auto grab_field = [&](uint32_t sb, const u32x4 &w) {
      if (fpos != ~0u && fpos >= sb && fpos < sb + 1024) {
        const uint32_t rel = fpos - sb;
        const uint32_t lb = rel >> 4, r = rel & 15u;
        const uint32_t d = dev::read_lane(r < 4 ? w.x : (r < 8 ? w.y : (r < 12 ? w.z : w.w)), lb);
        fword = (r & 2u) ? (d >> 16) : (d & 0xFFFFu);
      }
    };

    u32x4 ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ring[u] = load_step(static_cast<uint32_t>(u));

    for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t st = g + u;
        const uint32_t sb = st << 10;
        u32x4 w = ring[u];
        if (sb == 0 || sb + 1024 > span) {  // run edge: keep words of [lead, span) only
          const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
          const int32_t lo = min(max(static_cast<int32_t>(lead) - crel, 0), 16);
          const int32_t hi = min(max(static_cast<int32_t>(span) - crel, 0), 16);
          w = dev::apply_mask(w, dev::word_mask(lo, hi));
        }
        if constexpr (OP == kFill) grab_field(sb, w);
        const uint32_t tot = dev::ref_chunk_sum(w);
        const uint32_t incl = dev::wave_inclusive_scan(tot);
        while (nb < sb + 1024 && jn < nimg) {  // scalar: boundaries in this step
          const uint32_t rel = nb - sb;
          const uint32_t lb = rel >> 4;
          const uint32_t r = rel & 15u;
          uint32_t P = carry + dev::read_lane(incl, lb) - dev::read_lane(tot, lb);
          if (r)
            P += dev::words_before(r, dev::read_lane(w.x, lb), dev::read_lane(w.y, lb), dev::read_lane(w.z, lb),
                                   dev::read_lane(w.w, lb));
          if constexpr (OP == kFill) {
            emit(jn - 1, P - p_last - (fpos != ~0u ? fword : 0u), fpos);
            fpos = lnext >= 30 ? nb + 28 : ~0u;  // the next image's field
            fword = 0;
            grab_field(sb, w);
          } else {
            emit(jn - 1, P - p_last, 0);
          }
          p_last = P;
          nb += lnext;
          ++jn;
          lnext = lens[min(jn, nimg - 1)];  // scalar load, consumed at the next boundary
        }
        carry += dev::read_lane(incl, 63);
        ring[u] = load_step(st + U);
      }
    }
    bad = jn != nimg || nb != span;
    if (!bad) {
      if constexpr (OP == kFill)
        emit(nimg - 1, carry - p_last - (fpos != ~0u ? fword : 0u), fpos);
      else
        emit(nimg - 1, carry - p_last, 0);
      const uint32_t pending = nimg - out_rel;
      if (pending) flush(pending);
    }
  }
  if (bad) {  // wave-uniform: the layout is not what the walk assumed -> exact per-image pass
    for (uint64_t k = kb; k < ke; ++k) {
      const uint64_t st = offsets[k] - base;
      const uint32_t ln = lengths[k];
      const bool fld = OP == kFill && ln >= 30;
      const uint32_t sum = dev::wave_image_sum<2, kRef>(arena, st, ln, fld);
      if (lane == 0) store(k, sum, fld ? st + 28 : ~uint64_t{0});
    }
  }
}

template <int U, int OP, int SPLIT>
hipError_t launch_one(const SpanArgs &a, uint32_t num_cus, uint32_t blocks_per_cu, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(rvstream_kernel<U, OP, SPLIT>);
  const uint32_t cap = (blocks_per_cu && blocks_per_cu < per_cu) ? blocks_per_cu : per_cu;
  uint64_t blocks = static_cast<uint64_t>(cap) * num_cus;
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((rvstream_kernel<U, OP, SPLIT>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a.arena,
                     a.offsets, a.lengths, a.base, a.count, a.out);
  return hipGetLastError();
}

template <int U, int SPLIT = 0>
hipError_t dispatch(int op, const SpanArgs &a, uint32_t num_cus, uint32_t cap, hipStream_t s) {
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum, SPLIT>(a, num_cus, cap, s);
    case kFill: return launch_one<U, kFill, SPLIT>(a, num_cus, cap, s);
    case kVerify: return launch_one<U, kVerify, SPLIT>(a, num_cus, cap, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_rvstream(int op, int variant, const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  const uint32_t cap = static_cast<uint32_t>(variant >> 8) & 0xFFu;
  switch (variant & 0xFF) {
    case 0: return dispatch<4>(op, a, num_cus, cap, stream);
    case 1: return dispatch<2>(op, a, num_cus, cap, stream);
    case 2: return dispatch<8>(op, a, num_cus, cap, stream);
    case 3: return dispatch<4, 1>(op, a, num_cus, cap, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
