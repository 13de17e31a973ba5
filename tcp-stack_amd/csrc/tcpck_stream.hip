// tcpck_stream.hip -- the packed-layout "stream" kernel: every wave reads one
// contiguous, byte-balanced run of whole images as a single flat stream.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263 -- the
// sum of the image's LE u16 words mod 2^16, complemented (no carry fold).  That
// sum is a difference of prefix sums, sum(k) = P(start_{k+1}) - P(start_k)
// (mod 2^16), P(x) = word sum of the wave's run up to byte x, so the stream is
// never split per image:
//
//   * work split: wave w owns images [kb, ke): for a fixed stride kb = w*N/W;
//     for packed variable layouts the run is byte-balanced -- kb is the first
//     image starting at or after w/W of the batch's byte span, found by a
//     64-ary search over the offsets (one 64-lane probe per level, 4 levels
//     for 4M images); the wave validates its descriptors (packed:
//     off[k] + len[k] == off[k+1], len >= 16) and falls back to whole-wave
//     per-image summation when they are not;
//   * step s covers bytes [A0 + 1024 s, A0 + 1024 s + 1024): lane l reads the
//     16 B at 16 l with one global_load_dwordx4 (nt); U steps stay in flight
//     in a rolling register ring (the load for step s+U is issued as soon as
//     step s has been consumed), so a wave never drains its queue mid-run;
//   * per step the 64 lane sums are prefix-scanned with DPP (row_shr 1,2,4,8,
//     row_bcast 15/31) on top of a running carry (readlane 63);
//   * image boundaries (>= 16 B apart) are posted by the lanes that hold them
//     in the current batch of 64 boundary descriptors into a per-wave LDS slot
//     per 16-B chunk; the chunk's lane computes P(boundary) = carry +
//     exclusive scan + its words before the boundary, records it in a
//     128-entry LDS ring, and immediately emits the image that ends there:
//     ~(P(b_k) - P(b_{k-1})), stored as a 2-byte result (kFill: minus the
//     field word fetched with the descriptor batch, then written into bytes
//     28-29, tcp-header.h:177; kVerify: checksum == 0);
//   * only the first and last step of the run mask words (run edges).
// RFC 1071 mode is not served here (one's-complement prefix differences lose
// +0 / -0); the host routes it to the seg kernel.
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

constexpr uint32_t kRing = 128;

template <bool NT>
__device__ __forceinline__ u32x4 load16(const uint8_t *p) {
  if constexpr (NT) {
    return dev::load16_nt(p);
  } else {
    return *reinterpret_cast<const u32x4 *>(p);
  }
}

template <int OP>
__device__ __forceinline__ void emit(const SpanArgs &a, uint64_t k, uint32_t sum, uint8_t *field_ptr) {
  const uint16_t c = static_cast<uint16_t>(~sum);  // tcp-header.h:262
  if constexpr (OP == kVerify) {
    static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
  } else {
    if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
    if (OP == kFill && field_ptr) *reinterpret_cast<uint16_t *>(field_ptr) = c;
  }
}

// DIAG (timing experiments only; 2 and 3 produce wrong checksums):
//   0 = product, runs 16-B aligned; 1 = runs 128-B aligned (whole cache lines
//   per step); 2 = as 1 with boundary handling removed (stream + scan);
//   3 = as 1 with boundaries and scan removed (pure stream + per-lane sums).
template <int U, int OP, bool FIXED, bool NT, int DIAG = 0>
__global__ void __launch_bounds__(kBlock) stream_kernel(SpanArgs a) {
  __shared__ uint32_t s_slot[kWavesPerBlock][64];
  __shared__ uint32_t s_pb[kWavesPerBlock][kRing];   // P(start_k), ring by k
  __shared__ uint32_t s_pos[kWavesPerBlock][kRing];  // start_k - A0, ring by k
  __shared__ uint32_t s_fld[kWavesPerBlock][kRing];  // field word of image k (kFill)
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t *slot = s_slot[wv];
  uint32_t *pb = s_pb[wv];
  uint32_t *pos = s_pos[wv];
  uint32_t *fld = s_fld[wv];
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t w = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + wv;
  const uint64_t N = a.count;

  // ---- this wave's images [kb, ke) ----
  uint64_t kb, ke;
  if (FIXED) {
    kb = w * N / nw;
    ke = (w + 1) * N / nw;
  } else {
    const uint64_t first = a.offsets[0] - a.base;
    const uint64_t total = a.offsets[N - 1] - a.base + a.lengths[N - 1] - first;
    kb = w == 0 ? 0 : dev::find_first_ge(a.offsets, a.base, N, first + total / nw * w + (total % nw) * w / nw);
    ke = w + 1 == nw ? N
                     : dev::find_first_ge(a.offsets, a.base, N,
                                     first + total / nw * (w + 1) + (total % nw) * (w + 1) / nw);
  }
  if (kb >= ke) return;  // no block-level synchronisation below: waves may leave early

  auto start_of = [&](uint64_t k) -> uint64_t { return FIXED ? k * a.stride : a.offsets[k] - a.base; };
  auto len_of = [&](uint64_t k) -> uint32_t { return FIXED ? static_cast<uint32_t>(a.stride) : a.lengths[k]; };

  const uint64_t s0 = start_of(kb);
  const uint64_t s1 = start_of(ke - 1) + len_of(ke - 1);
  const uint64_t A0 = DIAG ? dev::align128_rel(a.arena, s0) : dev::align16_rel(a.arena, s0);

  if (!FIXED) {
    // validate the run: packed, every image >= 16 B, run shorter than 2^31 B
    bool bad = !(s1 > s0 && s1 - A0 < (uint64_t{1} << 31));
    for (uint64_t k0 = kb; k0 < ke && !bad; k0 += 64 * 4) {
      uint64_t o[4], on[4];
      uint32_t l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t k = k0 + 64 * u + lane;
        o[u] = k < ke ? a.offsets[k] : 0;
        l[u] = k < ke ? a.lengths[k] : 16;
        on[u] = k + 1 < ke ? a.offsets[k + 1] : o[u] + l[u];
      }
      bool b = false;
#pragma unroll
      for (int u = 0; u < 4; ++u) b |= (l[u] < 16) || (o[u] + l[u] != on[u]);
      bad = __ballot(b) != 0;
    }
    if (bad) {  // wave-uniform: exact per-image fallback
      for (uint64_t k = kb; k < ke; ++k) {
        const uint64_t st = start_of(k);
        const uint32_t ln = len_of(k);
        const uint32_t sum = dev::wave_image_sum<2, kRef>(a.arena, st, ln, OP == kFill && ln >= 30);
        if (lane == 0) {
          const uint16_t c = static_cast<uint16_t>(~sum);
          if constexpr (OP == kVerify) {
            static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
          } else {
            if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
            if (OP == kFill && ln >= 30) *reinterpret_cast<uint16_t *>(a.arena + st + 28) = c;
          }
        }
      }
      return;
    }
  }

  const uint32_t lead = static_cast<uint32_t>(s0 - A0);
  const uint32_t span = static_cast<uint32_t>(s1 - A0);
  const uint32_t nsteps = (span + 1023) >> 10;
  const uint32_t last_chunk = (span - 1) >> 4;
  const uint8_t *base = a.arena + A0;

  // ---- boundary batches: interior boundaries k = kb+1 .. ke-1, 64 per batch ----
  // Lane j of the current batch holds boundary kc + j as rb = start - A0 (~0u
  // past ke).  The next batch's raw descriptors are prefetched a whole batch
  // ahead and only turned into rb when the batch is activated, so the only
  // wait on them is at activation (once per 64 images), never per step.
  auto batch_raw = [&](uint64_t kc) -> uint64_t {  // raw descriptor load (variable layout)
    const uint64_t k = kc + lane;
    return (FIXED || k >= ke) ? 0 : a.offsets[k];
  };
  auto batch_rb = [&](uint64_t kc, uint64_t raw) -> uint32_t {
    const uint64_t k = kc + lane;
    if (k >= ke) return 0xFFFFFFFFu;
    return static_cast<uint32_t>((FIXED ? k * a.stride : raw - a.base) - A0);
  };
  auto batch_field = [&](uint64_t kc) -> uint32_t {  // field word of image kc + lane (kFill)
    const uint64_t k = kc + lane;
    if (OP != kFill || k >= ke || len_of(k) < 30) return 0;
    return *reinterpret_cast<const uint16_t *>(a.arena + start_of(k) + 28);
  };
  uint64_t kc = kb + 1;
  uint32_t rb = batch_rb(kc, batch_raw(kc));
  uint64_t nraw = batch_raw(kc + 64);      // prefetched next batch (not consumed until activation)
  uint32_t nfield = batch_field(kc + 64);
  if (OP == kFill) {
    const uint32_t f0 = batch_field(kb);  // image kb .. kb+63 fields (kb is not a routed boundary)
    if (kb + lane < ke) fld[(kb + lane) % kRing] = f0;
  }
  slot[lane] = 0;
  if (lane == 0) {
    pb[kb % kRing] = 0;
    pos[kb % kRing] = lead;
  }

  uint32_t carry = 0;
  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t ci = min((static_cast<uint32_t>(u) << 6) + lane, last_chunk);
    ring[u] = load16<NT>(base + 16 * static_cast<uint64_t>(ci));
  }

  // Steps past nsteps in the last unrolled group are harmless no-ops: their
  // words are masked (sb >= span), no boundary lies there, carry adds 0.  So the
  // unrolled body has no per-step condition and the ring refill stays in place
  // (a conditional refill made hipcc copy the freshly loaded slot, i.e. wait
  // vmcnt(0) every step).
  for (uint32_t s0i = 0; s0i < nsteps; s0i += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = s0i + u;
      {
        const uint32_t sb = st << 10;
        // post this step's boundaries (possibly from two consecutive batches)
        for (; DIAG < 2;) {
          if (rb - sb < 1024u) slot[(rb - sb) >> 4] = 0x80000000u | (static_cast<uint32_t>(kc + lane - kb) << 3) | ((rb & 15u) >> 1);
          const uint32_t last = dev::read_lane(rb, 63);  // largest rb of the batch (or ~0u)
          if (last == 0xFFFFFFFFu || last - sb >= 1024u) break;
          // whole batch posted: activate the next one (it may start in this step too)
          kc += 64;
          rb = batch_rb(kc, nraw);
          if (OP == kFill && kc + lane < ke) fld[(kc + lane) % kRing] = nfield;
          nraw = batch_raw(kc + 64);
          nfield = batch_field(kc + 64);
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t route = slot[lane];
        slot[lane] = 0;

        u32x4 wv4 = ring[u];
        const uint32_t crel = sb + (lane << 4);
        int32_t lo = 0;
        if (sb == 0 || sb + 1024 > span) {  // run edge (wave-uniform): mask words outside [lead, span)
          lo = min(max(static_cast<int32_t>(lead) - static_cast<int32_t>(crel), 0), 16);
          const int32_t hi = min(max(static_cast<int32_t>(span) - static_cast<int32_t>(crel), 0), 16);
          wv4 = dev::apply_mask(wv4, dev::word_mask(lo, hi));
        }
        // refill this ring slot with step st + U (clamped: never past the run)
        {
          const uint32_t ci = min(((st + U) << 6) + lane, last_chunk);
          ring[u] = load16<NT>(base + 16 * static_cast<uint64_t>(ci));
        }
        const uint32_t tot = dev::ref_chunk_sum(wv4);
        if (DIAG == 3) {
          carry += tot;
          continue;
        }
        const uint32_t incl = dev::wave_inclusive_scan(tot);
        if (DIAG < 2 && route) {
          const uint32_t r = (route & 7u) << 1;  // boundary byte offset inside the chunk
          const uint32_t head = dev::ref_chunk_sum(dev::apply_mask(wv4, dev::word_mask(lo, r)));
          const uint64_t k = kb + ((route >> 3) & 0x0FFFFFFFu);
          const uint32_t P = carry + (incl - tot) + head;
          pb[k % kRing] = P;
          pos[k % kRing] = crel + r;
          __builtin_amdgcn_wave_barrier();
          // image k-1 ends here
          const uint32_t km1 = static_cast<uint32_t>((k - 1) % kRing);
          const uint32_t p_prev = pb[km1];
          const uint32_t st_prev = pos[km1];
          const uint32_t f = OP == kFill ? fld[km1] : 0u;
          uint8_t *fp = (OP == kFill && crel + r - st_prev >= 30) ? const_cast<uint8_t *>(base) + st_prev + 28 : nullptr;
          emit<OP>(a, k - 1, P - p_prev - f, fp);
        }
        carry += dev::read_lane(incl, 63);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (DIAG >= 2) {  // keep the stream alive for timing; results are not checksums
    if (lane == 0 && a.out) static_cast<uint16_t *>(a.out)[kb] = static_cast<uint16_t>(carry);
    return;
  }
  if (lane == 0) {  // the last image ends at the end of the run
    const uint32_t km1 = static_cast<uint32_t>((ke - 1) % kRing);
    const uint32_t st_prev = pos[km1];
    const uint32_t f = OP == kFill ? fld[km1] : 0u;
    uint8_t *fp = (OP == kFill && span - st_prev >= 30) ? const_cast<uint8_t *>(base) + st_prev + 28 : nullptr;
    emit<OP>(a, ke - 1, carry - pb[km1] - f, fp);
  }
}

template <int U, int OP, bool FIXED, bool NT, int DIAG = 0>
hipError_t launch_one(const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(stream_kernel<U, OP, FIXED, NT, DIAG>);
  uint64_t blocks = static_cast<uint64_t>(per_cu) * num_cus;
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;  // >= 1 image per wave
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((stream_kernel<U, OP, FIXED, NT, DIAG>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                     stream, a);
  return hipGetLastError();
}

template <int U, bool NT>
hipError_t dispatch(int op, bool fixed, const SpanArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (op) {
    case kChecksum:
      return fixed ? launch_one<U, kChecksum, true, NT>(a, num_cus, s) : launch_one<U, kChecksum, false, NT>(a, num_cus, s);
    case kFill:
      return fixed ? launch_one<U, kFill, true, NT>(a, num_cus, s) : launch_one<U, kFill, false, NT>(a, num_cus, s);
    case kVerify:
      return fixed ? launch_one<U, kVerify, true, NT>(a, num_cus, s) : launch_one<U, kVerify, false, NT>(a, num_cus, s);
    default:
      return hipErrorInvalidValue;
  }
}

template <int U, int DIAG>
hipError_t launch_diag(int op, bool fixed, const SpanArgs &a, uint32_t num_cus, hipStream_t s) {
  if (op != kChecksum) return hipErrorInvalidValue;
  return fixed ? launch_one<U, kChecksum, true, true, DIAG>(a, num_cus, s)
               : launch_one<U, kChecksum, false, true, DIAG>(a, num_cus, s);
}

}  // namespace

// variant: 0 = default (U=4, nt), 1 = U=8 nt, 2 = U=4 plain loads, 3 = U=2 nt
hipError_t launch_stream(int op, bool fixed, int variant, const SpanArgs &a, uint32_t num_cus, hipStream_t stream) {
  switch (variant) {
    case 0: return dispatch<4, true>(op, fixed, a, num_cus, stream);
    case 1: return dispatch<8, true>(op, fixed, a, num_cus, stream);
    case 2: return dispatch<4, false>(op, fixed, a, num_cus, stream);
    case 3: return dispatch<2, true>(op, fixed, a, num_cus, stream);
    // timing experiments (fixed-stride checksum only): see DIAG above
    case 4: return launch_diag<4, 1>(op, fixed, a, num_cus, stream);
    case 5: return launch_diag<2, 1>(op, fixed, a, num_cus, stream);
    case 6: return launch_diag<4, 2>(op, fixed, a, num_cus, stream);
    case 7: return launch_diag<4, 3>(op, fixed, a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
