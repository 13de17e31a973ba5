// tcpck_rvstream.hip -- packed offset lists (C3) with rstream's scalar
// boundary walk: one contiguous run of whole images per wave, the image ends
// walked in SGPRs from the run's lengths.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  Packed images make the run one
// flat byte stream and sum(k) = P(end_k) - P(end_{k-1}) (mod 2^16), P the word
// sum of the run before byte x.
//
// Round 5, measured cold (every step on one of two identical batches): at
// C3's mean density (736 B) rstream's scalar walk streams 91.1 % of the roof
// where vvstream's per-step LDS prefix table streams 84.7 % (the same bytes as
// a fixed stride, scripts/cold_sweep.py, profiles/r05/cold_sweep_c3fixed.log).
// This kernel carries the walk to variable lengths:
//   * equal-count runs (the launcher's split, M x the resident grid), blocks
//     in XCD-chunked order, the run's first line read with the default policy
//     (the previous run's last line, found in L2 by its last step), every
//     other load nt; buffer loads with the step offset in an SGPR; v_dot2
//     chunk sums, DPP scan, carry from lane 63 -- all as rstream;
//   * the run's descriptors: offsets[kb], offsets[ke-1] and lengths[ke-1]
//     (scalar loads) give the span, then the data loads go out; the lengths
//     of images [64 i, 64 i + 64) of the run sit one per lane in a VGPR (one
//     coalesced load per 64 images, the next batch loaded a batch ahead) and
//     the walk reads the next one with v_readlane: nb += len(jn);
//   * at each boundary P = carry + scan(lane) - sum(lane) + the lane's words
//     before the byte (v_readlane), the image's sum P - P_prev staged in lane
//     k mod 64 of a VGPR, 64 results per store;
//   * a run whose lengths do not add up to its span (the PACKED hint wrong)
//     rewrites its results by the exact per-image pass (CHECKSUM / VERIFY
//     write only out[], so the check can wait for the walk's end).
// CHECKSUM and VERIFY, reference mode.
//
// Measured against vvstream (scripts/rvstream_probe.py, cold, profiles/r05/
// rvstream_probe*.log): C3 85.2 % at its best grid (U2, M 32) against 86.6 %,
// 1492-B images as an offset list 86.6 against 85.1 %, 639-B mean 75.7 vs
// 82.9 %, 159-B mean 28 vs 75 %.  Either kernel pays one descriptor round trip
// per run before its first data load, which the fixed-stride walk never does
// (rstream C2 92.3 %); the walk itself is not what costs.  Not AUTO's: the
// probe library only.
#include <map>
#include <mutex>
#include <utility>

#include "tcpck_device.h"

namespace tcpck {

#ifdef TCPCK_PROBE
namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

struct RVArgs {
  uint8_t *arena;
  const uint64_t *offsets;
  const uint32_t *lengths;
  uint64_t base;
  uint64_t count;
  void *out;               // u16 (CHECKSUM) or u8 (VERIFY)
  uint64_t per_wave, rem;  // equal-count split: count = per_wave * waves + rem
  uint32_t order;          // block order (dev::ordered_block)
  const uint64_t *table;   // variant 3: run r's byte span [table[r], table[r + 1]) (run_table_kernel)
};

// Variant 3 (probe): every run's start in one dense table, built by a pass
// before the stream, so a run's span comes from a line 16 runs share (in L2
// for most of them) instead of its own line of the offsets array.
__global__ void run_table_kernel(const uint64_t *offsets, const uint32_t *lengths, uint64_t base, uint64_t count,
                                 uint64_t per_wave, uint64_t rem, uint64_t runs, uint64_t *table) {
  const uint64_t r = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r > runs) return;
  const uint64_t end = offsets[count - 1] - base + lengths[count - 1];
  const uint64_t kb = r * per_wave + (r < rem ? r : rem);
  table[r] = kb < count ? offsets[kb] - base : end;
}

template <int U, int OP>
__global__ void __launch_bounds__(kBlock) rvstream_kernel(RVArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  uint64_t kb, ke;
  dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  if (kb >= ke) return;
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  // lengths of run images [64 i, 64 i + 64): lane l holds image 64 i + l's.  The
  // first batch depends only on kb: its load goes out with the offsets', before
  // the data loads (which wait for the run's start), so it is in when the walk begins
  const uint32_t *lens = a.lengths + kb;
  uint32_t vlen = lane < nimg ? lens[lane] : 0u;
  const uint64_t s0 = a.table ? a.table[wid] : a.offsets[kb] - a.base;
  const uint64_t s1 = a.table ? a.table[wid + 1] : a.offsets[ke - 1] - a.base + a.lengths[ke - 1];
  uint8_t *const arena = a.arena;
  const uint64_t A0 = dev::align128_rel(arena, s0);
  bool bad = !(s1 >= s0 && s1 - A0 < (uint64_t{1} << 31));

  auto store = [&](uint64_t k, uint16_t c) {
    if constexpr (OP == kVerify)
      static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
    else
      static_cast<uint16_t *>(a.out)[k] = c;
  };

  if (!bad) {
    const uint32_t lead = static_cast<uint32_t>(s0 - A0);
    const uint32_t span = static_cast<uint32_t>(s1 - A0);
    const uint32_t nsteps = (span + 1023) >> 10;
    const uint32_t last_chunk = span > 0 ? (span - 1) >> 4 : 0;
    const auto rsrc = dev::make_rsrc(arena + A0, (last_chunk + 1) << 4);

    // the run's first data loads go out first
    u32x4 ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u == 0 && lane < 8) {
        // the run's first line is the previous run's last: kept in L2 for its last step
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), 0, 0);
        ring[0] = u32x4{v.x, v.y, v.z, v.w};
      } else {
        ring[u] = dev::load16_buf_nt(rsrc, lane << 4, static_cast<uint32_t>(u) << 10);
      }
    }
    uint32_t vnext = lane + 64 < nimg ? lens[lane + 64] : 0u;
    {
      uint32_t nb = lead + dev::read_lane(vlen, 0);  // end of run image jn - 1
      uint32_t jn = 1;
      uint32_t carry = 0, p_last = 0;
      uint32_t stage = 0, out_rel = 0;  // results of run images out_rel .. out_rel + 63, lane-indexed
      auto flush = [&](uint32_t n) {
        if (lane < n) store(kb + out_rel + lane, static_cast<uint16_t>(stage));
      };
      auto emit = [&](uint32_t jr, uint32_t sum) {  // jr = run image index (wave-uniform)
        const uint32_t j = jr - out_rel;
        stage = lane == j ? static_cast<uint32_t>(dev::finish<kRef>(sum)) : stage;  // tcp-header.h:262
        if (j == 63) {
          flush(64);
          out_rel += 64;
        }
      };
      for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t st = g + u;  // steps past nsteps: masked to zero, no boundary, harmless
          const uint32_t sb = st << 10;
          u32x4 w = ring[u];
          if (sb == 0 || sb + 1024 > span) {  // run edge (wave-uniform): keep words of [lead, span) only
            const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
            const int32_t lo = min(max(static_cast<int32_t>(lead) - crel, 0), 16);
            const int32_t hi = min(max(static_cast<int32_t>(span) - crel, 0), 16);
            w = dev::apply_mask(w, dev::word_mask(lo, hi));
          }
          const uint32_t tot = dev::ref_chunk_sum_dot(w);
          const uint32_t incl = dev::wave_inclusive_scan(tot);
          while (nb < sb + 1024 && jn < nimg) {  // scalar: the image ends in this step
            const uint32_t rel = nb - sb;
            const uint32_t lb = rel >> 4;
            const uint32_t r = rel & 15u;
            uint32_t P = carry + dev::read_lane(incl, lb) - dev::read_lane(tot, lb);
            if (r)
              P += dev::words_before(r, dev::read_lane(w.x, lb), dev::read_lane(w.y, lb), dev::read_lane(w.z, lb),
                                     dev::read_lane(w.w, lb));
            emit(jn - 1, P - p_last);
            p_last = P;
            if ((jn & 63u) == 0) {  // the next 64 lengths; load the batch after them
              vlen = vnext;
              const uint32_t j2 = jn + 64 + lane;
              vnext = j2 < nimg ? lens[j2] : 0u;
            }
            nb += dev::read_lane(vlen, jn & 63u);
            ++jn;
          }
          carry += dev::read_lane(incl, 63);
          ring[u] = dev::load16_buf_nt(rsrc, lane << 4, (st + U) << 10);  // the slot's data is dead: refill
        }
      }
      // ends at the span not met in the loop (zero-length images at the run's
      // end when its last step is full): P there is the run's total
      for (; jn < nimg; ++jn) {
        emit(jn - 1, carry - p_last);
        p_last = carry;
        if ((jn & 63u) == 0) {
          vlen = vnext;
          const uint32_t j2 = jn + 64 + lane;
          vnext = j2 < nimg ? lens[j2] : 0u;
        }
        nb += dev::read_lane(vlen, jn & 63u);
      }
      emit(nimg - 1, carry - p_last);  // the last image ends at the run end
      if (nimg > out_rel) flush(nimg - out_rel);
      // the lengths must add up to the span (the PACKED contract): nb is now the
      // end of the run's last image by its lengths.  If they do not, the results
      // above are rewritten by the exact pass below (only out[] was written).
      bad = nb != span;
    }
  }
  if (bad) {  // wave-uniform: the layout is not the packed run the walk assumed -> exact per-image pass
    for (uint64_t k = kb; k < ke; ++k) {
      const uint64_t start = a.offsets[k] - a.base;
      const uint32_t sum = dev::wave_image_sum<2, kRef>(arena, start, a.lengths[k], false);
      if (lane == 0) store(k, dev::finish<kRef>(sum));
    }
  }
}

template <int U, int OP>
hipError_t launch_one(const RunArgs &s, uint32_t num_cus, hipStream_t stream, bool table = false) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(rvstream_kernel<U, OP>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  // M x the resident grid as rstream: the largest power of two keeping runs >= 4 KiB
  const uint64_t bytes = s.total_bytes ? s.total_bytes : s.count * 1024;
  uint64_t blocks = resident * dev::oversub_for(s.oversub, bytes, resident * kWavesPerBlock, 1024);
  const uint64_t need = (s.count + kWavesPerBlock - 1) / kWavesPerBlock;  // >= 1 image per wave
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  RVArgs a{};
  a.arena = s.arena;
  a.offsets = s.offsets;
  a.lengths = s.lengths;
  a.base = s.base;
  a.count = s.count;
  a.out = s.out;
  a.per_wave = s.count / (blocks * kWavesPerBlock);
  a.rem = s.count % (blocks * kWavesPerBlock);
  a.order = 4u;  // XCD-chunked: groups of 16 blocks per XCD
  if (table) {
    // (probe) one table buffer per device (a single process-wide
    // buffer was reused across devices and freed under concurrent callers),
    // grown as needed; the lock covers the growth and both launches, and a
    // growth first drains the device, so no launch still reads the old buffer
    static std::mutex mu;
    static std::map<int, std::pair<uint64_t *, uint64_t>> tables;  // device -> (buffer, entries)
    std::lock_guard<std::mutex> lk(mu);
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return hipGetLastError();
    auto &t = tables[device];
    const uint64_t runs = blocks * kWavesPerBlock;
    if (runs + 1 > t.second) {
      if (t.first) {
        (void)hipDeviceSynchronize();
        (void)hipFree(t.first);
      }
      t = {nullptr, 0};
      void *p = nullptr;
      if (hipMalloc(&p, (runs + 1) * 8) != hipSuccess) {
        (void)hipGetLastError();
        return hipErrorOutOfMemory;
      }
      t = {static_cast<uint64_t *>(p), runs + 1};
    }
    hipLaunchKernelGGL(run_table_kernel, dim3(static_cast<uint32_t>((runs + 256) / 256)), dim3(256), 0, stream,
                       s.offsets, s.lengths, s.base, s.count, a.per_wave, a.rem, runs, t.first);
    a.table = t.first;
    hipLaunchKernelGGL((rvstream_kernel<U, OP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((rvstream_kernel<U, OP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

}  // namespace
#endif

// variant: 0 = U4, 1 = U8, 2 = U2 (M by size, runs >= 4 KiB as rstream;
// param >> 16 = M).  The product library refuses it.
hipError_t launch_rvstream(int op, int variant, const RunArgs &a, uint32_t num_cus, hipStream_t stream) {
#ifdef TCPCK_PROBE
  if (a.count == 0) return hipSuccess;
  if (a.mode != kRef || !a.out || (op != kChecksum && op != kVerify)) return hipErrorInvalidValue;
  if (variant == 0)
    return op == kVerify ? launch_one<4, kVerify>(a, num_cus, stream) : launch_one<4, kChecksum>(a, num_cus, stream);
  if (variant == 1)
    return op == kVerify ? launch_one<8, kVerify>(a, num_cus, stream) : launch_one<8, kChecksum>(a, num_cus, stream);
  if (variant == 2)
    return op == kVerify ? launch_one<2, kVerify>(a, num_cus, stream) : launch_one<2, kChecksum>(a, num_cus, stream);
  if (variant == 3 || variant == 4)  // 0 / 2 with the run table (packed batches only: a run's end is the next's start)
    return variant == 3 ? (op == kVerify ? launch_one<4, kVerify>(a, num_cus, stream, true)
                                         : launch_one<4, kChecksum>(a, num_cus, stream, true))
                        : (op == kVerify ? launch_one<2, kVerify>(a, num_cus, stream, true)
                                         : launch_one<2, kChecksum>(a, num_cus, stream, true));
#else
  (void)op;
  (void)variant;
  (void)a;
  (void)num_cus;
  (void)stream;
#endif
  return hipErrorInvalidValue;
}

}  // namespace tcpck
