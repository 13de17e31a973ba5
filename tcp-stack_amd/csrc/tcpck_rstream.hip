// tcpck_rstream.hip -- fixed-stride packed batches (stride == image length):
// one contiguous run of whole images per wave, image boundaries walked in
// scalar registers.
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  Images are back to back at a
// fixed stride S, so sum(k) = P((k+1)S) - P(kS) (mod 2^16) where P(x) is the
// word sum of the wave's run before byte x: the run is read as one flat stream.
//
//   * wave w owns an equal share of the images (dev::count_split; the split is
//     computed by the launcher, no device division): one contiguous run per wave
//     (measured faster than interleaved tiles on this part), its start rounded
//     down to a 128-B line so that every 1 KiB step covers exactly eight whole
//     lines;
//   * lane l reads the 16 B at 1024 s + 16 l of step s; U steps stay in flight
//     in a register ring refilled at the end of each step (the slot's data is
//     dead by then, so the load lands in the same registers -- no copies, no
//     vmcnt(0) drains);
//   * per step: the lane's word sum, a 64-lane DPP inclusive scan, the step
//     total by readlane 63 -- the only per-step vector work;
//   * the next image boundary is wave-uniform (next = previous + S), so the
//     boundary walk is scalar: when it falls in this step, P(boundary) =
//     carry + scan(lane) - sum(lane) + the lane's words before the byte,
//     each read with v_readlane into SGPRs; the image that ends there gets
//     ~(P - P_prev), selected into lane (k mod 64) of a staging VGPR, and 64
//     results leave as one coalesced store;
//   * kFill reads each image's checksum word (bytes 28-29) as the stream
//     passes it (one v_readlane) and subtracts it from the image's sum, so the
//     results are the checksums of the zero-field images (exact in both modes:
//     the RFC 1071 prefix is an exact word sum); they go into bytes 28-29
//     (tcp-header.h:177); kVerify stores checksum == 0.
//     With FixedStreamArgs::defer_field, kFill writes only the results, and
//     launch_patch_fields (tcpck_header.hip) stores the fields afterwards,
//     one write-through 2-B store per image (AUTO's choice; FILL without a
//     results buffer uses the context's scratch for them).
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

// PRIO: 0 = default arbitration; 1 = s_setprio(wave slot / 2), 2 = s_setprio(1)
// for slots >= 4 -- the SIMD issues by priority, then age, so younger waves
// (higher slots) otherwise starve: identical runs took 105 us in slot 0 and
// 224 us in slot 7 of a C2 launch (scripts/stamps.py).
// FLAV bit 0: chunk sums with v_dot2_u32_u16; bit 1: buffer (SRSRC) loads with
// the step offset in an SGPR instead of per-lane 64-bit clamped addresses;
// bit 2 (with bit 1): the run's first step read with the default cache policy;
// bit 3 (with bit 1): every step read with the default cache policy;
// bit 5 (kFill, stride >= 128): each field's whole 64-B block written back
// from the stream's own registers with the checksum in place, write-through
// (sc0 sc1 nt) -- a whole-block store needs no read-modify-write of the line,
// a 2-B store does (scripts/fill_drain_probe.py, profiles/r03/fill_blind.log);
// bit 8 (probe, with bit 2): only the run's first LINE with the default
// policy, the rest of step 0 nt;
// bit 7 (kFill, probe): the chunks of each field's 64-B block read with the
// default cache policy (the rest nt), so a field pass after the stream finds
// the block in the caches (the memory-side Infinity Cache holds C2's 1M field
// lines: 128 MB) and can write it back whole without reading HBM;
// a.order (runtime): the block order, dev::ordered_block -- with the XCD
// orders each XCD streams compact regions instead of every eighth run
// (measured +4% at C2, profiles/DESIGN_history_r01-r04.md section 4; the HBM bytes do not change), and
// neighbouring runs share an XCD's L2 for the run-edge line (FLAV bit 2).
// MODE: kRef, or kRfc1071 -- the run's prefix P is an exact u32 running sum
// of its words, so P(end) - P(start) is an image's exact word sum (< 2^32 for
// images < 128 KiB) and RFC 1071 folds it like any other sum
template <int U, int OP, bool STAMP, int PRIO = 0, int FLAV = 0, int MODE = kRef>
__global__ void __launch_bounds__(kBlock) rstream_kernel(FixedStreamArgs a) {
  // SECT: the field blocks of the run's images, staged as the stream passes
  // them (image j in slot j mod 32) until 16 results are ready.  Fields are
  // >= 128 B apart: <= 15 staged and waiting + <= 9 staged per step < 32
  constexpr bool SECT = OP == kFill && (FLAV & 32) != 0;
  __shared__ u32x4 s_sec[kWavesPerBlock][SECT ? 32 * 4 : 1];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  // readfirstlane: the wave index is uniform, but hipcc cannot prove anything
  // derived from threadIdx is; without it every boundary variable below lives
  // in VGPRs and each uniform test becomes an exec-masked region
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock +
                       static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  uint64_t t_start = 0;
  if (STAMP) t_start = __builtin_amdgcn_s_memrealtime();
  if (PRIO) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t slot = hw & 0xFu;
    if (PRIO == 1) {
      if (slot >= 6) {
        __builtin_amdgcn_s_setprio(3);
      } else if (slot >= 4) {
        __builtin_amdgcn_s_setprio(2);
      } else if (slot >= 2) {
        __builtin_amdgcn_s_setprio(1);
      }
    } else if (slot >= 4) {
      __builtin_amdgcn_s_setprio(1);
    }
  }
  uint64_t kb, ke;
  dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  if (kb >= ke) return;
  const uint32_t S = static_cast<uint32_t>(a.stride);
  const uint64_t s0 = kb * S;
  const uint64_t A0 = dev::align128_rel(a.arena, s0);
  const uint32_t lead = static_cast<uint32_t>(s0 - A0);
  const uint32_t span = lead + static_cast<uint32_t>(ke - kb) * S;
  const uint32_t nsteps = (span + 1023) >> 10;
  const uint32_t last_chunk = (span - 1) >> 4;
  const uint8_t *base = a.arena + A0;

  // buffer flavour: records cover whole chunks of the run; steps past it read 0
  const auto rsrc = dev::make_rsrc(base, (last_chunk + 1) << 4);
  // FLAV bit 7: the next field whose block the load walk has not yet passed
  // (steps are loaded in order, so one scalar walker serves every load)
  uint32_t nl = lead + 28;
  auto load_step = [&](uint32_t st) -> u32x4 {
    if constexpr ((FLAV & 128) != 0 && OP == kFill) {
      const uint32_t sb = st << 10;
      uint64_t m = 0;  // lanes holding a chunk of a field block of this step
      while (nl < sb + 1024 && nl < span) {
        m |= uint64_t{0xF} << (((nl & ~63u) - sb) >> 4);  // blocks are 64-B aligned inside the 1-KiB step
        nl += S;
      }
      if ((m >> lane) & 1u) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), static_cast<int>(sb), 0);
        return u32x4{v.x, v.y, v.z, v.w};
      }
      return dev::load16_buf_nt(rsrc, lane << 4, sb);
    } else if constexpr (FLAV & 2) {
      if constexpr (FLAV & 8) {  // default cache policy for every step (FILL: the field's line stays in L2)
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), static_cast<int>(st << 10), 0);
        return u32x4{v.x, v.y, v.z, v.w};
      } else {
        return dev::load16_buf_nt(rsrc, lane << 4, st << 10);
      }
    } else {
      const uint32_t ci = min((st << 6) + lane, last_chunk);  // clamp: always a legal address
      return dev::load16_nt(base + 16 * static_cast<uint64_t>(ci));
    }
  };

  // wave-uniform boundary walk, all in 32-bit run-relative terms (SGPRs):
  // image jn of the run starts at byte nb (relative to A0)
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  uint32_t nb = lead + S;
  uint32_t jn = 1;
  uint32_t nf = lead + 28;  // kFill: next checksum field (image jf's, run-relative)
  uint32_t jf = 0;
  // kFill: image j's field word, parked in lane j mod 64 of fstage and
  // subtracted from the image's sum when its end is resolved -- the same
  // result as zeroing the field in the stream (socket-manager.cc:9: Checksum()
  // = 0 before the sum), without touching the data registers.  A step's
  // fields are read before its ends, but image j + 64's field lies past image
  // j's end by more than a step (images >= 30 B hold <= 35 fields per KiB),
  // so no slot is reused before it is consumed.
  uint32_t fstage = 0;
  uint32_t ns = lead + 28;  // SECT: the field whose block is being staged, of run image js
  uint32_t js = 0;
  // SECT + FLAV bit 6 (probe): a run of <= 32 images keeps every block in LDS
  // and stores them after its last load -- no store shares vmcnt with the ring
  const bool end_flush = SECT && (FLAV & 64) != 0 && nimg <= 32;
  uint32_t carry = 0;       // P at the step start
  uint32_t p_last = 0;      // P at the latest boundary (run start: 0)
  // results staged in lane (j - out_rel) until 64 are ready
  uint32_t stage = 0;
  uint32_t out_rel = 0;

  auto flush = [&](uint32_t n) {  // store staged results for run images out_rel .. out_rel + n - 1
    if (lane < n) {
      const uint64_t k = kb + out_rel + lane;
      const uint16_t c = static_cast<uint16_t>(stage);
      if constexpr (OP == kVerify) {
        static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
      } else {
        if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
        if (OP == kFill && !a.defer_field && !SECT) {
          if constexpr (FLAV & 16)  // write-through streaming store (sc0 sc1 nt): not left dirty in the MALL
            __builtin_amdgcn_raw_buffer_store_b16(c, rsrc, static_cast<int>((out_rel + lane) * S + lead + 28), 0, 19);
          else
            dev::store16_field(rsrc, (out_rel + lane) * S + lead + 28, c);  // tcp-header.h:177
        }
      }
    }
  };
  // SECT: the blocks of run images j0 .. j0 + n - 1 (n <= 16), four lanes per
  // block, each image's checksum from its staging lane
  auto flush_sect = [&](uint32_t j0, uint32_t n) {
    const uint32_t i = j0 + (lane >> 2), c = lane & 3u;
    // FLAV bit 9 (probe, SIDE): the blocks go to the dense side buffer instead
    // of in place -- 16 images' blocks are one contiguous KiB, one coalesced store
    const uint32_t cs = static_cast<uint32_t>(__shfl(static_cast<int>(stage), static_cast<int>((i - out_rel) & 63u), 64));
    if (lane < 4 * n) {
      const uint32_t f = lead + 28 + i * S;  // the field, run-relative
      const uint32_t b = f & ~63u;           // its block (A0 is 128-B aligned: so is the block in memory)
      const uint32_t o = f & 63u;
      u32x4 v = s_sec[wv][((i & 31u) << 2) | c];
      if ((o >> 4) == c) {  // the field's chunk: the checksum into bytes o, o + 1 (tcp-header.h:177)
        const uint32_t di = (o & 15u) >> 2;
        const uint32_t sh = (o & 2u) << 3;
        const uint32_t m = ~(0xFFFFu << sh), x = (cs & 0xFFFFu) << sh;
        v.x = di == 0 ? (v.x & m) | x : v.x;
        v.y = di == 1 ? (v.y & m) | x : v.y;
        v.z = di == 2 ? (v.z & m) | x : v.z;
        v.w = di == 3 ? (v.w & m) | x : v.w;
      }
      if constexpr ((FLAV & 512) != 0) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        v4u *dst = reinterpret_cast<v4u *>(a.side + (kb + i) * 64 + 16 * c);
        const v4u x{v.x, v.y, v.z, v.w};
        if (a.side_nt)
          __builtin_nontemporal_store(x, dst);
        else
          *dst = x;
        (void)b;
      } else if (static_cast<int64_t>(A0) + static_cast<int64_t>(b) >= 0) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, rsrc, static_cast<int>(b + 16 * c), 0, 19);
      } else if ((o >> 4) == c) {  // the block starts before the arena: the field alone
        dev::store16_field(rsrc, f, static_cast<uint16_t>(cs));
      }
    }
  };
  auto emit = [&](uint32_t jr, uint32_t sum) {  // jr = run-relative image index, sum = its word sum
    if constexpr (OP == kFill) sum -= dev::read_lane(fstage, jr & 63u);
    const uint32_t j = jr - out_rel;
    stage = lane == j ? static_cast<uint32_t>(dev::finish<MODE>(sum)) : stage;  // j, sum wave-uniform: v_cmp + v_cndmask
    if constexpr (SECT)
      if (!end_flush && (j & 15u) == 15u) flush_sect(jr - 15u, 16u);
    if (j == 63) {
      flush(64);
      out_rel += 64;
    }
  };

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (u == 0 && (FLAV & 6) == 6) {
      // step 0 with the default policy: its first line is the previous run's
      // last line; kept in L2 (nt lines go first), the neighbour's last step
      // can find it there instead of reading it from HBM a second time
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      if constexpr ((FLAV & 256) != 0) {
        // (probe) only that shared line (lanes 0-7) with the default policy, the
        // step's other 7 lines nt
        if (lane < 8) {
          const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), 0, 0);
          ring[0] = u32x4{v.x, v.y, v.z, v.w};
        } else {
          ring[0] = dev::load16_buf_nt(rsrc, lane << 4, 0);
        }
      } else {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<int>(lane << 4), 0, 0);
        ring[0] = u32x4{v.x, v.y, v.z, v.w};
      }
    } else {
      ring[u] = load_step(static_cast<uint32_t>(u));
    }
  }

  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = g + u;  // steps past nsteps: masked to zero, no boundary, harmless
      const uint32_t sb = st << 10;
      u32x4 w = ring[u];
      if constexpr (SECT) {  // the field blocks passing through this step, before the run-edge mask
        const uint32_t q = sb + (lane << 4);
        while (js < nimg) {
          const uint32_t b = ns & ~63u;
          if (b >= sb + 1024) break;
          if ((q & ~63u) == b) s_sec[wv][((js & 31u) << 2) | ((q >> 4) & 3u)] = w;
          if (b + 64 > sb + 1024) break;  // the block's other chunks come with the next step
          ns += S;
          ++js;
        }
      }
      if (sb == 0 || sb + 1024 > span) {  // run edge (wave-uniform): keep words of [lead, span) only
        const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
        const int32_t lo = min(max(static_cast<int32_t>(lead) - crel, 0), 16);
        const int32_t hi = min(max(static_cast<int32_t>(span) - crel, 0), 16);
        w = dev::apply_mask(w, dev::word_mask(lo, hi));
      }
      if constexpr (OP == kFill) {  // the checksum fields passing through this step: read, not zeroed
        while (nf < sb + 1024 && nf < span) {
          const uint32_t rel = nf - sb;
          const uint32_t lb = rel >> 4, wi = (rel & 15u) >> 1, di = wi >> 1;  // wave-uniform
          const uint32_t d = dev::read_lane(di == 0 ? w.x : (di == 1 ? w.y : (di == 2 ? w.z : w.w)), lb);
          const uint32_t fw = (wi & 1u) ? d >> 16 : d & 0xFFFFu;
          fstage = lane == (jf & 63u) ? fw : fstage;
          nf += S;
          ++jf;
        }
      }
      const uint32_t tot = (FLAV & 1) ? dev::ref_chunk_sum_dot(w) : dev::ref_chunk_sum(w);
      const uint32_t incl = dev::wave_inclusive_scan(tot);
      while (nb < sb + 1024 && jn < nimg) {  // scalar: boundaries in this step
        const uint32_t rel = nb - sb;
        const uint32_t lb = rel >> 4;
        const uint32_t r = rel & 15u;
        uint32_t P = carry + dev::read_lane(incl, lb) - dev::read_lane(tot, lb);
        if (r)
          P += dev::words_before<MODE == kRfc1071>(r, dev::read_lane(w.x, lb), dev::read_lane(w.y, lb), dev::read_lane(w.z, lb),
                            dev::read_lane(w.w, lb));
        emit(jn - 1, P - p_last);
        p_last = P;
        nb += S;
        ++jn;
      }
      carry += dev::read_lane(incl, 63);
      ring[u] = load_step(st + U);  // the slot's data is dead: refill in place
    }
  }
  emit(nimg - 1, carry - p_last);  // the last image ends at the run end
  if constexpr (SECT) {
    if (end_flush) {  // every block of the run after its last load
      for (uint32_t j0 = 0; j0 < nimg; j0 += 16) flush_sect(j0, min(nimg - j0, 16u));
    } else if (nimg & 15u) {
      flush_sect(nimg & ~15u, nimg & 15u);
    }
  }
  const uint32_t pending = nimg - out_rel;
  if (pending) flush(pending);
  if (STAMP && lane == 0 && a.dbg) {
    uint32_t hw_id, xcc_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    a.dbg[4 * wid] = t_start;
    a.dbg[4 * wid + 1] = __builtin_amdgcn_s_memrealtime();
    a.dbg[4 * wid + 2] = hw_id;
    a.dbg[4 * wid + 3] = xcc_id;
  }
}

template <int U, int OP, bool STAMP, int PRIO = 0, int FLAV = 0, int MODE = kRef>
hipError_t launch_one(const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(rstream_kernel<U, OP, STAMP, PRIO, FLAV, MODE>);
  const uint32_t cap = (a.blocks_per_cu && a.blocks_per_cu < per_cu) ? a.blocks_per_cu : per_cu;
  const uint64_t resident = static_cast<uint64_t>(cap) * num_cus;
  // runs of >= 4 KiB (4-8 KiB: C2 1M x 1492 B at 32x, C5 8M at 256x), up to 1024 x the resident grid
  uint64_t blocks = resident * dev::oversub_for(a.oversub, a.count * a.stride, resident * kWavesPerBlock, 1024);
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;  // >= 1 image per wave
  // images of >= 3.5 KiB that the policy's grid would give fewer than two per
  // wave: one each (at C2's size 4096 B: 1.46 per wave, runs of 4 or 8 KiB,
  // 89.3 % -> 91.2-91.9 % with one; 4000 B 91.3 -> 93.4 %; 3500 B 91.3 -> 92.0 %;
  // 3000 B keeps the policy: 3-KiB runs 87.6 %; scripts/pow2_probe.py,
  // scripts/run_len_probe.py, profiles/r03/pow2_probe.log, run_len_probe.log)
  if (!a.oversub && a.stride >= 3584 && a.count < 2 * blocks * kWavesPerBlock) blocks = need;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  FixedStreamArgs b = a;
  b.per_wave = a.count / (blocks * kWavesPerBlock);
  b.rem = a.count % (blocks * kWavesPerBlock);
  hipLaunchKernelGGL((rstream_kernel<U, OP, STAMP, PRIO, FLAV, MODE>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                     stream, b);
  return hipGetLastError();
}

template <int U, bool STAMP, int PRIO = 0, int FLAV = 0, int MODE = kRef>
hipError_t dispatch(int op, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum, STAMP, PRIO, FLAV, MODE>(a, num_cus, s);
    case kFill: return launch_one<U, kFill, STAMP, PRIO, FLAV, MODE>(a, num_cus, s);
    case kVerify: return launch_one<U, kVerify, STAMP, PRIO, FLAV, MODE>(a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_rstream(int op, int variant, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  // per-wave run must stay below 2^31 bytes (u32 run arithmetic)
  if (a.stride < 16 || a.count == 0) return hipErrorInvalidValue;
  const uint64_t max_run = ((a.count + 2047) / 2048 + 1) * a.stride + 128;
  if (max_run >= (uint64_t{1} << 31)) return hipErrorInvalidValue;
  if (a.mode != kRef) {  // RFC 1071: the policy's variant, images < 128 KiB (exact u32 sums)
    if (variant != 20 || a.stride >= (1u << 17)) return hipErrorInvalidValue;
    FixedStreamArgs b = a;
    b.order = 4u;
    return dispatch<4, false, 0, 263, kRfc1071>(op, b, num_cus, stream);
  }
  if (variant == 20) {
    // the policy (AUTO): U4, v_dot2 sums, buffer loads, XCD-chunked order, the
    // run's first line L2-kept.  Only that line: round 1-4 read the whole first
    // step with the default policy, and those 256 MB per C2 launch (1 KiB x
    // 256K runs) were found in the Infinity Cache by the next launch over the
    // same arena -- 93 % re-reading one arena, 91 % cold (two arenas in turn);
    // the shared line alone: 92.3 % either way (scripts/cold_sweep.py,
    // profiles/r05/cold_sweep_31.log; variant 32 keeps the whole step)
    FixedStreamArgs b = a;
    b.order = 4u;
    return dispatch<4, false, 0, 263>(op, b, num_cus, stream);
  }
#ifdef TCPCK_PROBE
  // measurement-only variants (libtcpck_probe.so): steps in flight, time
  // stamps, issue priorities, sum/load flavours and block orders
  switch (variant) {
    case 0: return dispatch<4, false>(op, a, num_cus, stream);
    case 1: return dispatch<2, false>(op, a, num_cus, stream);
    case 2: return dispatch<8, false>(op, a, num_cus, stream);
    case 3: return op == kChecksum ? launch_one<4, kChecksum, true>(a, num_cus, stream) : hipErrorInvalidValue;
    case 4: return dispatch<4, false, 1>(op, a, num_cus, stream);
    case 5: return dispatch<4, false, 2>(op, a, num_cus, stream);
    case 6: return dispatch<8, false, 1>(op, a, num_cus, stream);
    case 7: return op == kChecksum ? launch_one<4, kChecksum, true, 1>(a, num_cus, stream) : hipErrorInvalidValue;
    case 8: return dispatch<2, false, 1>(op, a, num_cus, stream);
    case 9: return dispatch<4, false, 0, 1>(op, a, num_cus, stream);
    case 10: return dispatch<4, false, 0, 3>(op, a, num_cus, stream);
    case 11: return dispatch<4, false, 0, 2>(op, a, num_cus, stream);
    case 12: return dispatch<2, false, 0, 3>(op, a, num_cus, stream);
    case 13: return dispatch<8, false, 0, 3>(op, a, num_cus, stream);
    case 21: {  // 14 with the first step read with the default policy (FLAV bit 2)
      FixedStreamArgs b = a;
      b.order = dev::kOrderXcd;
      return dispatch<4, false, 0, 7>(op, b, num_cus, stream);
    }
    case 22: {  // 20 with every step read with the default policy (FLAV bit 3)
      FixedStreamArgs b = a;
      b.order = 4u;
      return dispatch<4, false, 0, 11>(op, b, num_cus, stream);
    }
    case 27: {  // 20 with FILL's whole field blocks written from the stream (FLAV bit 5)
      if (a.stride < 128 || a.defer_field) return hipErrorInvalidValue;
      FixedStreamArgs b = a;
      b.order = 4u;
      return dispatch<4, false, 0, 39>(op, b, num_cus, stream);
    }
    case 28: {  // 27 with a short run's blocks stored after the run's last load (FLAV bit 6)
      if (a.stride < 128 || a.defer_field) return hipErrorInvalidValue;
      FixedStreamArgs b = a;
      b.order = 4u;
      return dispatch<4, false, 0, 103>(op, b, num_cus, stream);
    }
    case 33: case 34: {  // 20's FILL with each field's block (checksum in place) to the side buffer a.side
                         // (FLAV bits 5 + 9; 34: + bit 6, a short run's blocks after its last load), for
                         // launch_side_copy (tcpck_ex_probe.hip)
      if (op != kFill || a.stride < 128 || a.defer_field || !a.side) return hipErrorInvalidValue;
      FixedStreamArgs b = a;
      b.order = 4u;
      return variant == 33 ? launch_one<4, kFill, false, 0, 807>(b, num_cus, stream)
                           : launch_one<4, kFill, false, 0, 871>(b, num_cus, stream);
    }
    case 29: case 30: {  // FILL's deferred stream alone (a.defer_field): 29 with the field blocks read
                         // with the default policy (FLAV bit 7), 30 the policy's stream (timing)
      if (op != kFill || !a.defer_field || a.stride < 64) return hipErrorInvalidValue;
      FixedStreamArgs b = a;
      b.order = 4u;
      return variant == 29 ? launch_one<4, kFill, false, 0, 135>(b, num_cus, stream)
                           : launch_one<4, kFill, false, 0, 7>(b, num_cus, stream);
    }
    case 26: {  // 20 with the FILL field stores write-through streaming (sc0 sc1 nt, FLAV bit 4)
      FixedStreamArgs b = a;
      b.order = 4u;
      return dispatch<4, false, 0, 23>(op, b, num_cus, stream);
    }
    case 31: case 32: {  // 31: 20 (FLAV bit 8: only the run's first line with the default policy);
                         // 32: the policy before round 5, the whole first step with the default policy
      FixedStreamArgs b = a;
      b.order = 4u;
      return variant == 31 ? dispatch<4, false, 0, 263>(op, b, num_cus, stream)
                           : dispatch<4, false, 0, 7>(op, b, num_cus, stream);
    }
    case 23: case 24: {  // 20 with 8 (23) or 2 (24) steps in flight
      FixedStreamArgs b = a;
      b.order = 4u;
      return variant == 23 ? dispatch<8, false, 0, 7>(op, b, num_cus, stream)
                           : dispatch<2, false, 0, 7>(op, b, num_cus, stream);
    }
    case 14: case 15: case 16: case 17: case 18: case 19: {
      // 10 (14, 16-19) or 13 (15) with an XCD order: whole regions (14, 15) or
      // interleaved groups of 2, 4, 16, 64 blocks (16-19)
      FixedStreamArgs b = a;
      b.order = variant <= 15 ? dev::kOrderXcd : (variant == 16 ? 1u : (variant == 17 ? 2u : (variant == 18 ? 4u : 6u)));
      return variant == 15 ? dispatch<8, false, 0, 3>(op, b, num_cus, stream) : dispatch<4, false, 0, 3>(op, b, num_cus, stream);
    }
    default: break;
  }
#endif
  return hipErrorInvalidValue;
}

}  // namespace tcpck
