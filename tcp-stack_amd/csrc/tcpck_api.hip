// tcpck_api.hip -- the C-ABI of libtcpck.so (declared in include/tcpck.h).
//
// Replaces, for batches, the reference's per-packet checksum
// (filixi/TCP-stack include/tcp-header.h:252-263) at its call sites
// src/socket-manager.cc:9-10, include/socket-manager.h:259-260 (send: insert)
// and include/socket-manager.h:182 (receive: verify).  See include/tcpck.h.
//
// Ownership and threading: callers own every buffer; the hot
// batch calls allocate nothing and only enqueue work on the caller's stream;
// the current HIP device of the calling thread is saved and restored around
// every call (no hidden global device state).  The host-batch (end-to-end)
// calls use ctx-owned streams and staging and are serialised per ctx.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "tcpck.h"
#include "tcpck_tuning.h"
#include "tcpck_internal.h"
#include "tcpck_api_internal.h"

using tcpck::SegArgs;
using tcpck::api::DeviceGuard;
using tcpck::api::Hooks;
using tcpck::api::hip_status;

namespace tcpck {
namespace api {

int hip_status(hipError_t e) { return e == hipSuccess ? TCPCK_OK : TCPCK_EHIP - static_cast<int>(e); }

DeviceGuard::DeviceGuard(int device) {
  // A stale error left in the thread's last-error slot by an earlier failed
  // HIP call -- the caller's, or e.g. tcpck_device_supported(-1) -- would be
  // read back by the launchers' hipGetLastError() as this call's launch
  // status (found by tests/cpp/abi_host_test.cc): clear it first.
  (void)hipGetLastError();
  if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
  if (prev_ != device) ok_ = hipSetDevice(device);
}

DeviceGuard::~DeviceGuard() {
  if (prev_ >= 0) (void)hipSetDevice(prev_);
}

}  // namespace api
}  // namespace tcpck

namespace {

size_t out_elem(int op) { return op == TCPCK_OP_VERIFY ? 1 : 2; }

bool valid_op_mode(int op, int mode) {
  return (op == TCPCK_OP_CHECKSUM || op == TCPCK_OP_FILL || op == TCPCK_OP_VERIFY) &&
         (mode == TCPCK_MODE_REF || mode == TCPCK_MODE_RFC1071);
}
// device batches also take RECEIVE (VERIFY + TcpHeaderN2H)
bool valid_device_op_mode(int op, int mode) { return valid_op_mode(op == TCPCK_OP_RECEIVE ? TCPCK_OP_VERIFY : op, mode); }

// ---- host single-image path (product code, not the oracle) ---------------
// The exact sum of the image's LE u16 words is tcpck::host::word_sum
// (tcpck_host.cc: AVX2 where the CPU has it, else SWAR); REF needs it mod
// 2^16, RFC 1071 mod 0xFFFF with zero-ness.
uint16_t finish_host(uint64_t total, int mode) {
  if (mode == TCPCK_MODE_REF) return static_cast<uint16_t>(~total);  // tcp-header.h:262
  while (total >> 16) total = (total & 0xFFFF) + (total >> 16);
  return static_cast<uint16_t>(~total);
}

// Grows the host-batch staging buffers.  New buffers are allocated into
// temporaries and swapped in only when every allocation succeeded, so a failed
// (ENOMEM) request leaves the context's previous buffers and sizes intact and a
// later smaller request still runs on them.
int ensure_stage(tcpck_ctx *ctx, uint64_t bytes, uint64_t images) {
  if (!ctx->s[0]) {
    for (int i = 0; i < 2; ++i) {
      hipError_t e = hipStreamCreateWithFlags(&ctx->s[i], hipStreamNonBlocking);
      if (e != hipSuccess) return hip_status(e);
    }
  }
  if (bytes > ctx->stage_bytes) {
    if (bytes > UINT64_MAX - 16) return TCPCK_ENOMEM;
    uint8_t *fresh[2] = {nullptr, nullptr};
    for (int i = 0; i < 2; ++i) {
      if (hipMalloc(&fresh[i], bytes + 16) != hipSuccess) {
        for (int j = 0; j < 2; ++j)
          if (fresh[j]) (void)hipFree(fresh[j]);
        (void)hipGetLastError();  // clear the allocation error so the caller's next launch check is clean
        return TCPCK_ENOMEM;
      }
    }
    for (int i = 0; i < 2; ++i) {
      if (ctx->stage[i]) (void)hipFree(ctx->stage[i]);
      ctx->stage[i] = fresh[i];
    }
    ctx->stage_bytes = bytes;
  }
  if (images > ctx->stage_images) {
    if (images > UINT64_MAX / 8) return TCPCK_ENOMEM;
    void *fresh[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    const uint64_t size[3] = {images * 2, images * 8, images * 4};
    for (int i = 0; i < 2; ++i) {
      for (int k = 0; k < 3; ++k) {
        if (hipMalloc(&fresh[i][k], size[k]) != hipSuccess) {
          for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 3; ++b)
              if (fresh[a][b]) (void)hipFree(fresh[a][b]);
          (void)hipGetLastError();
          return TCPCK_ENOMEM;
        }
      }
    }
    for (int i = 0; i < 2; ++i) {
      if (ctx->stage_out[i]) (void)hipFree(ctx->stage_out[i]);
      if (ctx->stage_off[i]) (void)hipFree(ctx->stage_off[i]);
      if (ctx->stage_len[i]) (void)hipFree(ctx->stage_len[i]);
      ctx->stage_out[i] = static_cast<uint8_t *>(fresh[i][0]);
      ctx->stage_off[i] = static_cast<uint64_t *>(fresh[i][1]);
      ctx->stage_len[i] = static_cast<uint32_t *>(fresh[i][2]);
    }
    ctx->stage_images = images;
  }
  return TCPCK_OK;
}

void free_stage(tcpck_ctx *ctx) {
  for (auto &slot : ctx->scratch) {
    if (slot.ev) {
      (void)hipEventSynchronize(slot.ev);
      (void)hipEventDestroy(slot.ev);
    }
    if (slot.buf) (void)hipFree(slot.buf);
  }
  if (ctx->pipe) {
    (void)hipStreamSynchronize(ctx->pipe);
    (void)hipStreamDestroy(ctx->pipe);
  }
  for (auto &ev : ctx->pipe_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (ctx->probe_side) (void)hipFree(ctx->probe_side);
  if (ctx->side) {
    (void)hipEventDestroy(ctx->fork);
    (void)hipEventDestroy(ctx->join);
    (void)hipStreamDestroy(ctx->side);
  }
  for (int i = 0; i < 2; ++i) {
    if (ctx->stage[i]) (void)hipFree(ctx->stage[i]);
    if (ctx->stage_out[i]) (void)hipFree(ctx->stage_out[i]);
    if (ctx->stage_off[i]) (void)hipFree(ctx->stage_off[i]);
    if (ctx->stage_len[i]) (void)hipFree(ctx->stage_len[i]);
    if (ctx->s[i]) (void)hipStreamDestroy(ctx->s[i]);
  }
}

// ---- kernel selection (AUTO; measurements in profiles/DESIGN_history_r01-r04.md section 4) ------------
// reference mode:
//   fixed, stride == len   < 512 B vvstream (prefix table), 512 B..4 KiB
//                          rstream (scalar boundary walk), larger seg with
//                          W waves per image (~4 KiB per wave) where the
//                          image fills seg's steps, else rstream
//   fixed, stride > len    small gaps vvstream (gaps streamed as virtual
//                          images), larger gaps sstream (compacted slot
//                          stream) in slots of a multiple of 16 B, else seg
//                          with 8 lanes per image
//   packed variable        vvstream, every op
//   sorted variable        (TCPCK_LAYOUT_SORTED: receive slots) sstream for
//                          CHECKSUM / VERIFY
// everything else -- unordered offsets, gaps in variable layouts, RFC 1071
// mode, variable or gapped layouts of images above 16 KiB (where one wave per
// image already streams whole 1 KiB steps) -- seg.
constexpr uint64_t kRunMaxLen = 32768;       // packed variable layouts, typical image: above, seg
constexpr uint64_t kFixedRunMaxLen = 4096;   // packed fixed: rstream up to here; above, seg with W waves
                                             // per image where the image fills its steps (jumbo_on_seg;
                                             // C4 64 KiB: W16 91% vs rstream 85-88%, 6 KiB: W2 90.6% vs
                                             // 87.0%, profiles/r01/jumbo_probe.log), else rstream
// Policy parameters.  Every kernel takes its runs in the XCD-chunked block
// order (dev::ordered_block, groups of 16 blocks per XCD): each XCD streams
// compact regions instead of every eighth run (C2 86.3% -> 90.6%, C3 82.7 ->
// 84.1%, C4 85.5 -> 87.4%, profiles/r01/xcd_*.log; the HBM bytes do not
// change, PMC).  rstream also reads each run's first line with the default
// cache policy: that line is the previous run's last line, and the
// neighbour's last step then finds it in L2 (PMC bytes x1.015 -> x1.000;
// C2 90.9 -> 93.1% warm with the whole first step; since round 5 only the
// first line, 92.3% cold and warm), and large batches keep runs of 4-8 KiB with up to
// 1024 x the resident grid (C5: 256x, 84.7% at 32x -> 92.5%,
// profiles/r01/oversub_c5_first_step.log, split_probe.log); vvstream the
// same with runs >= 8 KiB (C3 86.3 -> 89.5%, profiles/r01/xcd_first_step_probe.log).
constexpr int kRstreamPolicy = 20;       // v_dot2 sums, buffer loads, XCD-chunked order, L2-kept first line
constexpr int kRstreamDeferFill = 25;    // FILL: kRstreamPolicy's stream to out, then the 2-B write-through field pass
constexpr int kVvPolicy = 4 | 8 | 16;    // size policy, XCD-chunked order, L2-kept first line
constexpr int kSegXcdOrder = 1 << 24;    // seg: XCD-chunked order
// seg W16 on packed jumbo images (C4): image k's chunk walk starts at 1-KiB
// step (29 k) mod 64 and wraps (SegArgs::rot), so the blocks in flight --
// consecutive images, 64 KiB apart -- read different offsets at the same time:
// C4 90.4 -> 92.7 % (multipliers = 1 mod 16 gain nothing, the other odd ones
// 91.8-92.9 %; W8 at 32 KiB loses 1-1.5 points, so W16 only;
// scripts/c4_rot_sweep.py, profiles/r03/c4_rot_sweep*.log)
constexpr int kSegW16Rot = 29;
// FILL of small images: nearly every line holds a checksum field, so the
// run kernels read every step with the default cache policy; the line is then
// still in L2 when the field store lands and leaves as a whole line instead of
// a masked partial write (scripts/keep_probe.py, profiles/r01/keep_probe.log:
// 96 B 20.4 -> 29.9 % of the roof, 192 B 28.6 -> 38.1 %, 320 B 38.0 -> 44.1 %,
// 480 B +0.6 %, the C3 mix -3.7 %: bytes per image up to 448)
constexpr uint64_t kFillKeepMaxLen = 448;
constexpr int kVvKeep = 32;              // vvstream: kFill reads with the default policy
constexpr int kVvDeferFill = 64;         // vvstream: kFill writes the results only, the field pass follows
// FILL with a results buffer on the run kernels: the stream writes only the
// results and the write-through field pass stores the fields, for (typical)
// images of at least this many bytes; smaller images pay more for 1M-per-
// 38-us scattered field stores than the in-stream stores cost them
constexpr uint64_t kDeferFillMinLen = 512;
// packed fixed images: vvstream's deferred form from 320 B up to 1 KiB, where
// it beats the in-stream forms and rstream's (round-4 re-check after the
// write-through field pass, scripts/fill_policy_sweep.py,
// profiles/r04/fill_policy_sweep.log, us per 1.5 GB: 320 B 448 -> 430, 384 B
// 427 -> 397, 448 B 408 -> 366, 512 B 347 (gstream) -> 328, 640 B 359
// (rstream 25) -> 322, 768 B 318 -> 308; 1 KiB stays on rstream 25: 279 vs 284)
constexpr uint64_t kVvDeferPackedMin = 320, kVvDeferPackedEnd = 1024;
constexpr int kSstreamDeferFill = 128;   // sstream: kFill writes the results only, the field pass follows
// variable layouts: vvstream's in-stream zeroing costs ~25 us per 1M images, so
// its deferred form pays only for larger images (C3's mean 732 B: 718 -> 702
// us; 256-1024 B: 700 -> 740 us; 1492 B: 365 -> 262 us; profiles/r03/fill_forms.log)
constexpr uint64_t kDeferFillMinVar = 1024;
constexpr int kSstreamHdrStream = 32;    // sstream RECEIVE: headers from the stream's registers
constexpr uint64_t kHdrStreamMaxLen = 256;  // ... for (typical) images up to this length
// RECEIVE: with an explicit kernel the product carries only the
// stream-register form (+ kSstreamHdrStream) and otherwise runs the header
// pass; the probe library can fuse the headers into any kernel that can
// (Hooks::fuse_any_hdr: sstream's after-the-verdicts conversion, HDR 1)

// Packed fixed images above 4 KiB: seg's W-wave shapes stream W KiB of an
// image per step (shape_for_len: W = 2, 4, 8, 16 up to 8, 16, 32, 64 KiB), so
// an image that ends early in its last step wastes the rest of that step --
// 9000 B on W4 reads as 3 x 4 KiB: 72 % of the roof against rstream's 90 %
// (profiles/r01/jumbo_fit_probe.log).  seg keeps the sizes it fills to >= 85 %
// (W16: only in four steps);
// FILL only from 24 KiB (below, rstream's batched field stores win even at a
// perfect fit: 8-24 KiB 77-81 % vs 82-84 %).
static bool jumbo_on_seg(int op, uint64_t len) {
  if (len > 65536) return true;
  const uint64_t step = len <= 8192 ? 2048 : (len <= 16384 ? 4096 : (len <= 32768 ? 8192 : 16384));
  const uint64_t steps = (len + step - 1) / step;
  const bool fits = 100 * len >= 85 * steps * step && (step < 16384 || steps == 4);  // W16: 48 KiB 81 vs 83 %
  return op == TCPCK_OP_FILL ? fits && len > 24576 : fits;
}

// The caller's TCPCK_PARAM_* bits, read before AUTO's choice rewrites param.
struct CallerBits {
  bool two_pass;   // RECEIVE: keep the separate header pass
  bool instream;   // FILL under AUTO: the field zeroed in the stream, no deferred field pass
  explicit CallerBits(int param)
      : two_pass((param & TCPCK_PARAM_RECEIVE_TWO_PASS) != 0), instream((param & TCPCK_PARAM_FILL_INSTREAM) != 0) {}
};

// FILL under AUTO with a results buffer on a fixed layout: whether AUTO's
// kernel takes its deferred form (the stream writes the results only, the
// write-through field pass stores them from the results; see run_fixed_impl).
bool fixed_fill_defers(int kernel, int param, uint64_t stride, uint32_t len) {
  switch (kernel) {
    case TCPCK_KERNEL_RSTREAM: return stride >= 30 && (param & 0xFF) == kRstreamPolicy;
    case TCPCK_KERNEL_SSTREAM: return len >= kDeferFillMinLen;
    case TCPCK_KERNEL_VVSTREAM: return len >= (stride == len ? kVvDeferPackedMin : kDeferFillMinLen);
    default: return false;
  }
}

// The same on an offset list (run_var_impl): vvstream from kDeferFillMinVar.
bool var_fill_defers(int kernel, uint64_t typical) {
  return kernel == TCPCK_KERNEL_VVSTREAM && typical >= kDeferFillMinVar;
}

// AUTO's kernel for a fixed layout: sets kernel (from TCPCK_KERNEL_AUTO) and
// its param (measurements in profiles/DESIGN_history_r01-r04.md section 4).
void pick_fixed(int op, int mode, const uint8_t *arena, uint64_t stride, uint32_t len, int &kernel, int &param) {
  if (mode == TCPCK_MODE_RFC1071 && stride == len && len >= 512 && len <= kFixedRunMaxLen) {
    // RFC 1071 on packed fixed images: rstream's prefix is an exact u32 word
    // sum, so its image differences fold like any sum (C2 in RFC 1071 mode at
    // the REF rate instead of seg's; profiles/r02/rfc_probe.log)
    kernel = TCPCK_KERNEL_RSTREAM;
    param = kRstreamPolicy;
  } else if (mode == TCPCK_MODE_RFC1071 && stride == len && len >= 2 && len < 512 &&
             (op != TCPCK_OP_FILL || len >= 30)) {
    // RFC 1071 on small packed images: vvstream's fixed mode with exact u32 prefix tables
    kernel = TCPCK_KERNEL_VVSTREAM;
    param = kVvPolicy;
  }
  if (kernel == TCPCK_KERNEL_AUTO) {
    // jumbo images in slots with small gaps (9000 B in 9216-B slots): vvstream
    // streams the gaps as virtual images, 86 % against seg's 70 % (FILL 78 vs
    // 64 %; profiles/r01/jumbo_layout_probe.log, jumbo_layout_fill_probe.log)
    const bool jumbo_hull = stride > len && len <= 65536 && 16 * stride <= 17 * static_cast<uint64_t>(len);
    // jumbo images in slots with larger gaps: the compacted slot stream where
    // the slot is a multiple of 16 B (9000 B in 16-KiB slots 74.2 -> 85.0 %,
    // FILL 65.6 -> 79.0 %, profiles/r02/slot_probe_ss3.log), else seg
    const bool jumbo_slots = stride > len && !jumbo_hull && tcpck::sstream_fixed_applies(stride, len) &&
                             (op != TCPCK_OP_FILL || len >= 30);
    // RFC 1071: slots with larger gaps (beyond vvstream's hull rule) on sstream
    // with exact u32 prefix tables; every other layout not routed above on seg
    const bool rfc_slots = mode == TCPCK_MODE_RFC1071 && stride > len && len < (1u << 17) &&
                           tcpck::sstream_fixed_applies(stride, len) && (op != TCPCK_OP_FILL || len >= 30);
    if (rfc_slots) {
      kernel = TCPCK_KERNEL_SSTREAM;
      param = 0;
    } else if (mode != TCPCK_MODE_REF || len < 2 ||
        (len > kFixedRunMaxLen && !jumbo_slots && (stride > len ? !jumbo_hull : jumbo_on_seg(op, len))) ||
        stride > (1u << 24)) {
      kernel = TCPCK_KERNEL_SEG;
      param = kSegXcdOrder;  // shape by length
      if (mode == TCPCK_MODE_REF && stride == len && len <= 65536 && op != TCPCK_OP_FILL &&
          tcpck::shape_for_len(len) == tcpck::kShapeW16)
        param |= kSegW16Rot << 8;
    } else if (stride > len) {
      // gapped fixed strides (e.g. MSS slots) (scripts/gap_probe.py,
      // profiles/r01/gap_probe.log): streaming the gaps with the images
      // (vvstream, virtual gap images) wins while they are small -- 128/96 B
      // 57% of the roof for image bytes vs seg's 39% -- else seg with 8 lanes
      // per image (1536/1492 B 81% vs 77% for the length-based shape)
      const uint64_t l = len;
      const bool hull = len < 512 ? stride <= 2 * l : (len < 1024 ? 4 * stride <= 5 * l : 16 * stride <= 17 * l);
      // (jumbo images reach here in slots: jumbo_hull -> vvstream, jumbo_slots -> sstream)
      if (hull && (op != TCPCK_OP_FILL || len >= 30)) {
        kernel = TCPCK_KERNEL_VVSTREAM;
        param = kVvPolicy | (op == TCPCK_OP_FILL && stride <= kFillKeepMaxLen ? kVvKeep : 0);
      } else if (tcpck::sstream_fixed_applies(stride, len) && (op != TCPCK_OP_FILL || len >= 30)) {
        // larger gaps in slots of a multiple of 16 B: the compacted slot stream
        // reads only the images' chunks (scripts/slot_probe.py,
        // profiles/r02/slot_probe_ss3.log, % of the roof in image bytes, seg ->
        // sstream): 1492 B in 2048-B slots 77.4 -> 83.1 % (FILL 57.7 -> 60.1),
        // in 4-KiB slots 65.7 -> 81.2 %, 96 in 256 B 39.9 -> 55.7 %
        kernel = TCPCK_KERNEL_SSTREAM;
        param = 0;
      } else {
        kernel = TCPCK_KERNEL_SEG;
        param = (tcpck::kShapeSmall + 1) | kSegXcdOrder;
      }
    } else if (op == TCPCK_OP_FILL && len <= 256 && tcpck::gstream_applies(arena, stride, len)) {
      // send-path FILL of power-of-two images, 32 B (pure ACKs) .. 256 B, and
      // of the other multiples of 16 B up to 240 B (512 B and 1 KiB: the
      // deferred-field forms since round 3's write-through field pass,
      // vvstream 328 vs 347 us and rstream 279 vs 299 us per 1.5 GB,
      // profiles/r04/fill_policy_sweep.log):
      // gstream; up to 256 B every line holds a checksum field, and reading
      // the lines with the default cache policy keeps them in L2 until the
      // field store lands, so they leave as whole lines rather than masked
      // partial writes (scripts/gstream_probe.py, profiles/r01/gstream_fill.log:
      // 32 B 21.4 -> 32 % of the roof, 256 B 33 -> 43 %, 512 B 46 -> 57 %).
      // Up to 128 B, writing every chunk back whole (twice the bytes, all of
      // them full-line writes) beats even that (profiles/r01/gstream_writeback.log:
      // 32 B 33.9 -> 41.3 %, 64 B 32.5 -> 40.2 %, 128 B 36.3 -> 40.3 %; 256 B
      // 44.7 vs 39.9 % keeps the default-policy loads).  The other multiples of
      // 16 B up to 240 B take the same rule (profiles/r01/gstream_np.log: 48 B
      // 29.0 -> 36.1 %, 96 B 29.7 -> 37.0 %; 144-240 B default-policy loads
      // 1-2 points ahead of vvstream FIXED)
      kernel = TCPCK_KERNEL_GSTREAM;
      param = len <= 128 ? tcpck::kGstreamWriteBack : (len <= 256 ? tcpck::kGstreamDefaultLoads : 0);
    } else if (len < 512 || (op == TCPCK_OP_FILL && len < kVvDeferPackedEnd)) {
      // (FILL up to 1 KiB stays here: from kVvDeferPackedMin on in vvstream's deferred form, run_fixed_impl)
      // packed, by image length (scripts/policy_sweep.py, profiles/r01/policy_small.log):
      // below 512 B boundaries are dense enough that resolving all of a step's
      // ends in parallel from the prefix table wins (vvstream FIXED, 80-81% at
      // 96-256 B, profiles/r01/fill_probe.log); from 512 B the scalar boundary
      // walk (rstream: 92-93% of the HBM roof on C2)
      kernel = (op == TCPCK_OP_FILL && len < 30) ? TCPCK_KERNEL_SEG : TCPCK_KERNEL_VVSTREAM;
      param = kernel == TCPCK_KERNEL_SEG ? kSegXcdOrder
                                         : kVvPolicy | (op == TCPCK_OP_FILL && len <= kFillKeepMaxLen ? kVvKeep : 0);
    } else {
      kernel = TCPCK_KERNEL_RSTREAM;
      param = kRstreamPolicy;
    }
  }
}

hipError_t run_fixed_impl(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, uint64_t stride, uint32_t len,
                          uint64_t count, void *out, int kernel, int param, hipStream_t s, bool *patch,
                          const Hooks &hk, uint8_t *hdr = nullptr, bool *hdr_done = nullptr) {
  const uint32_t num_cus = static_cast<uint32_t>(ctx->num_cus);
  const bool auto_pick = kernel == TCPCK_KERNEL_AUTO;
  const CallerBits caller(param);
  if (auto_pick) pick_fixed(op, mode, arena, stride, len, kernel, param);
  // RECEIVE into a header array: for small images in slots sstream emits each
  // host-order header from the stream's registers (one launch, the header
  // bytes read once); elsewhere the header pass follows the VERIFY pass, which
  // measured faster than any fused form for MSS-sized images (header stores
  // inside the read stream cost more than a separate pass: profiles/DESIGN_history_r01-r04.md "Receive
  // path", profiles/r03/receive_fused_probe.log)
  // (TCPCK_PARAM_RECEIVE_TWO_PASS keeps the separate pass, AUTO included)
  if (auto_pick && op == TCPCK_OP_RECEIVE && hdr && kernel == TCPCK_KERNEL_SSTREAM && len <= kHdrStreamMaxLen &&
      !caller.two_pass)
    param |= kSstreamHdrStream;
  const bool fuse_hdr = op == TCPCK_OP_RECEIVE && hdr && !caller.two_pass &&
                        ((hk.fuse_any_hdr && !auto_pick) || (param & kSstreamHdrStream));
  if (op == TCPCK_OP_RECEIVE) op = TCPCK_OP_VERIFY;  // the header pass follows (run_fixed)
  // FILL on rstream with a results buffer: the stream writes only the results,
  // then a second pass stores each field with a write-through 2-B store.
  // Scattered field stores inside a read stream, or left dirty in the
  // Infinity Cache for the next stream to write back, cost ~70 us per 1M
  // images; written through to HBM in their own pass they cost 38 us (C2:
  // 280 -> 248 us, scripts/fill_drain_probe.py, profiles/r03/fill_*.log)
  // (TCPCK_PARAM_FILL_INSTREAM keeps the in-stream form)
  const bool may_defer = auto_pick && !caller.instream && op == TCPCK_OP_FILL && out;
  if (may_defer && kernel == TCPCK_KERNEL_RSTREAM && fixed_fill_defers(kernel, param, stride, len))
    param = (param & ~0xFF) | kRstreamDeferFill;
  if (kernel == TCPCK_KERNEL_RSTREAM) {
    if (stride != len || len < 16 || len > (1u << 24)) return hipErrorInvalidValue;
    tcpck::FixedStreamArgs a{};
    a.mode = mode == TCPCK_MODE_REF ? tcpck::kRef : tcpck::kRfc1071;
    a.arena = arena;
    a.stride = stride;
    a.count = count;
    a.order = 0xFFu;  // default block order (variants 14-19 choose an XCD order)
    a.out = out;
    a.dbg = static_cast<uint64_t *>(ctx->dbg);  // set by the probe library only
    a.blocks_per_cu = static_cast<uint32_t>(param >> 8) & 0xFFu;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    int variant = param & 0xFF;
    if (variant == kRstreamDeferFill) {  // FILL: the policy's stream, the fields in a second pass
      if (op != TCPCK_OP_FILL || !out || stride < 30) return hipErrorInvalidValue;
      a.defer_field = 1;
      *patch = true;
      variant = kRstreamPolicy;
    }
    return tcpck::launch_rstream(op, variant, a, num_cus, s);
  }
  if (kernel == TCPCK_KERNEL_GSTREAM) {  // stride == len, a power of two in [32, 1024], 16-B aligned arena
    if (mode != TCPCK_MODE_REF || !tcpck::gstream_applies(arena, stride, len)) return hipErrorInvalidValue;
    tcpck::GroupStreamArgs a{};
    a.arena = arena;
    a.len = len;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    return tcpck::launch_gstream(op, param & 0xFFFF, a, num_cus, s);
  }
  if (kernel == TCPCK_KERNEL_SSTREAM) {  // fixed slots: stride % 16 == 0, stride >= len
    if (may_defer && fixed_fill_defers(kernel, param, stride, len)) param |= kSstreamDeferFill;
    if (param & kSstreamDeferFill) *patch = true;
    if (count == 1) stride = (static_cast<uint64_t>(len) + 15) & ~uint64_t{15};  // one image: never read
    if (!tcpck::sstream_fixed_applies(stride, len) || (op == TCPCK_OP_FILL && len < 30) ||
        (mode != TCPCK_MODE_REF && len >= (1u << 17)))
      return hipErrorInvalidValue;
    tcpck::RunArgs a{};
    a.mode = mode == TCPCK_MODE_REF ? tcpck::kRef : tcpck::kRfc1071;
    a.arena = arena;
    a.stride = stride;
    a.len = len;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    if (fuse_hdr) {
      a.hdr = hdr;
      *hdr_done = true;
    }
    return tcpck::launch_sstream(op, param & 0xFF, true, a, num_cus, s);
  }
  if (kernel == TCPCK_KERNEL_VVSTREAM) {  // any even length: the prefix table takes any number of ends per step
    if (len == 0 || stride > (1u << 24) || (op == TCPCK_OP_FILL && len < 30)) return hipErrorInvalidValue;
    if (may_defer && fixed_fill_defers(kernel, param, stride, len))
      param = (param & ~kVvKeep) | kVvDeferFill;  // (the default-policy reads served the in-stream stores)
    if (param & kVvDeferFill) *patch = true;
    if (mode != TCPCK_MODE_REF && (len >= (1u << 17) || (param & 32))) return hipErrorInvalidValue;
    tcpck::RunArgs a{};
    a.mode = mode == TCPCK_MODE_REF ? tcpck::kRef : tcpck::kRfc1071;
    a.arena = arena;
    a.stride = stride;
    a.len = len;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    a.blocks_per_cu = static_cast<uint32_t>(param >> 8) & 0xFFu;
    a.dbg = static_cast<uint64_t *>(ctx->dbg);  // set by the probe library only
    return tcpck::launch_vvstream(op, param & 0xFF, true, a, num_cus, s);
  }
  if (kernel != TCPCK_KERNEL_SEG) return hipErrorInvalidValue;
  SegArgs a{};
  a.arena = arena;
  a.stride = stride;
  a.len = len;
  a.count = count;
  a.out = out;
  a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
  a.order = ((param >> 24) & 1u) ? 4u : 0xFFu;  // bit 24: XCD-chunked order, groups of 16 blocks
  a.rot = static_cast<uint32_t>(param >> 8) & 0xFFu;  // bits 8-15: the W-wave shapes' rotation multiplier
  const auto shape = (param & 0xFF) > 0 ? static_cast<tcpck::SegShape>((param & 0xFF) - 1) : tcpck::shape_for_len(len);
  return tcpck::launch_seg(op, mode, true, shape, a, num_cus, s);
}

// RECEIVE = the VERIFY pass, then the header pass on the same stream (fusing
// the header work into rstream's stream measured no faster: profiles/DESIGN_history_r01-r04.md "Receive
// path").  hdr: host-order headers to hdr[32k, 32k + 32) instead of in place.
// FILL as CHECKSUM + field update (reference mode, a results buffer): the
// layout's CHECKSUM kernel at its full streaming rate, then the field pass
// derives each zero-field checksum from the old field, c = ~(~C - f) mod 2^16,
// and writes it through into the field and out[k].  Round 3 (the pass's stores
// written through, scripts/fill_defer_vv_probe.py, profiles/r03/fill_forms.log,
// % of the roof, in-stream -> update): packed variable batches on vvstream,
// whose in-stream field zeroing costs ~25 us per 1M images, gain most -- C3 53.7 ->
// 62.2 %, a 608/1492 mix 46.6 -> 69.2 %, 256-1024 B 48.3 -> 55.4 % -- so AUTO
// takes it there for typical images >= 448 B (below, vvstream's default-policy
// in-stream FILL); gapped fixed jumbo images keep it (9000 B in 9216-B slots
// 85.2 %); elsewhere the deferred-field form (the stream zeroes the fields and
// writes only the results, then the same pass stores them) ties with it or
// wins (C2 254 vs 258 us), and TCPCK_PARAM_FILL_UPDATE selects it.
constexpr uint64_t kFillUpdateMinVar = kFillKeepMaxLen;
bool fill_by_update(int op, int mode, const void *out, int kernel, int param, bool fixed, uint64_t stride,
                    uint32_t len, const tcpck_layout *layout = nullptr, uint64_t count = 0) {
  if (op != TCPCK_OP_FILL || mode != TCPCK_MODE_REF || !out) return false;
  if (param & TCPCK_PARAM_FILL_UPDATE) return true;
  if (kernel != TCPCK_KERNEL_AUTO || (param & TCPCK_PARAM_FILL_INSTREAM)) return false;
  if (fixed) return stride > len && len > 4096;
  const uint64_t typical = (layout && layout->total_bytes && count) ? layout->total_bytes / count : 0;
  return layout && (layout->flags & TCPCK_LAYOUT_PACKED) && typical >= kFillUpdateMinVar && typical <= kRunMaxLen;
}

// RECEIVE into a header array: whether the VERIFY kernel writes the headers
// itself (sstream's stream-register form) -- the same choice run_fixed_impl
// makes.  Otherwise the separate header pass runs FIRST: its one 128-B line
// per image (128 MB for 1M datagrams) is then still in the 256-MB Infinity
// Cache when the VERIFY stream reads the images, where after VERIFY it read
// every line from HBM again.  On a receive ring taken in turn with others (no
// step sees the previous step's lines) 158.1 -> 152.5 us per 1M datagrams of
// 96/608/1492 B in 2048-B slots (scripts/receive_ring_probe.py,
// profiles/r05/receive_ring_probe.log); the verdicts and headers are the same
// either way (the header array is not the arena).
bool fixed_receive_fuses(int mode, const uint8_t *arena, uint64_t stride, uint32_t len, int kernel, int param,
                         const Hooks &hk) {
  const bool auto_pick = kernel == TCPCK_KERNEL_AUTO;
  const CallerBits caller(param);
  int k = kernel, p = param;
  if (auto_pick) pick_fixed(TCPCK_OP_RECEIVE, mode, arena, stride, len, k, p);
  if (auto_pick && k == TCPCK_KERNEL_SSTREAM && len <= kHdrStreamMaxLen && !caller.two_pass) p |= kSstreamHdrStream;
  return k == TCPCK_KERNEL_SSTREAM && !caller.two_pass && ((hk.fuse_any_hdr && !auto_pick) || (p & kSstreamHdrStream));
}

void pick_var(int op, int mode, const tcpck_layout *layout, uint64_t count, bool hdr, bool two_pass, int &kernel,
              int &param, bool &fuse_small);

bool var_receive_fuses(int mode, const tcpck_layout *layout, uint64_t count, int kernel, int param, const Hooks &hk) {
  const bool auto_pick = kernel == TCPCK_KERNEL_AUTO;
  const CallerBits caller(param);
  int k = kernel, p = param;
  bool fuse_small = false;
  if (auto_pick) pick_var(TCPCK_OP_RECEIVE, mode, layout, count, true, caller.two_pass, k, p, fuse_small);
  return k == TCPCK_KERNEL_SSTREAM && !caller.two_pass &&
         ((hk.fuse_any_hdr && !auto_pick) || fuse_small || (p & kSstreamHdrStream));
}

// The header pass before VERIFY: under AUTO (whose choices are always valid),
// or with an explicit kernel in the probe library; with an explicit kernel the
// product runs it after VERIFY, so that a rejected kernel / param leaves the
// caller's header array untouched.
bool receive_hdr_first(int kernel, const Hooks &hk) {
  return !hk.hdr_after && (kernel == TCPCK_KERNEL_AUTO || hk.hdr_first_explicit);
}

// FILL's field pass on `s`, or -- pipelined FILL (fill_pipelined) -- on `ps`
// after the event `pev` recorded on `s` behind the stream pass it reads.
hipError_t launch_patch_on(const tcpck::PatchArgs &pa, uint32_t num_cus, hipStream_t s, hipStream_t ps,
                           hipEvent_t pev) {
  if (ps) {
    hipError_t e = hipEventRecord(pev, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(ps, pev, 0);
    if (e != hipSuccess) return e;
    s = ps;
  }
  return tcpck::launch_patch_fields(pa, num_cus, s);
}

hipError_t run_fixed_r(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, uint64_t stride, uint32_t len,
                       uint64_t count, void *out, int kernel, int param, hipStream_t s, uint8_t *hdr, const Hooks &hk,
                       hipStream_t ps = nullptr, hipEvent_t pev = nullptr) {
  bool patch = false;
  const auto ncu = static_cast<uint32_t>(ctx->num_cus);
  if (op == TCPCK_OP_RECEIVE && hdr && receive_hdr_first(kernel, hk) &&
      !fixed_receive_fuses(mode, arena, stride, len, kernel, param, hk)) {
    tcpck::HeaderArgs h{};  // the header pass first (fixed_receive_fuses), then VERIFY
    h.arena = arena;
    h.stride = stride;
    h.count = count;
    h.out = hdr;
    h.store_bits = hk.hdr_store_bits;
    const hipError_t eh = tcpck::launch_header_swap(h, static_cast<uint32_t>(ctx->num_cus), s);
    if (eh != hipSuccess) return eh;
    return run_fixed_impl(ctx, TCPCK_OP_VERIFY, mode, arena, stride, len, count, out, kernel, param, s, &patch, hk);
  }
  if (stride >= 30 && fill_by_update(op, mode, out, kernel, param, true, stride, len)) {
    const int p = param & ~(TCPCK_PARAM_FILL_UPDATE | TCPCK_PARAM_FILL_INSTREAM);
    const hipError_t e = run_fixed_impl(ctx, TCPCK_OP_CHECKSUM, mode, arena, stride, len, count, out, kernel, p, s,
                                        &patch, hk);
    if (e != hipSuccess) return e;
    tcpck::PatchArgs pa{};
    pa.arena = arena;
    pa.stride = stride;
    pa.count = count;
    pa.sums = static_cast<uint16_t *>(out);
    pa.lo = 0;
    pa.hi = (count - 1) * stride + len;
    pa.update = 1;
    pa.reverse = hk.patch_reverse ? 1u : 0u;
    return launch_patch_on(pa, ncu, s, ps, pev);
  }
  bool hdr_done = false;
  const hipError_t e =
      run_fixed_impl(ctx, op, mode, arena, stride, len, count, out, kernel, param, s, &patch, hk, hdr, &hdr_done);
  if (e != hipSuccess) return e;
  if (patch) {
    tcpck::PatchArgs p{};
    p.arena = arena;
    p.stride = stride;
    p.count = count;
    p.sums = static_cast<uint16_t *>(out);
    p.lo = 0;
    p.hi = (count - 1) * stride + len;
    p.reverse = hk.patch_reverse ? 1u : 0u;
    return launch_patch_on(p, ncu, s, ps, pev);
  }
  if (op != TCPCK_OP_RECEIVE || hdr_done) return e;
  tcpck::HeaderArgs h{};
  h.arena = arena;
  h.stride = stride;
  h.count = count;
  h.out = hdr;
  h.store_bits = hk.hdr_store_bits;
  return tcpck::launch_header_swap(h, static_cast<uint32_t>(ctx->num_cus), s);
}

// AUTO's kernel for an offset list: sets kernel (from TCPCK_KERNEL_AUTO) and
// its param; fuse_small: RECEIVE into a header array on a ring of small
// datagrams, the headers from sstream's registers (below).
void pick_var(int op, int mode, const tcpck_layout *layout, uint64_t count, bool hdr, bool two_pass, int &kernel,
              int &param, bool &fuse_small) {
  const uint64_t typical = (layout && layout->total_bytes) ? layout->total_bytes / count : 1500;
  const bool packed = mode == TCPCK_MODE_REF && layout && (layout->flags & TCPCK_LAYOUT_PACKED);
  // packed, reference mode: vvstream for every op (any image lengths; C3 89.1%
  // at 32x oversubscription, profiles/r01/c3_bench_r01_final.log).  The
  // packed flag must be true when set (tcpck.h); a wave whose lengths do not
  // add up to its span falls back to per-image sums, but that check cannot see
  // a gap that an overlap elsewhere in the run cancels
  if (kernel == TCPCK_KERNEL_AUTO) {
    // packed jumbo batches stay on vvstream up to a typical image of 32 KiB
    // (20000 B 86 % vs seg 76 %, FILL 82 vs 71 %; a 9000/20000/40000 mix 83
    // vs 72 %, FILL 79 vs 66 %), seg above (a 40000/60032 mix: 83.5 vs 82 %,
    // FILL 83 vs 79 %; profiles/r01/jumbo_layout_probe.log, jumbo_layout_fill_probe.log)
    const bool rfc_packed = mode == TCPCK_MODE_RFC1071 && layout && (layout->flags & TCPCK_LAYOUT_PACKED) &&
                            typical <= kRunMaxLen && layout->max_len != 0 && layout->max_len < (1u << 17) &&
                            (op != TCPCK_OP_FILL || (layout->min_len != 0 && layout->min_len >= 30));
    if (rfc_packed) {
      // RFC 1071 on packed variable layouts: vvstream with exact u32 prefix
      // tables (C3 in RFC 1071 mode, profiles/r02/rfc_probe.log)
      kernel = TCPCK_KERNEL_VVSTREAM;
      param = kVvPolicy;
    } else if (!packed && typical <= kRunMaxLen && op != TCPCK_OP_FILL && layout &&
               (layout->flags & TCPCK_LAYOUT_SORTED) &&
               (mode == TCPCK_MODE_REF || (layout->max_len != 0 && layout->max_len < (1u << 17)))) {
      // (RFC 1071 too, with exact u32 prefix tables, when every image is below 128 KiB)
      // images in order with gaps (receive slots): the compacted slot stream
      // (profiles/r02/slot_probe_ss3.log, seg -> sstream, CHECKSUM): a
      // 96/608/1492 mix in 2048-B slots 60.5 -> 70.3 %, in 1536-B slots 57.4
      // -> 68.5 %, 1492 B in 2048-B slots 73.5 -> 78.3 %; FILL stays on seg
      // (41-58 % either way: the scattered field writes bound it)
      kernel = TCPCK_KERNEL_SSTREAM;
      param = 0;
      if (op == TCPCK_OP_RECEIVE && hdr && typical <= kHdrStreamMaxLen && !two_pass) {
        fuse_small = true;
        param = kSstreamHdrStream;
      }
    } else if (!packed || typical > kRunMaxLen ||
               (op == TCPCK_OP_FILL && layout->min_len != 0 && layout->min_len < 30)) {
      kernel = TCPCK_KERNEL_SEG;
      param = kSegXcdOrder;
    } else {
      kernel = TCPCK_KERNEL_VVSTREAM;
      param = kVvPolicy | (op == TCPCK_OP_FILL && typical <= kFillKeepMaxLen ? kVvKeep : 0);
    }
  }
}

hipError_t run_var_impl(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, const uint64_t *off, const uint32_t *len,
                        uint64_t base, uint64_t count, void *out, const tcpck_layout *layout, int kernel, int param,
                        hipStream_t s, const Hooks &hk, uint8_t *hdr = nullptr, bool *hdr_done = nullptr,
                        bool *patch = nullptr) {
  const uint64_t typical = (layout && layout->total_bytes) ? layout->total_bytes / count : 1500;
  bool fuse_small = false;  // RECEIVE into a header array on a ring of small datagrams (pick_var)
  const bool auto_pick = kernel == TCPCK_KERNEL_AUTO;
  const CallerBits caller(param);
  if (auto_pick) pick_var(op, mode, layout, count, hdr != nullptr, caller.two_pass, kernel, param, fuse_small);
  // RECEIVE into a header array (as run_fixed_impl): on rings of small images
  // sstream emits the headers from its stream (4M 32-254-B datagrams in 256-B
  // slots: 190 us against 259 with the header pass, 235 with the run's
  // headers re-read after its verdicts); otherwise the header pass follows
  bool fuse_hdr = op == TCPCK_OP_RECEIVE && hdr && !caller.two_pass &&
                  ((hk.fuse_any_hdr && !auto_pick) || fuse_small || (param & kSstreamHdrStream));
  if (op == TCPCK_OP_RECEIVE) op = TCPCK_OP_VERIFY;  // the header pass follows (run_var)
  if (kernel == TCPCK_KERNEL_VVSTREAM) {
    if (mode != TCPCK_MODE_REF && (param & 32)) return hipErrorInvalidValue;
    // (REF packed batches of typical >= 448 B take the update form in run_var)
    if (auto_pick && !caller.instream && op == TCPCK_OP_FILL && out && patch && var_fill_defers(kernel, typical))
      param |= kVvDeferFill;
    if (param & kVvDeferFill) {
      if (!patch) return hipErrorInvalidValue;
      *patch = true;
    }
    tcpck::RunArgs a{};
    a.mode = mode == TCPCK_MODE_REF ? tcpck::kRef : tcpck::kRfc1071;
    a.arena = arena;
    a.offsets = off;
    a.lengths = len;
    a.base = base;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    a.total_bytes = layout ? layout->total_bytes : 0;
    a.blocks_per_cu = static_cast<uint32_t>(param >> 8) & 0xFFu;
    a.dbg = static_cast<uint64_t *>(ctx->dbg);  // set by the probe library only
    return tcpck::launch_vvstream(op, param & 0xFF, false, a, static_cast<uint32_t>(ctx->num_cus), s);
  }
  if (kernel == TCPCK_KERNEL_RVSTREAM) {  // packed offset lists, REF, CHECKSUM / VERIFY
    if (mode != TCPCK_MODE_REF || op == TCPCK_OP_FILL || !out) return hipErrorInvalidValue;
    tcpck::RunArgs a{};
    a.mode = tcpck::kRef;
    a.arena = arena;
    a.offsets = off;
    a.lengths = len;
    a.base = base;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    a.total_bytes = layout ? layout->total_bytes : 0;
    return tcpck::launch_rvstream(op, param & 0xFF, a, static_cast<uint32_t>(ctx->num_cus), s);
  }
  if (kernel == TCPCK_KERNEL_SSTREAM) {  // any offset list (runs of <= 128 images)
    if (param & kSstreamDeferFill) {
      if (!patch) return hipErrorInvalidValue;
      *patch = true;
    }
    tcpck::RunArgs a{};
    a.mode = mode == TCPCK_MODE_REF ? tcpck::kRef : tcpck::kRfc1071;
    a.arena = arena;
    a.offsets = off;
    a.lengths = len;
    a.base = base;
    a.count = count;
    a.out = out;
    a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
    a.total_bytes = layout ? layout->total_bytes : 0;
    if (fuse_hdr) {
      a.hdr = hdr;
      *hdr_done = true;
    }
    return tcpck::launch_sstream(op, param & 0xFF, false, a, static_cast<uint32_t>(ctx->num_cus), s);
  }
  if (kernel != TCPCK_KERNEL_SEG) return hipErrorInvalidValue;
  SegArgs a{};
  a.arena = arena;
  a.offsets = off;
  a.lengths = len;
  a.base = base;
  a.count = count;
  a.out = out;
  a.oversub = static_cast<uint32_t>(param >> 16) & 0xFFu;
  a.order = ((param >> 24) & 1u) ? 4u : 0xFFu;  // bit 24: XCD-chunked order, groups of 16 blocks
  const auto shape = (param & 0xFF) > 0 ? static_cast<tcpck::SegShape>((param & 0xFF) - 1) : tcpck::shape_for_len(typical);
  return tcpck::launch_seg(op, mode, false, shape, a, static_cast<uint32_t>(ctx->num_cus), s);
}

hipError_t run_var_r(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, const uint64_t *off, const uint32_t *len,
                     uint64_t base, uint64_t count, void *out, const tcpck_layout *layout, int kernel, int param,
                     hipStream_t s, uint8_t *hdr, const Hooks &hk, hipStream_t ps = nullptr,
                     hipEvent_t pev = nullptr) {
  const auto ncu = static_cast<uint32_t>(ctx->num_cus);
  if (op == TCPCK_OP_RECEIVE && base != 0) return hipErrorInvalidValue;  // device batches only
  if (fill_by_update(op, mode, out, kernel, param, false, 0, 0, layout, count)) {
    const int p = param & ~(TCPCK_PARAM_FILL_UPDATE | TCPCK_PARAM_FILL_INSTREAM);
    const hipError_t e =
        run_var_impl(ctx, TCPCK_OP_CHECKSUM, mode, arena, off, len, base, count, out, layout, kernel, p, s, hk);
    if (e != hipSuccess) return e;
    tcpck::PatchArgs pa{};
    pa.arena = arena;
    pa.offsets = off;
    pa.lengths = len;
    pa.base = base;
    pa.count = count;
    pa.sums = static_cast<uint16_t *>(out);
    pa.update = 1;
    pa.reverse = hk.patch_reverse ? 1u : 0u;
    pa.packed = (layout && (layout->flags & TCPCK_LAYOUT_PACKED)) ? 1u : 0u;
    return launch_patch_on(pa, ncu, s, ps, pev);
  }
  tcpck::HeaderArgs h{};
  h.arena = arena;
  h.offsets = off;
  h.count = count;
  h.out = hdr;
  h.store_bits = hk.hdr_store_bits;
  if (op == TCPCK_OP_RECEIVE && hdr && receive_hdr_first(kernel, hk) &&
      !var_receive_fuses(mode, layout, count, kernel, param, hk)) {
    // the header pass first, then VERIFY (fixed_receive_fuses)
    const hipError_t eh = tcpck::launch_header_swap(h, static_cast<uint32_t>(ctx->num_cus), s);
    if (eh != hipSuccess) return eh;
    return run_var_impl(ctx, TCPCK_OP_VERIFY, mode, arena, off, len, base, count, out, layout, kernel,
                        param & ~TCPCK_PARAM_RECEIVE_TWO_PASS, s, hk);
  }
  bool hdr_done = false, patch = false;
  const hipError_t e = run_var_impl(ctx, op, mode, arena, off, len, base, count, out, layout, kernel, param, s, hk,
                                    hdr, &hdr_done, &patch);
  if (e != hipSuccess) return e;
  if (patch) {  // the fields the stream left: write-through 2-B stores (launch_patch_fields)
    tcpck::PatchArgs pa{};
    pa.arena = arena;
    pa.offsets = off;
    pa.lengths = len;
    pa.base = base;
    pa.count = count;
    pa.sums = static_cast<uint16_t *>(out);
    pa.reverse = hk.patch_reverse ? 1u : 0u;
    return launch_patch_on(pa, ncu, s, ps, pev);
  }
  if (op != TCPCK_OP_RECEIVE || hdr_done) return e;
  return tcpck::launch_header_swap(h, ncu, s);
}

// A sub-range of an offset-list batch keeps the flags and the length bounds,
// and its byte hint scales with its image count, so its typical image -- the
// quantity AUTO chooses by -- is the whole batch's and every chunk runs the
// same form (tcpck_tuning.h).
tcpck_layout sub_layout(const tcpck_layout &layout, uint64_t n, uint64_t count) {
  tcpck_layout sub = layout;
  sub.total_bytes = static_cast<uint64_t>(static_cast<unsigned __int128>(layout.total_bytes) * n / count);
  return sub;
}

// Patches bytes 28-29 of host images after a FILL computed on the device
// (the device filled its staging copy; the host image is the caller's).
void patch_fields(uint8_t *arena, uint64_t k0, uint64_t n, const uint16_t *res,
                  const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t flen) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t o = off ? off[k0 + k] : (k0 + k) * stride;
    const uint32_t l = len ? len[k0 + k] : flen;
    if (l >= 30) std::memcpy(arena + o + 28, &res[k], 2);
  }
}

}  // namespace

// ---- the router's entry points (tcpck_api_internal.h) -------------------------
namespace tcpck {
namespace api {

hipError_t run_fixed(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, uint64_t stride, uint32_t len, uint64_t count,
                     void *out, int kernel, int param, hipStream_t s, uint8_t *hdr, const Hooks &hk) {
  return run_fixed_r(ctx, op, mode, arena, stride, len, count, out, kernel, param, s, hdr, hk);
}

hipError_t run_var(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, const uint64_t *off, const uint32_t *len,
                   uint64_t base, uint64_t count, void *out, const tcpck_layout *layout, int kernel, int param,
                   hipStream_t s, uint8_t *hdr, const Hooks &hk) {
  return run_var_r(ctx, op, mode, arena, off, len, base, count, out, layout, kernel, param, s, hdr, hk);
}

namespace {

// FILL without a results buffer under AUTO (the reference's call shape,
// socket-manager.cc:9-10): when AUTO's form for the layout reads the results
// back -- rstream's and vvstream's deferred fields, the update pass (C2
// in-stream 69.3 % -> 76-77 %, C3 53.7 -> 62 %, profiles/r03/fill_forms.log)
// -- the results go to a ctx scratch slot; every other form (gstream, seg,
// the in-stream run forms) launches with out = NULL and takes no slot.
bool fill_reads_results_fixed(int mode, const uint8_t *arena, uint64_t stride, uint32_t len, int param) {
  if (param & TCPCK_PARAM_FILL_INSTREAM) return false;
  const int dummy = 0;
  if (stride >= 30 && fill_by_update(TCPCK_OP_FILL, mode, &dummy, TCPCK_KERNEL_AUTO, param, true, stride, len))
    return true;
  int k = TCPCK_KERNEL_AUTO, p = param;
  pick_fixed(TCPCK_OP_FILL, mode, arena, stride, len, k, p);
  return fixed_fill_defers(k, p, stride, len);
}

bool fill_reads_results_var(int mode, const tcpck_layout *layout, uint64_t count, int param) {
  if (param & TCPCK_PARAM_FILL_INSTREAM) return false;
  const int dummy = 0;
  if (fill_by_update(TCPCK_OP_FILL, mode, &dummy, TCPCK_KERNEL_AUTO, param, false, 0, 0, layout, count)) return true;
  int k = TCPCK_KERNEL_AUTO, p = param;
  bool fuse_small = false;
  pick_var(TCPCK_OP_FILL, mode, layout, count, false, false, k, p, fuse_small);
  const uint64_t typical = (layout && layout->total_bytes) ? layout->total_bytes / count : 1500;
  return var_fill_defers(k, typical);
}

// A scratch slot for one out-less FILL, its mutex held (nullptr: none, the
// caller runs the in-stream form).  None while `s` is under stream capture:
// a captured event record would order later uncaptured FILLs against a graph
// node, and a replayed graph would share the slot with no ordering at all.
tcpck_ctx::ScratchSlot *take_scratch(tcpck_ctx *ctx, hipStream_t s, std::unique_lock<std::mutex> &held) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (cs != hipStreamCaptureStatusNone) return nullptr;
  constexpr int n = tcpck_ctx::kScratchSlots;
  int pick = -1;
  {
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    ++ctx->scratch_calls;
    if (!ctx->scratch[0].buf) {  // first use (or a retry after a refusal): every slot, or none
      if (ctx->scratch_calls < ctx->scratch_retry_at) return nullptr;
      for (auto &slot : ctx->scratch) {
        void *p = nullptr;
        hipEvent_t ev = nullptr;
        const bool forced = ctx->probe_scratch_fail > 0;  // probe library (tests): a refused allocation
        if (forced) --ctx->probe_scratch_fail;
        if (forced || hipMalloc(&p, tcpck::api::kScratchImages * 2) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
          if (p) (void)hipFree(p);
          (void)hipGetLastError();
          for (auto &sl : ctx->scratch) {
            if (sl.buf) (void)hipFree(sl.buf);
            if (sl.ev) (void)hipEventDestroy(sl.ev);
            sl.buf = nullptr;
            sl.ev = nullptr;
          }
          // not latched: the refusal may be transient (memory pressure, another
          // thread capturing a graph in global mode); this call and the next
          // kScratchRetry - 1 run the in-stream form, then allocation is retried
          ++ctx->scratch_refusals;
          ctx->scratch_retry_at = ctx->scratch_calls + tcpck::api::kScratchRetry;
          return nullptr;
        }
        slot.buf = static_cast<uint16_t *>(p);
        slot.ev = ev;
      }
      ctx->scratch_images = tcpck::api::kScratchImages;
    }
    // an idle slot (never used, or its last user's work done), else the next in turn
    for (int i = 0; i < n && pick < 0; ++i) {
      auto &slot = ctx->scratch[(ctx->scratch_next + i) % n];
      std::unique_lock<std::mutex> try_lk(slot.mu, std::try_to_lock);
      if (!try_lk.owns_lock()) continue;
      if (!slot.used || hipEventQuery(slot.ev) == hipSuccess) {
        pick = static_cast<int>((ctx->scratch_next + i) % n);
        held = std::move(try_lk);
      }
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    if (pick < 0) pick = static_cast<int>(ctx->scratch_next % n);
    ctx->scratch_next = static_cast<unsigned>(pick + 1);
  }
  // every slot busy: wait for the chosen one's holder with scratch_mu released,
  // so other callers can still take a slot that frees meanwhile
  if (!held.owns_lock()) held = std::unique_lock<std::mutex>(ctx->scratch[pick].mu);
  return &ctx->scratch[pick];
}

// launch(k0, n, results) for images [k0, k0 + n), n <= scratch_images, with
// the slot's previous use waited for first (always, not only when the stream
// differs -- a destroyed stream's handle can come back for a new stream while
// the old one's work still runs) and the slot's event recorded after.
template <typename Launch>
hipError_t with_scratch(tcpck_ctx *ctx, tcpck_ctx::ScratchSlot *slot, uint64_t count, hipStream_t s,
                        Launch launch) {
  hipError_t e = hipSuccess;
  if (slot->used) e = hipStreamWaitEvent(s, slot->ev, 0);
  for (uint64_t k0 = 0; k0 < count && e == hipSuccess; k0 += ctx->scratch_images)
    e = launch(k0, std::min(ctx->scratch_images, count - k0), slot->buf);
  const hipError_t er = hipEventRecord(slot->ev, s);
  if (er == hipSuccess) slot->used = true;
  return e != hipSuccess ? e : er;
}

// ---- pipelined FILL (round 6) --------------------------
// A FILL whose form has a field pass (the deferred-field forms and the update
// form: fill_reads_results_*) runs the stream over all images and then the
// field pass over all images, one after the other.  Pipelined, the batch is cut
// into K chunks: chunk i's stream pass goes on the caller's stream, its field
// pass on the context's `pipe` stream after an event behind that stream pass,
// so the field pass of chunk i runs beside the stream pass of chunk i + 1, and
// the caller's stream waits for the last field pass (pipe_ev[K]) before
// anything it enqueues next.  Chunks are disjoint image ranges: a field pass
// writes only bytes 28-29 of its own chunk's images, which no other chunk's
// stream sums, and it reads only its own chunk's results.

constexpr int kFillPipeAuto = 0;          // AUTO's chunk count (0: not pipelined), DESIGN.md section 8
constexpr uint64_t kFillPipeMinImages = 4096;  // per chunk

hipError_t ensure_pipe(tcpck_ctx *ctx) {
  if (ctx->pipe) return hipSuccess;
  hipStream_t st = nullptr;
  hipError_t e = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, ctx->pipe_prio);
  for (int i = 0; i <= tcpck_ctx::kPipeMax && e == hipSuccess; ++i)
    if (!ctx->pipe_ev[i]) e = hipEventCreateWithFlags(&ctx->pipe_ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {  // the events made so far stay for the next attempt; freed by free_pipe
    if (st) (void)hipStreamDestroy(st);
    (void)hipGetLastError();
    return e;
  }
  ctx->pipe = st;
  return hipSuccess;
}

// K for this FILL (<= 1: not pipelined).  Only forms with a field pass, only
// with the caller's stream not capturing (the pipe stream would join the
// capture), and at least kFillPipeMinImages per chunk.
int fill_pipe_k(int op, int kernel, bool has_field_pass, uint64_t count, hipStream_t s, const Hooks &hk) {
  if (op != TCPCK_OP_FILL || kernel != TCPCK_KERNEL_AUTO || !has_field_pass) return 0;
  int k = hk.fill_pipe >= 0 ? hk.fill_pipe : kFillPipeAuto;
  k = static_cast<int>(std::min<uint64_t>(std::min(k, tcpck_ctx::kPipeMax), count / kFillPipeMinImages));
  if (k <= 1) return 0;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return cs == hipStreamCaptureStatusNone ? k : 0;
}

// launch(k0, n, ps, pev) enqueues images [k0, k0 + n): the stream pass on s,
// the field pass on ps after pev (ps == nullptr: everything on s).
// (one_stream, probe library: the same chunks with both passes on s -- the
// cost of chunking alone, without the second stream)
template <typename Launch>
hipError_t fill_pipelined(tcpck_ctx *ctx, int k, uint64_t count, hipStream_t s, bool one_stream, Launch launch) {
  std::lock_guard<std::mutex> lk(ctx->pipe_mu);
  if (ensure_pipe(ctx) != hipSuccess) return launch(0, count, nullptr, nullptr);  // the serial form
  hipError_t e = hipSuccess;
  const uint64_t per = (count + static_cast<uint64_t>(k) - 1) / static_cast<uint64_t>(k);
  int i = 0;
  for (uint64_t k0 = 0; k0 < count && e == hipSuccess; k0 += per, ++i)
    e = one_stream ? launch(k0, std::min(per, count - k0), nullptr, nullptr)
                   : launch(k0, std::min(per, count - k0), ctx->pipe, ctx->pipe_ev[i]);
  // join, also after an error: nothing the caller enqueues next may overtake a field pass already queued
  hipError_t ej = hipEventRecord(ctx->pipe_ev[tcpck_ctx::kPipeMax], ctx->pipe);
  if (ej == hipSuccess) ej = hipStreamWaitEvent(s, ctx->pipe_ev[tcpck_ctx::kPipeMax], 0);
  return e != hipSuccess ? e : ej;
}

// run_fixed / run_var for a FILL, pipelined when fill_pipe_k says so.
hipError_t fill_fixed(tcpck_ctx *ctx, int mode, uint8_t *arena, uint64_t stride, uint32_t len, uint64_t count,
                      uint16_t *out, int kernel, int param, hipStream_t s, const Hooks &hk) {
  const bool field_pass = out && kernel == TCPCK_KERNEL_AUTO && fill_reads_results_fixed(mode, arena, stride, len, param);
  const int k = fill_pipe_k(TCPCK_OP_FILL, kernel, field_pass, count, s, hk);
  if (k <= 1)
    return run_fixed(ctx, TCPCK_OP_FILL, mode, arena, stride, len, count, out, kernel, param, s, nullptr, hk);
  return fill_pipelined(ctx, k, count, s, hk.pipe_one_stream, [&](uint64_t k0, uint64_t n, hipStream_t ps, hipEvent_t pev) {
    return run_fixed_r(ctx, TCPCK_OP_FILL, mode, arena + k0 * stride, n == 1 ? len : stride, len, n, out + k0, kernel,
                       param, s, nullptr, hk, ps, pev);
  });
}

hipError_t fill_var(tcpck_ctx *ctx, int mode, uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    uint64_t count, uint16_t *out, const tcpck_layout *layout, int kernel, int param, hipStream_t s,
                    const Hooks &hk) {
  const bool field_pass = out && kernel == TCPCK_KERNEL_AUTO && fill_reads_results_var(mode, layout, count, param);
  const int k = fill_pipe_k(TCPCK_OP_FILL, kernel, field_pass, count, s, hk);
  if (k <= 1) return run_var(ctx, TCPCK_OP_FILL, mode, arena, off, len, 0, count, out, layout, kernel, param, s, nullptr, hk);
  return fill_pipelined(ctx, k, count, s, hk.pipe_one_stream, [&](uint64_t k0, uint64_t n, hipStream_t ps, hipEvent_t pev) {
    tcpck_layout sub{};
    if (layout) sub = sub_layout(*layout, n, count);
    return run_var_r(ctx, TCPCK_OP_FILL, mode, arena, off + k0, len + k0, 0, n, out + k0, layout ? &sub : nullptr,
                     kernel, param, s, nullptr, hk, ps, pev);
  });
}

}  // namespace

int batch_fixed_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, uint64_t stride, uint32_t len, uint64_t count,
                   void *d_out, int kernel, int param, hipStream_t s, const Hooks &hk) {
  if (!ctx || !valid_device_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  // images start at even addresses: the kernels pair bytes into u16 words by address
  if (!d_arena || (reinterpret_cast<uintptr_t>(d_arena) & 1) || (len & 1) || (stride & 1) ||
      (count > 1 && stride < len))
    return TCPCK_EINVAL;
  if (!d_out && op != TCPCK_OP_FILL) return TCPCK_EINVAL;
  if (op == TCPCK_OP_FILL && len < 30) return TCPCK_EINVAL;
  if (op == TCPCK_OP_RECEIVE && len < TCPCK_HEADER_BYTES) return TCPCK_EINVAL;
  if (count > 1 && stride > (UINT64_MAX - len) / (count - 1)) return TCPCK_EINVAL;
  if (count == 1) stride = len;  // one image: its stride is never read; the run kernels assume stride >= len
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  auto *arena = static_cast<uint8_t *>(d_arena);
  if (op == TCPCK_OP_FILL && !d_out && kernel == TCPCK_KERNEL_AUTO &&
      fill_reads_results_fixed(mode, arena, stride, len, param)) {
    std::unique_lock<std::mutex> held;
    if (auto *slot = take_scratch(ctx, s, held))
      return hip_status(with_scratch(ctx, slot, count, s, [&](uint64_t k0, uint64_t n, uint16_t *res) {
        return fill_fixed(ctx, mode, arena + k0 * stride, n == 1 ? len : stride, len, n, res, kernel, param, s, hk);
      }));
  }
  if (op == TCPCK_OP_FILL)
    return hip_status(fill_fixed(ctx, mode, arena, stride, len, count, static_cast<uint16_t *>(d_out), kernel, param,
                                 s, hk));
  return hip_status(run_fixed(ctx, op, mode, arena, stride, len, count, d_out, kernel, param, s, nullptr, hk));
}

int batch_var_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, const uint64_t *d_offsets,
                 const uint32_t *d_lengths, uint64_t count, void *d_out, const tcpck_layout *layout, int kernel,
                 int param, hipStream_t s, const Hooks &hk) {
  if (!ctx || !valid_device_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!d_arena || !d_offsets || !d_lengths || (reinterpret_cast<uintptr_t>(d_arena) & 1)) return TCPCK_EINVAL;
  if (!d_out && op != TCPCK_OP_FILL) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  auto *arena = static_cast<uint8_t *>(d_arena);
  if (op == TCPCK_OP_FILL && !d_out && kernel == TCPCK_KERNEL_AUTO &&
      fill_reads_results_var(mode, layout, count, param)) {
    std::unique_lock<std::mutex> held;
    if (auto *slot = take_scratch(ctx, s, held))
      return hip_status(with_scratch(ctx, slot, count, s, [&](uint64_t k0, uint64_t n, uint16_t *res) {
        tcpck_layout sub{};
        if (layout) sub = sub_layout(*layout, n, count);
        return fill_var(ctx, mode, arena, d_offsets + k0, d_lengths + k0, n, res, layout ? &sub : nullptr, kernel,
                        param, s, hk);
      }));
  }
  if (op == TCPCK_OP_FILL)
    return hip_status(fill_var(ctx, mode, arena, d_offsets, d_lengths, count, static_cast<uint16_t *>(d_out), layout,
                               kernel, param, s, hk));
  return hip_status(run_var(ctx, op, mode, arena, d_offsets, d_lengths, 0, count, d_out, layout, kernel, param, s,
                            nullptr, hk));
}

int check_receive(const tcpck_ctx *ctx, int mode, const void *d_arena, uint64_t &stride, uint32_t len,
                  const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, const uint8_t *d_ok,
                  const void *d_hdr) {
  if (!ctx || !valid_device_op_mode(TCPCK_OP_VERIFY, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!d_arena || !d_ok || (reinterpret_cast<uintptr_t>(d_arena) & 1) || (reinterpret_cast<uintptr_t>(d_hdr) & 3))
    return TCPCK_EINVAL;
  if (count > (UINT64_MAX >> 6)) return TCPCK_EINVAL;
  if (!d_offsets) {
    if ((len & 1) || (stride & 1) || len < TCPCK_HEADER_BYTES || (count > 1 && stride < len)) return TCPCK_EINVAL;
    if (count > 1 && stride > (UINT64_MAX - len) / (count - 1)) return TCPCK_EINVAL;
    if (count == 1) stride = len;
  } else if (!d_lengths) {
    return TCPCK_EINVAL;
  }
  return TCPCK_OK;
}

int batch_receive_ex(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                     const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                     void *d_hdr, const tcpck_layout *layout, int kernel, int param, hipStream_t s,
                     const Hooks &hk) {
  if (!d_hdr) {  // TCPCK_OP_RECEIVE: the headers converted in place
    return d_offsets ? batch_var_ex(ctx, TCPCK_OP_RECEIVE, mode, d_arena, d_offsets, d_lengths, count, d_ok, layout,
                                    kernel, param, s, hk)
                     : batch_fixed_ex(ctx, TCPCK_OP_RECEIVE, mode, d_arena, stride, len, count, d_ok, kernel, param,
                                      s, hk);
  }
  const int rc = check_receive(ctx, mode, d_arena, stride, len, d_offsets, d_lengths, count, d_ok, d_hdr);
  if (rc != TCPCK_OK || count == 0) return rc;
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  auto *arena = static_cast<uint8_t *>(d_arena);
  auto *hdr = static_cast<uint8_t *>(d_hdr);
  return hip_status(d_offsets ? run_var(ctx, TCPCK_OP_RECEIVE, mode, arena, d_offsets, d_lengths, 0, count, d_ok,
                                        layout, kernel, param, s, hdr, hk)
                              : run_fixed(ctx, TCPCK_OP_RECEIVE, mode, arena, stride, len, count, d_ok, kernel,
                                          param, s, hdr, hk));
}

}  // namespace api
}  // namespace tcpck

// helpers of tcpck_host_batch_*_multi
namespace {

// Runs shard i of n as job(i) -- shards 1.. on their own threads, shard 0 on the
// caller's -- and returns the first nonzero status in shard order.
template <typename Job>
int run_shards(int n, Job job_raw) {
  // nothing may escape a shard's thread (std::terminate) or the C ABI
  auto job = [&job_raw](int i) -> int {
    try {
      return job_raw(i);
    } catch (const std::bad_alloc &) {
      return TCPCK_ENOMEM;
    } catch (...) {
      return TCPCK_EINVAL;
    }
  };
  std::vector<int> rc;
  std::vector<std::thread> th;
  try {
    rc.assign(static_cast<size_t>(n), TCPCK_OK);
    th.reserve(static_cast<size_t>(n));
  } catch (...) {
    return TCPCK_ENOMEM;
  }
  for (int i = 1; i < n; ++i) {
    try {
      th.emplace_back([&rc, &job, i] { rc[static_cast<size_t>(i)] = job(i); });
    } catch (...) {  // no thread: run it here
      rc[static_cast<size_t>(i)] = job(i);
    }
  }
  rc[0] = job(0);
  for (auto &t : th) t.join();
  for (int r : rc)
    if (r != TCPCK_OK) return r;
  return TCPCK_OK;
}

bool valid_ctx_list(tcpck_ctx *const *ctxs, int n_ctx) {
  if (!ctxs || n_ctx < 1) return false;
  for (int i = 0; i < n_ctx; ++i)
    if (!ctxs[i]) return false;
  return true;
}

}  // namespace

extern "C" {

int tcpck_abi_version(void) { return TCPCK_ABI_VERSION; }

const char *tcpck_strerror(int status) {
  if (status == TCPCK_OK) return "ok";
  if (status == TCPCK_EINVAL) return "invalid argument (odd length/offset, null pointer, overflow)";
  if (status == TCPCK_ENOMEM) return "out of memory";
  if (status == TCPCK_ENODEV) return "no such HIP device";
  if (status <= TCPCK_EHIP) return hipGetErrorString(static_cast<hipError_t>(TCPCK_EHIP - status));
  return "unknown status";
}

int tcpck_device_supported(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    (void)hipGetLastError();  // no stale error for the caller's next HIP call
    return 0;
  }
  return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

int tcpck_ctx_create(int device, tcpck_ctx **out) {
  if (!out) return TCPCK_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    (void)hipGetLastError();
    return TCPCK_ENODEV;
  }
  if (!tcpck_device_supported(device)) return TCPCK_ENODEV;  // gfx950 code object only
  auto *ctx = new (std::nothrow) tcpck_ctx;
  if (!ctx) return TCPCK_ENOMEM;
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  // (the results scratch of out-less FILLs is allocated on first use: take_scratch)
  *out = ctx;
  return TCPCK_OK;
}

int tcpck_ctx_destroy(tcpck_ctx *ctx) {
  if (!ctx) return TCPCK_EINVAL;
  {
    DeviceGuard g(ctx->device);
    free_stage(ctx);
  }
  delete ctx;
  return TCPCK_OK;
}

int tcpck_ctx_device(const tcpck_ctx *ctx) { return ctx ? ctx->device : TCPCK_EINVAL; }

int tcpck_ctx_set_chunk_bytes(tcpck_ctx *ctx, uint64_t bytes) {
  if (!ctx || bytes < 4096) return TCPCK_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->chunk_bytes = bytes;
  return TCPCK_OK;
}

// ---- single image, host ----------------------------------------------------
int tcpck_checksum16(const void *image, size_t len, int mode, uint16_t *out) {
  if ((!image && len) || !out || (len & 1) ||
      (mode != TCPCK_MODE_REF && mode != TCPCK_MODE_RFC1071))
    return TCPCK_EINVAL;
  *out = finish_host(tcpck::host::word_sum(static_cast<const uint8_t *>(image), len), mode);
  return TCPCK_OK;
}

int tcpck_fill16(void *image, size_t len, int mode, uint16_t *out) {
  // validate everything before the image is touched: a rejected call leaves bytes 28-29 as they were
  if (!image || len < 30 || (len & 1) || (mode != TCPCK_MODE_REF && mode != TCPCK_MODE_RFC1071))
    return TCPCK_EINVAL;
  auto *b = static_cast<uint8_t *>(image);
  b[28] = 0;  // socket-manager.cc:9
  b[29] = 0;
  uint16_t c;
  int rc = tcpck_checksum16(image, len, mode, &c);  // socket-manager.cc:10
  if (rc) return rc;
  std::memcpy(b + 28, &c, 2);
  if (out) *out = c;
  return TCPCK_OK;
}

uint16_t tcpck_update16(uint16_t checksum, uint16_t old_word, uint16_t new_word, int mode) {
  if (mode == TCPCK_MODE_REF) {
    // stored C = ~S (mod 2^16)  =>  C' = ~(S - old + new)
    const uint16_t s = static_cast<uint16_t>(~checksum);
    return static_cast<uint16_t>(~static_cast<uint16_t>(s - old_word + new_word));
  }
  // RFC 1624 eqn. 3: C' = ~(~C + ~m + m') in one's complement arithmetic.
  uint32_t s = static_cast<uint16_t>(~checksum) + static_cast<uint32_t>(static_cast<uint16_t>(~old_word)) +
               new_word;
  s = (s & 0xFFFF) + (s >> 16);
  s = (s & 0xFFFF) + (s >> 16);
  if (s == 0) s = 0xFFFF;  // a real (non-all-zero) image never folds to +0
  return static_cast<uint16_t>(~s);
}

// ---- batched, device-resident -------------------------------------------------
int tcpck_batch_fixed(tcpck_ctx *ctx, int op, int mode, void *d_arena, uint64_t stride,
                      uint32_t len, uint64_t count, void *d_out, tcpck_stream stream) {
  return tcpck::api::batch_fixed_ex(ctx, op, mode, d_arena, stride, len, count, d_out, TCPCK_KERNEL_AUTO, 0,
                                    static_cast<hipStream_t>(stream), Hooks{});
}

int tcpck_batch_var(tcpck_ctx *ctx, int op, int mode, void *d_arena, const uint64_t *d_offsets,
                    const uint32_t *d_lengths, uint64_t count, void *d_out,
                    const tcpck_layout *layout, tcpck_stream stream) {
  return tcpck::api::batch_var_ex(ctx, op, mode, d_arena, d_offsets, d_lengths, count, d_out, layout,
                                  TCPCK_KERNEL_AUTO, 0, static_cast<hipStream_t>(stream), Hooks{});
}

// (tcpck_batch_fixed_ex / tcpck_batch_var_ex / tcpck_batch_receive_ex, the
// tuning entry points: tcpck_ex.hip, and tcpck_ex_probe.hip in the probe library)

// ---- batched retransmit: ACK rewrite + incremental update ----------------------
int tcpck_batch_set_ack(tcpck_ctx *ctx, int mode, void *d_arena, const uint64_t *d_offsets, uint64_t stride,
                        uint64_t count, const uint32_t *d_acks, uint32_t ack, uint16_t *d_out,
                        tcpck_stream stream) {
  if (!ctx || (mode != TCPCK_MODE_REF && mode != TCPCK_MODE_RFC1071)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!d_arena || (reinterpret_cast<uintptr_t>(d_arena) & 1)) return TCPCK_EINVAL;
  if (!d_offsets) {
    if ((stride & 1) || (count > 1 && stride < 30)) return TCPCK_EINVAL;
    if (count > 1 && stride > (UINT64_MAX - 30) / (count - 1)) return TCPCK_EINVAL;
  }
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  tcpck::AckArgs a{};
  a.arena = static_cast<uint8_t *>(d_arena);
  a.offsets = d_offsets;
  a.stride = stride;
  a.count = count;
  a.acks = d_acks;
  a.ack = ack;
  a.out = d_out;
  return hip_status(tcpck::launch_set_ack(mode, a, static_cast<uint32_t>(ctx->num_cus),
                                          static_cast<hipStream_t>(stream)));
}

// ---- receive batch: verdicts + host-order headers ------------------------------------
int tcpck_batch_receive(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                        const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                        void *d_hdr, const tcpck_layout *layout, tcpck_stream stream) {
  return tcpck::api::batch_receive_ex(ctx, mode, d_arena, stride, len, d_offsets, d_lengths, count, d_ok, d_hdr,
                                      layout, TCPCK_KERNEL_AUTO, 0, static_cast<hipStream_t>(stream), Hooks{});
}

// ---- header byte order: TcpHeaderN2H / TcpHeaderH2N in place -----------------------
int tcpck_batch_header_swap(tcpck_ctx *ctx, void *d_arena, const uint64_t *d_offsets, uint64_t stride,
                            uint64_t count, tcpck_stream stream) {
  if (!ctx) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!d_arena || (reinterpret_cast<uintptr_t>(d_arena) & 1)) return TCPCK_EINVAL;
  if (count > (UINT64_MAX >> 4)) return TCPCK_EINVAL;
  if (!d_offsets) {
    if ((stride & 1) || (count > 1 && stride < TCPCK_HEADER_BYTES)) return TCPCK_EINVAL;
    if (count > 1 && stride > (UINT64_MAX - TCPCK_HEADER_BYTES) / (count - 1)) return TCPCK_EINVAL;
  }
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  tcpck::HeaderArgs a{};
  a.arena = static_cast<uint8_t *>(d_arena);
  a.offsets = d_offsets;
  a.stride = stride;
  a.count = count;
  return hip_status(tcpck::launch_header_swap(a, static_cast<uint32_t>(ctx->num_cus),
                                              static_cast<hipStream_t>(stream)));
}

// ---- batched segmentation: send stream -> checksummed images --------------------
int tcpck_batch_segment(tcpck_ctx *ctx, int mode, const void *d_payload, uint64_t payload_bytes, uint32_t seg,
                        const void *hdr, uint32_t seq0, void *d_images, uint64_t stride, uint16_t *d_out,
                        tcpck_stream stream) {
  return tcpck_batch_segment_ex(ctx, mode, d_payload, payload_bytes, seg, hdr, seq0, d_images, stride, d_out, 0,
                                stream);
}

int tcpck_batch_segment_ex(tcpck_ctx *ctx, int mode, const void *d_payload, uint64_t payload_bytes, uint32_t seg,
                           const void *hdr, uint32_t seq0, void *d_images, uint64_t stride, uint16_t *d_out,
                           int param, tcpck_stream stream) {
  if (!ctx || (mode != TCPCK_MODE_REF && mode != TCPCK_MODE_RFC1071)) return TCPCK_EINVAL;
  if (payload_bytes == 0) return TCPCK_OK;
  if (!d_payload || !d_images || !hdr || (payload_bytes & 1)) return TCPCK_EINVAL;
  if (seg < 4 || seg > 65532 || (seg & 3) || (stride & 15) || stride < 32ull + seg || stride > (1u << 24))
    return TCPCK_EINVAL;
  if ((reinterpret_cast<uintptr_t>(d_payload) & 3) || (reinterpret_cast<uintptr_t>(d_images) & 15))
    return TCPCK_EINVAL;
  const uint64_t n = (payload_bytes + seg - 1) / seg;
  if (n > UINT64_MAX / stride) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  tcpck::SegmentArgs a{};
  a.payload = static_cast<const uint8_t *>(d_payload);
  a.images = static_cast<uint8_t *>(d_images);
  a.payload_bytes = payload_bytes;
  a.count = n;
  a.out = d_out;
  a.seg = seg;
  a.stride = static_cast<uint32_t>(stride);
  std::memcpy(a.hdr, hdr, 32);
  a.seq0 = seq0;
  return hip_status(tcpck::launch_segment(mode, param & 0xFF, a, static_cast<uint32_t>(param >> 16) & 0xFFFFu,
                                          static_cast<uint32_t>(ctx->num_cus), static_cast<hipStream_t>(stream)));
}

// ---- batched, host memory: chunked H2D -> kernel -> D2H on two streams ---------
int tcpck_host_batch_fixed(tcpck_ctx *ctx, int op, int mode, void *h_arena, uint64_t stride,
                           uint32_t len, uint64_t count, void *h_out) {
  if (!ctx || !valid_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!h_arena || (len & 1) || (stride & 1) || (count > 1 && stride < len)) return TCPCK_EINVAL;
  if (!h_out && op != TCPCK_OP_FILL) return TCPCK_EINVAL;
  if (op == TCPCK_OP_FILL && len < 30) return TCPCK_EINVAL;
  if (count > 1 && stride > (UINT64_MAX - len) / (count - 1)) return TCPCK_EINVAL;
  if (count == 1) stride = len;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  const uint64_t step = std::max<uint64_t>(stride, 2);
  const uint64_t per = std::max<uint64_t>(1, ctx->chunk_bytes / step);
  const uint64_t chunk_imgs = std::min(per, count);
  int rc = ensure_stage(ctx, (chunk_imgs - 1) * stride + len, chunk_imgs);
  if (rc) return rc;
  std::vector<uint16_t> fill_res;
  if (op == TCPCK_OP_FILL && !h_out) fill_res.resize(count);
  auto *arena = static_cast<uint8_t *>(h_arena);
  auto *out_bytes = h_out ? static_cast<uint8_t *>(h_out) : reinterpret_cast<uint8_t *>(fill_res.data());
  const size_t es = out_elem(op);
  hipError_t e = hipSuccess;
  uint64_t c = 0;
  for (uint64_t k0 = 0; k0 < count && e == hipSuccess; k0 += chunk_imgs, ++c) {
    const int slot = static_cast<int>(c & 1);
    const uint64_t n = std::min(chunk_imgs, count - k0);
    const uint64_t bytes = (n - 1) * stride + len;
    hipStream_t s = ctx->s[slot];
    e = hipMemcpyAsync(ctx->stage[slot], arena + k0 * stride, bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) break;
    e = tcpck::api::run_fixed(ctx, op, mode, ctx->stage[slot], stride, len, n, ctx->stage_out[slot],
                              TCPCK_KERNEL_AUTO, 0, s, nullptr, Hooks{});
    if (e != hipSuccess) break;
    e = hipMemcpyAsync(out_bytes + k0 * es, ctx->stage_out[slot], n * es, hipMemcpyDeviceToHost, s);
  }
  for (int i = 0; i < 2; ++i) {
    hipError_t e2 = hipStreamSynchronize(ctx->s[i]);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return hip_status(e);
  if (op == TCPCK_OP_FILL)
    patch_fields(arena, 0, count, reinterpret_cast<const uint16_t *>(out_bytes), nullptr, nullptr,
                 stride, len);
  return TCPCK_OK;
}

int tcpck_host_batch_var(tcpck_ctx *ctx, int op, int mode, void *h_arena, const uint64_t *h_offsets,
                         const uint32_t *h_lengths, uint64_t count, void *h_out) {
  if (!ctx || !valid_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!h_arena || !h_offsets || !h_lengths) return TCPCK_EINVAL;
  if (!h_out && op != TCPCK_OP_FILL) return TCPCK_EINVAL;
  uint64_t max_len = 0, min_len = UINT64_MAX;
  bool packed = true, sorted = true;
  for (uint64_t k = 0; k < count; ++k) {
    if ((h_offsets[k] | h_lengths[k]) & 1) return TCPCK_EINVAL;
    if (op == TCPCK_OP_FILL && h_lengths[k] < 30) return TCPCK_EINVAL;
    max_len = std::max<uint64_t>(max_len, h_lengths[k]);
    min_len = std::min<uint64_t>(min_len, h_lengths[k]);
    if (k + 1 < count && h_offsets[k] + h_lengths[k] != h_offsets[k + 1]) packed = false;
    if (k + 1 < count && h_offsets[k] + h_lengths[k] > h_offsets[k + 1]) sorted = false;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  if (g.status() != hipSuccess) return hip_status(g.status());
  const uint64_t cap = std::max<uint64_t>(ctx->chunk_bytes, max_len + 16);
  const uint64_t max_imgs = std::min<uint64_t>(count, std::max<uint64_t>(cap / 32, 1));
  int rc = ensure_stage(ctx, cap, max_imgs);
  if (rc) return rc;
  std::vector<uint16_t> fill_res;
  if (op == TCPCK_OP_FILL && !h_out) fill_res.resize(count);
  auto *arena = static_cast<uint8_t *>(h_arena);
  auto *out_bytes = h_out ? static_cast<uint8_t *>(h_out) : reinterpret_cast<uint8_t *>(fill_res.data());
  const size_t es = out_elem(op);
  tcpck_layout lay{};
  lay.min_len = static_cast<uint32_t>(std::min<uint64_t>(min_len, UINT32_MAX));
  lay.max_len = static_cast<uint32_t>(std::min<uint64_t>(max_len, UINT32_MAX));
  lay.flags = (packed ? TCPCK_LAYOUT_PACKED : 0u) | (sorted ? TCPCK_LAYOUT_SORTED : 0u);
  hipError_t e = hipSuccess;
  uint64_t c = 0;
  for (uint64_t k0 = 0; k0 < count && e == hipSuccess; ++c) {
    // greedy chunk: extend while the hull [lo, hi) of the chunk fits the stage
    uint64_t lo = h_offsets[k0] & ~uint64_t{15}, hi = h_offsets[k0] + h_lengths[k0];
    uint64_t k1 = k0 + 1, chunk_bytes = h_lengths[k0];
    while (k1 < count && k1 - k0 < max_imgs) {
      const uint64_t nlo = std::min(lo, h_offsets[k1] & ~uint64_t{15});
      const uint64_t nhi = std::max(hi, h_offsets[k1] + h_lengths[k1]);
      if (nhi - nlo > cap) break;
      lo = nlo;
      hi = nhi;
      chunk_bytes += h_lengths[k1];
      ++k1;
    }
    lay.total_bytes = chunk_bytes;  // the kernel policy sizes its grid by this launch's bytes
    const uint64_t n = k1 - k0;
    const int slot = static_cast<int>(c & 1);
    hipStream_t s = ctx->s[slot];
    e = hipMemcpyAsync(ctx->stage[slot], arena + lo, hi - lo, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ctx->stage_off[slot], h_offsets + k0, n * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ctx->stage_len[slot], h_lengths + k0, n * 4, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) break;
    e = tcpck::api::run_var(ctx, op, mode, ctx->stage[slot], ctx->stage_off[slot], ctx->stage_len[slot], lo, n,
                            ctx->stage_out[slot], &lay, TCPCK_KERNEL_AUTO, 0, s, nullptr, Hooks{});
    if (e != hipSuccess) break;
    e = hipMemcpyAsync(out_bytes + k0 * es, ctx->stage_out[slot], n * es, hipMemcpyDeviceToHost, s);
    k0 = k1;
  }
  for (int i = 0; i < 2; ++i) {
    hipError_t e2 = hipStreamSynchronize(ctx->s[i]);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return hip_status(e);
  if (op == TCPCK_OP_FILL)
    patch_fields(arena, 0, count, reinterpret_cast<const uint16_t *>(out_bytes), h_offsets, h_lengths,
                 0, 0);
  return TCPCK_OK;
}

// ---- host batches over several contexts (one per GPU) ---------------------------

int tcpck_host_batch_fixed_multi(tcpck_ctx *const *ctxs, int n_ctx, int op, int mode, void *h_arena,
                                 uint64_t stride, uint32_t len, uint64_t count, void *h_out) {
  if (!valid_ctx_list(ctxs, n_ctx) || !valid_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!h_arena || (!h_out && op != TCPCK_OP_FILL)) return TCPCK_EINVAL;
  if (count > 1 && stride > (UINT64_MAX - len) / (count - 1)) return TCPCK_EINVAL;
  const uint64_t n = std::min<uint64_t>(static_cast<uint64_t>(n_ctx), count);
  const size_t es = out_elem(op);
  auto *arena = static_cast<uint8_t *>(h_arena);
  auto *out = static_cast<uint8_t *>(h_out);
  return run_shards(static_cast<int>(n), [&](int i) {
    const uint64_t q = count / n, r = count % n, ui = static_cast<uint64_t>(i);
    const uint64_t k0 = ui * q + std::min(ui, r), k1 = k0 + q + (ui < r ? 1 : 0);
    return tcpck_host_batch_fixed(ctxs[i], op, mode, arena + k0 * stride, stride, len, k1 - k0,
                                  out ? out + k0 * es : nullptr);
  });
}

int tcpck_host_batch_var_multi(tcpck_ctx *const *ctxs, int n_ctx, int op, int mode, void *h_arena,
                               const uint64_t *h_offsets, const uint32_t *h_lengths, uint64_t count,
                               void *h_out) {
  if (!valid_ctx_list(ctxs, n_ctx) || !valid_op_mode(op, mode)) return TCPCK_EINVAL;
  if (count == 0) return TCPCK_OK;
  if (!h_arena || !h_offsets || !h_lengths || (!h_out && op != TCPCK_OP_FILL)) return TCPCK_EINVAL;
  const uint64_t n = std::min<uint64_t>(static_cast<uint64_t>(n_ctx), count);
  // shard starts balanced by bytes: shard i begins at the first image whose
  // byte prefix reaches i/n of the total (a 1492-B image is 15.5x a 96-B one)
  uint64_t total = 0;
  for (uint64_t k = 0; k < count; ++k) total += h_lengths[k];
  std::vector<uint64_t> cut;
  try {
    cut.assign(n + 1, count);
  } catch (...) {
    return TCPCK_ENOMEM;
  }
  cut[0] = 0;
  uint64_t pre = 0, k = 0;
  for (uint64_t i = 1; i < n; ++i) {
    const uint64_t target = static_cast<uint64_t>((static_cast<unsigned __int128>(total) * i) / n);
    while (k < count && pre < target) pre += h_lengths[k++];
    cut[i] = std::max(k, cut[i - 1]);
  }
  const size_t es = out_elem(op);
  auto *out = static_cast<uint8_t *>(h_out);
  return run_shards(static_cast<int>(n), [&](int i) {
    const uint64_t k0 = cut[static_cast<size_t>(i)], k1 = cut[static_cast<size_t>(i) + 1];
    if (k1 <= k0) return TCPCK_OK;
    return tcpck_host_batch_var(ctxs[i], op, mode, h_arena, h_offsets + k0, h_lengths + k0, k1 - k0,
                                out ? out + k0 * es : nullptr);
  });
}

// ---- memory helpers -----------------------------------------------------------
int tcpck_host_alloc(size_t bytes, void **out) {
  if (!out) return TCPCK_EINVAL;
  *out = nullptr;
  return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? TCPCK_OK : TCPCK_ENOMEM;
}

int tcpck_host_free(void *p) { return hip_status(hipHostFree(p)); }

int tcpck_device_alloc(tcpck_ctx *ctx, size_t bytes, void **out) {
  if (!ctx || !out) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  *out = nullptr;
  return hipMalloc(out, bytes) == hipSuccess ? TCPCK_OK : TCPCK_ENOMEM;
}

int tcpck_device_free(tcpck_ctx *ctx, void *p) {
  if (!ctx) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  return hip_status(hipFree(p));
}

int tcpck_memcpy_h2d(tcpck_ctx *ctx, void *dst, const void *src, size_t bytes) {
  if (!ctx) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  return hip_status(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
}

int tcpck_memcpy_d2h(tcpck_ctx *ctx, void *dst, const void *src, size_t bytes) {
  if (!ctx) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  return hip_status(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
}

int tcpck_stream_sync(tcpck_ctx *ctx, tcpck_stream stream) {
  if (!ctx) return TCPCK_EINVAL;
  DeviceGuard g(ctx->device);
  return hip_status(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

}  // extern "C"
