// tcpck_api_internal.h -- the context and the batch router shared by the C-ABI
// layer (tcpck_api.hip), its tuning entry points (tcpck_ex.hip in libtcpck.so)
// and their measurement twins (tcpck_ex_probe.hip in libtcpck_probe.so).  Not
// installed.
//
// The router (tcpck::api::batch_*_ex) is the product's kernel policy and
// nothing else; the probe library passes it a Hooks value to reach the
// measured alternatives (header pass forms, fused headers on explicit kernels),
// the product library always passes Hooks{}.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>

#include "tcpck.h"

struct tcpck_ctx {
  int device = 0;
  int num_cus = 256;

  // end-to-end (host batch) pipeline state, created lazily
  std::mutex mu;
  hipStream_t s[2] = {nullptr, nullptr};
  uint8_t *stage[2] = {nullptr, nullptr};     // image bytes
  uint8_t *stage_out[2] = {nullptr, nullptr}; // results
  uint64_t *stage_off[2] = {nullptr, nullptr};
  uint32_t *stage_len[2] = {nullptr, nullptr};
  uint64_t stage_bytes = 0;
  uint64_t stage_images = 0;
  uint64_t chunk_bytes = 64ull << 20;

  // FILL without a results buffer (the reference's insert stores only into the
  // packet, socket-manager.cc:9-10) where AUTO's form reads the results back
  // (the stream writes them, the write-through field pass stores them): the
  // results go to one of kScratchSlots ctx-owned slots, allocated on first use.
  // A call takes an idle slot (or, all busy, the next in turn) under
  // `scratch_mu`, then holds that slot's own mutex while it waits on the
  // slot's event, launches and records the event again -- so FILLs from
  // several threads on several streams overlap, and a slot's reuse still waits
  // for its previous user's work.  Batches of more images run in chunks.
  struct ScratchSlot {
    std::mutex mu;
    uint16_t *buf = nullptr;
    hipEvent_t ev = nullptr;
    bool used = false;  // ev recorded at least once
  };
  static constexpr int kScratchSlots = 4;
  std::mutex scratch_mu;
  ScratchSlot scratch[kScratchSlots];
  uint64_t scratch_images = 0;
  unsigned scratch_next = 0;
  // A refused allocation is not latched: the call runs the in-stream form and
  // the slots are tried again after kScratchRetry more out-less FILLs.
  uint64_t scratch_retry_at = 0;   // out-less FILL count from which allocation is tried again
  uint64_t scratch_calls = 0;      // out-less FILLs that asked for a slot
  uint64_t scratch_refusals = 0;   // allocations refused so far (tcpck_probe_scratch_state)
  int probe_scratch_fail = 0;      // probe library: refuse this many more allocation attempts (tests)

  // Pipelined FILL (round 6): the batch in K chunks, chunk i's stream pass on
  // the caller's stream and its field pass on `pipe` after the event
  // pipe_ev[i], so the field pass of chunk i runs beside the stream of chunk
  // i + 1; pipe_ev[K] joins `pipe` back into the caller's stream.  Created on
  // first use; one pipelined call is enqueued at a time (pipe_mu).
  static constexpr int kPipeMax = 32;
  std::mutex pipe_mu;
  hipStream_t pipe = nullptr;
  hipEvent_t pipe_ev[kPipeMax + 1] = {};
  int pipe_prio = 0;               // the pipe stream's priority (probe: tcpck_probe_set_fill_pipe)
  int probe_fill_pipe = -1;        // probe library: K (0/1 off, -1 AUTO's rule)
  bool probe_pipe_one_stream = false;  // probe library: the K chunks one after the other on the caller's stream

  // probe library only (tcpck_ex_probe.hip): per-wave time stamp buffer, and the
  // side stream + events of the concurrent RECEIVE form
  void *dbg = nullptr;
  uint8_t *probe_side = nullptr;   // rstream 33 / 34: the field blocks' side buffer (64 B per image)
  uint64_t probe_side_cap = 0;
  std::mutex side_mu;
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

namespace tcpck {
namespace host {
// The exact sum of the little-endian u16 words of p[0, n) (n even), host code
// (tcpck_host.cc); tcpck_checksum16 finishes it.
uint64_t word_sum(const uint8_t *p, size_t n);
}  // namespace host

namespace api {

constexpr uint64_t kScratchImages = 8ull << 20;  // 16 MiB of u16 results: C5's 8M images in one chunk
constexpr uint64_t kScratchRetry = 64;           // out-less FILLs between allocation attempts after a refusal

// Measurement hooks (libtcpck_probe.so only; the product passes Hooks{}).
struct Hooks {
  bool fuse_any_hdr = false;     // RECEIVE, explicit kernel: fuse the headers into any kernel that can
                                 // (sstream's after-the-verdicts conversion, HDR 1)
  bool hdr_after = false;        // RECEIVE into a header array: the separate header pass after VERIFY (the
                                 // product runs it first under AUTO, tcpck_api.hip fixed_receive_fuses)
  bool hdr_first_explicit = false;  // ... first with an explicit VERIFY kernel too (the product runs it after
                                    // an explicit kernel, so a rejected choice leaves the header array as it was)
  uint32_t hdr_store_bits = 0;   // HeaderArgs::store_bits of the header pass
  bool patch_reverse = false;    // FILL's field pass in reverse image order (PatchArgs::reverse)
  int fill_pipe = -1;            // pipelined FILL chunks: -1 AUTO's rule, 0 / 1 off, K > 1 K chunks
  bool pipe_one_stream = false;  // ... every chunk's passes on the caller's stream (the chunking cost alone)
};

// probe library: tcpck_batch_*_ex param bit selecting Hooks::patch_reverse
constexpr int kProbeParamPatchReverse = 1 << 27;

int hip_status(hipError_t e);

// Saves the calling thread's current device, switches to `device`, restores.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device);
  ~DeviceGuard();
  hipError_t status() const { return ok_; }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;

 private:
  int prev_ = -1;
  hipError_t ok_ = hipSuccess;
};

// The validated device-batch entry points (tcpck_tuning.h semantics).
int batch_fixed_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, uint64_t stride, uint32_t len, uint64_t count,
                   void *d_out, int kernel, int param, hipStream_t stream, const Hooks &hk);
int batch_var_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, const uint64_t *d_offsets,
                 const uint32_t *d_lengths, uint64_t count, void *d_out, const tcpck_layout *layout, int kernel,
                 int param, hipStream_t stream, const Hooks &hk);
int batch_receive_ex(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                     const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                     void *d_hdr, const tcpck_layout *layout, int kernel, int param, hipStream_t stream,
                     const Hooks &hk);
// batch_receive_ex's checks without the launch (TCPCK_OK or the error status)
int check_receive(const tcpck_ctx *ctx, int mode, const void *d_arena, uint64_t &stride, uint32_t len,
                  const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, const uint8_t *d_ok,
                  const void *d_hdr);

// The routed launches behind them (device already selected, arguments valid).
hipError_t run_fixed(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, uint64_t stride, uint32_t len, uint64_t count,
                     void *out, int kernel, int param, hipStream_t s, uint8_t *hdr, const Hooks &hk);
hipError_t run_var(tcpck_ctx *ctx, int op, int mode, uint8_t *arena, const uint64_t *off, const uint32_t *len,
                   uint64_t base, uint64_t count, void *out, const tcpck_layout *layout, int kernel, int param,
                   hipStream_t s, uint8_t *hdr, const Hooks &hk);

}  // namespace api
}  // namespace tcpck
