/*
 * tcpck_probe.h -- measurement-only entry points, exported by
 * libtcpck_probe.so alone (tcp-stack_amd/Makefile builds it from the same
 * sources with -DTCPCK_PROBE).  The product library libtcpck.so does not
 * carry them: scripts/ and the variant tests use them to time kernels.
 */
#ifndef TCPCK_PROBE_H_
#define TCPCK_PROBE_H_

#include "tcpck_tuning.h"

#ifdef __cplusplus
extern "C" {
#endif

/* tcpck_batch_fixed_ex kernel id: FILL's deferred field pass ALONE, in one of
 * its measured forms (launch_patch_fields' timing kernels) -- d_out[k] (u16)
 * stored into image k's field; no checksum is computed.  For timing the pass
 * apart from the stream (scripts/fill_drain_probe.py).  param = 1 + the
 * stores' cache bits (sc0 1 | nt 2 | sc1 4), 0 = a plain C++ store, | form
 * << 4: 0 the field's 64-B block read and written back whole, 1 the 16-B
 * chunk, 2 the 2-B field, 3 the 128-B line, 4-7 the 2-B write-through field
 * with other thread maps (cache bits ignored), 12 the 32-B block; 8 / 9 / 10 /
 * 11 the 64-B / 128-B / 16-B / 32-B block written without reading it (zeros
 * around the field: destroys the images, whole-block write timing only).
 * param 0 is therefore the 64-B block with a plain store; the product's pass
 * (one 2-B write-through store per image) is form 2 with bits sc0 sc1 nt,
 * param 0x28. */
#define TCPCK_KERNEL_PATCH 12

/* tcpck_probe_receive_ex: tcpck_batch_receive_ex with the header pass in a
 * measured form, chosen by a flags word of its own (param keeps
 * tcpck_tuning.h's meaning):
 *   HDR_FIRST   (accepted, no effect: since round 5 the product runs a separate
 *               header pass into a header array before the VERIFY pass)
 *   HDR_AFTER   the separate header pass after the VERIFY pass (the order
 *               before round 5)
 *   CONCURRENT  the header pass on the context's side stream, beside VERIFY
 *   HDR_WT      the header array stores written through (sc0 sc1 nt)
 *   HDR_WIDE    two lanes per 16-B aligned image, one 16-B buffer load each,
 *               with the load cache bits (flags >> CACHE_SHIFT) & 3: 0
 *               default, 1 nt, 2 sc0 sc1, 3 sc1
 *   ORDER       (flags >> ORDER_SHIFT) & 3, the product's header pass in
 *               another image order: 1 XCD-chunked blocks, 2 blocks scattered
 *               over the batch, 3 each block's images 1/128 of the batch
 *               apart (0: in order) */
#define TCPCK_PROBE_RECEIVE_HDR_FIRST 1
#define TCPCK_PROBE_RECEIVE_HDR_AFTER 16
#define TCPCK_PROBE_RECEIVE_CONCURRENT 2
#define TCPCK_PROBE_RECEIVE_HDR_WT 4
#define TCPCK_PROBE_RECEIVE_HDR_WIDE 8
#define TCPCK_PROBE_RECEIVE_CACHE_SHIFT 4
#define TCPCK_PROBE_RECEIVE_ORDER_SHIFT 8
int tcpck_probe_receive_ex(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                           const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                           void *d_hdr, const tcpck_layout *layout, int kernel, int param, int probe_flags,
                           tcpck_stream stream);

/* tcpck_batch_fixed_ex / tcpck_batch_var_ex param bit: FILL's field pass
 * (deferred or update form) walks the images in reverse index order, so it
 * starts on the lines the stream read last (probe library only). */
#define TCPCK_PROBE_PARAM_PATCH_REVERSE (1 << 27)

/* Device buffer of 4 x u64 per wave receiving {start, end} s_memrealtime
 * (100 MHz) stamps, HW_ID and XCC_ID from the rstream variants built with
 * stamps (3, 7; NULL = off). */
int tcpck_ctx_set_debug(tcpck_ctx *ctx, void *d_buf);

/* The context's results-scratch slots (tcpck.h, out-less FILL): how many are
 * allocated and a bit per slot that a FILL has used (its event recorded). */
int tcpck_probe_scratch_state(tcpck_ctx *ctx, int *allocated, int *used_mask);

/* Fault injection for the scratch slots: the next n allocation attempts of an
 * out-less FILL are refused as if hipMalloc had failed.  *refusals (may be
 * NULL) receives the refusals so far.  After a refusal the context retries
 * the allocation 64 out-less FILLs later (not latched). */
int tcpck_probe_scratch_fail(tcpck_ctx *ctx, int n, uint64_t *refusals);

/* The pipelined FILL (round 6; tcp-stack_amd/csrc/tcpck_api.hip
 * fill_pipelined) under TCPCK_KERNEL_AUTO in this context: k chunks (0 / 1:
 * the serial form, -1: AUTO's rule), the field pass of chunk i on a context
 * stream of priority prio (hipStreamCreateWithPriority; a changed priority
 * recreates the stream after draining it) beside the stream pass of chunk
 * i + 1.  Applies to FILLs whose form has a field pass, at least 4096 images
 * per chunk, k <= 32.  k | TCPCK_PROBE_PIPE_ONE_STREAM: the same k chunks
 * with both passes on the caller's stream (the cost of chunking alone). */
#define TCPCK_PROBE_PIPE_ONE_STREAM 0x100
int tcpck_probe_set_fill_pipe(tcpck_ctx *ctx, int k, int prio);

/* Timing-only streaming micro-kernel over d_buf (results are not checksums):
 * variant = chunks per lane per step x steps in flight x scan, see
 * tcp-stack_amd/csrc/tcpck_diag.hip.  d_out: u32 per wave. */
int tcpck_diag_stream(tcpck_ctx *ctx, int variant, const void *d_buf, uint64_t bytes, void *d_out,
                      tcpck_stream stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* TCPCK_PROBE_H_ */
