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

/* tcpck_batch_fixed_ex kernel id: FILL's deferred field pass ALONE
 * (launch_patch_fields) -- each field's 64-B block read and written back whole
 * with d_out[k] (u16) patched in; no checksum is computed.  For timing the
 * pass apart from the stream (scripts/fill_drain_probe.py).  param = 1 + the
 * block stores' cache bits (sc0 1 | nt 2 | sc1 4), 0 = a plain store, | form
 * << 4: 0 the 64-B block, 1 the 16-B chunk, 2 the 2-B field, 3 the 128-B line,
 * 4-7 the 2-B write-through field with other thread maps, 12 the 32-B block;
 * 8 / 9 / 10 / 11 the 64-B / 128-B / 16-B / 32-B block written without
 * reading it (zeros around the field: destroys the images, whole-block write
 * timing only). */
#define TCPCK_KERNEL_PATCH 12

/* Device buffer of 4 x u64 per wave receiving {start, end} s_memrealtime
 * (100 MHz) stamps, HW_ID and XCC_ID from the rstream variants built with
 * stamps (3, 7; NULL = off). */
int tcpck_ctx_set_debug(tcpck_ctx *ctx, void *d_buf);

/* Timing-only streaming micro-kernel over d_buf (results are not checksums):
 * variant = chunks per lane per step x steps in flight x scan, see
 * tcp-stack_amd/csrc/tcpck_diag.hip.  d_out: u32 per wave. */
int tcpck_diag_stream(tcpck_ctx *ctx, int variant, const void *d_buf, uint64_t bytes, void *d_out,
                      tcpck_stream stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* TCPCK_PROBE_H_ */
