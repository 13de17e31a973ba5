/*
 * tcpck_tuning.h -- kernel-selection entry points for benchmarking and tuning.
 * Not needed by a drop-in caller: tcpck_batch_fixed / tcpck_batch_var
 * (tcpck.h) pick the kernel themselves.  Results never depend on the kernel
 * chosen; an inapplicable choice returns an error.
 *
 * Two libraries export these functions:
 *   libtcpck.so        the product.  It holds only the kernels the AUTO
 *                      policy picks, so here it accepts exactly AUTO's own
 *                      choices: SEG shapes 0 (by length), 1, 2, 7, 8, 9, 11;
 *                      RSTREAM variant 20 (FILL also 25); VVSTREAM variant 4
 *                      with any of the flags + 8 / + 16 / + 32 / + 64;
 *                      GSTREAM FILL with 0, 0x80 or 0x401 (+ 4); SSTREAM 0,
 *                      + 32 (RECEIVE into a header array) and + 128 (FILL
 *                      with a results buffer); tcpck_batch_segment_ex
 *                      variant 0 (+ 8); with any oversubscription / cap bits
 *                      and the TCPCK_PARAM_* bits below.  Any other value
 *                      returns an error there (hipErrorInvalidValue).
 *   libtcpck_probe.so  the same router and kernels built with -DTCPCK_PROBE
 *                      (tcp-stack_amd/csrc/tcpck_ex_probe.hip in place of
 *                      tcpck_ex.hip): every variant documented below, plus
 *                      tcpck_probe.h.  With an explicit kernel its RECEIVE
 *                      also fuses the headers into sstream's other forms.
 */
#ifndef TCPCK_TUNING_H_
#define TCPCK_TUNING_H_

#include "tcpck.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TCPCK_KERNEL_AUTO 0 /* library policy (what tcpck_batch_* use)              */
#define TCPCK_KERNEL_SEG 1  /* G lanes per image, any layout; param = shape + 1
                               (1: G8/U2, 2: G16/U6, 3: G64/U4, 4: G64/U2,
                                5: G32/U3, 6: G4/U8; W waves per image:
                                7: W4/U4, 8: W8/U4, 9: W16/U2, 10: W16/U4,
                                11: W2/U4), 0 = by length
                               | (grid oversubscription << 16)
                               | (1 << 24: each XCD takes groups of 16 blocks)  */
/* 2, 3, 4, 6, 7: span, stream, fstream, rvstream and vstream, measured in
   round 1 and removed (profiles/DESIGN_history_r01-r04.md section 4); 11: bstream (byte runs across
   image edges, round 2, removed); the numbers are not reused. */
#define TCPCK_KERNEL_RSTREAM 5 /* fixed stride == len only, MODE_REF: one run per
                                  wave, scalar boundary walk; param = variant
                                  (0: 4 loads in flight, 1: 2, 2: 8, 3: 4 with
                                  per-wave time stamps, checksum only; 4/6/8:
                                  4/8/2 loads with slot-graded s_setprio, 5: 4
                                  with s_setprio 1 for slots >= 4, 7: 3 + graded
                                  priority, 9: 4 with v_dot2 sums, 10/12/13:
                                  4/2/8 with v_dot2 sums and buffer loads, 11: 4
                                  with buffer loads; 14/15: 10/13 with each XCD
                                  taking one contiguous region of runs; 16-19: 10
                                  with each XCD taking groups of 2/4/16/64
                                  consecutive runs; 20/21: 18/14 with the run's
                                  first step read with the default cache policy,
                                  20 = the policy's (since round 5 only the
                                  run's first line, = 31; 32: the whole first
                                  step, the policy before round 5); 22: 18 with
                                  every step read
                                  with the default policy; 23/24: 20 with 8/2
                                  steps in flight; 25: 20's FILL with the fields
                                  stored by the write-through 2-B field pass,
                                  AUTO's FILL; 26: 20 with write-through field
                                  stores in the stream; 27/28: 20's FILL writing
                                  each field's whole 64-B block from the stream
                                  (28: a short run's blocks after its last load),
                                  stride >= 128)
                                  | (blocks per CU cap << 8)
                                  | (grid oversubscription << 16: 0 = by batch
                                  size, 1 = none, M = M x the resident grid)    */
#define TCPCK_KERNEL_VVSTREAM 8 /* MODE_REF, all ops: packed variable layouts and
                                   fixed strides (stride >= len, gaps streamed),
                                   any even image length; run per wave, a step's
                                   image ends resolved in parallel from an LDS
                                   prefix table; param = variant (0: 4 loads in
                                   flight, byte-balanced runs, 1: 8; 2/3: same
                                   with equal-count runs -- fixed layouts are
                                   always equal-count; 4: policy; + 8: each XCD
                                   takes groups of 16 consecutive runs; + 16: the
                                   run's first line read with the default cache
                                   policy (5 instead of 4, probe library: its
                                   whole first step, as before round 5); 28 =
                                   the policy's; + 32: FILL reads
                                   every step with the default policy, AUTO's
                                   choice for packed fixed images below 320 B
                                   and variable means up to 448 B; + 64: FILL
                                   with a results buffer writes the results
                                   only and the write-through field pass
                                   stores the fields, AUTO's for packed fixed
                                   images of 320 B - 1 KiB and gapped ones
                                   from 512 B; + 128, libtcpck_probe.so only:
                                   FILL stores each field's whole 64-B block
                                   from the stream's registers, written
                                   through -- images >= 64 B, MODE_REF, no
                                   gaps, not with + 32 / + 64; measured slower
                                   than AUTO)
                                   | (blocks per CU cap << 8: LDS padding)
                                   | (grid oversubscription << 16: 0 = by batch
                                   size, 1 = none, M = M x the resident grid)   */

#define TCPCK_KERNEL_GSTREAM 9 /* MODE_REF, all ops: fixed stride == len, len a
                                  power of two in [32, 1024], 16-B aligned
                                  arena; G = len / 16 lanes per image, DPP group
                                  sums, no boundary resolution; param = variant
                                  (0: 4 steps in flight, 1: 8, 2: 2; + 4: default
                                  block order, else XCD-chunked; 0x80: 4 in
                                  flight with default-policy loads, AUTO's FILL
                                  choice up to 256 B; tuning: 0x10/0x20/0x40
                                  results stored with the default/nt/sc1
                                  policy, 0x100: 0x80 + 0x10, 0x200-0x202:
                                  FILL field lines with default-policy loads,
                                  U4/U8/U2; FILL only: 0x400/0x800/0xC00 every
                                  16-B chunk written back whole with the
                                  nt/default/sc1 store policy, U4; 0x401: nt,
                                  U8, AUTO's FILL choice up to 128 B)
                                  | (grid oversubscription << 16: 0 = by batch
                                  size, 1 = none, M = M x the resident grid)    */
#define TCPCK_KERNEL_SSTREAM 10 /* all ops: slotted layouts -- fixed slots
                                   (stride % 16 == 0) or any offset list -- read
                                   as one compacted stream per wave (lines
                                   wholly in a gap are never read; runs of <= 128
                                   images for offset lists); REF and RFC 1071
                                   (images < 128 KiB); param = variant (0:
                                   policy = 4 steps in flight, scattered block
                                   order; RECEIVE into a header array: + 32
                                   each header from the stream's registers
                                   (AUTO's for images up to 256 B); FILL with
                                   a results buffer: + 128 the results only,
                                   the write-through field pass stores the
                                   fields (AUTO's from 512 B).  Probe library
                                   only: 1: 4 steps in flight, 2: 8; + 4:
                                   default block order, + 8: scattered, else
                                   XCD-chunked; + 64 with + 32: write-through
                                   header stores; without + 32 the headers are
                                   converted after the run's verdicts, + 16
                                   with the stream read with the default cache
                                   policy)
                                   | (grid oversubscription << 16: 0 = by batch
                                   size, M = M x the resident grid)             */
#define TCPCK_KERNEL_RVSTREAM 13 /* libtcpck_probe.so only (measured below
                                   vvstream on C3):
                                   offset lists of packed images (PACKED: the
                                   lengths of a run must add up to its span,
                                   else the run takes an exact per-image pass),
                                   MODE_REF, CHECKSUM / VERIFY: rstream's scalar
                                   boundary walk over the lengths, one run per
                                   wave; param = variant (0: policy = 4 steps in
                                   flight, XCD-chunked order, the run's first
                                   line L2-kept; probe library: 1: 8 in flight,
                                   2: 2; 3 / 4: 0 / 2 with each run's span from
                                   a run-start table built by a pass before the
                                   stream -- packed batches only, one table
                                   buffer per device) | (grid oversubscription
                                   << 16: 0 = by batch size, runs >= 4 KiB)     */
/* FILL in TCPCK_MODE_REF with a results buffer, any kernel (param bits, OR'ed
 * with the kernel's own param):
 *   TCPCK_PARAM_FILL_UPDATE    the kernel's CHECKSUM pass, then a field pass that
 *                              derives each zero-field checksum from the old field
 *                              (c = ~(~C - f) mod 2^16) and stores it (AUTO takes
 *                              it for fixed layouts with stride > len and images
 *                              above 4 KiB, and for packed variable layouts of
 *                              448 B .. 32 KiB typical images; fixed layouts
 *                              need stride >= 30)
 *   TCPCK_PARAM_FILL_INSTREAM  with TCPCK_KERNEL_AUTO: the field zeroed and
 *                              stored in the stream instead -- neither the
 *                              update form nor the deferred-field forms (rstream
 *                              25, vvstream + 64, sstream + 128)
 * Under TCPCK_KERNEL_AUTO a FILL without a results buffer (d_out NULL, the
 * reference's call shape) whose form reads the results back (the update form,
 * the deferred-field forms) writes them into a context scratch slot (tcpck.h:
 * 4 slots of 16 MiB, allocated on first use, 8M images per launch chunk), so
 * it takes the same forms as a FILL with one; the other forms launch with no
 * results at all.  A batch of more than 8M images on an offset list runs in
 * 8M-image chunks whose layout hint keeps the flags and length bounds and
 * scales total_bytes with the chunk's count, so AUTO sees the batch's own
 * typical image in every chunk. */
#define TCPCK_PARAM_FILL_UPDATE (1 << 28)
#define TCPCK_PARAM_FILL_INSTREAM (1 << 29)
/* RECEIVE into a header array (tcpck_batch_receive_ex): where the VERIFY kernel
 * is sstream it writes the headers itself (see TCPCK_KERNEL_SSTREAM); this bit
 * keeps the separate header pass instead, under TCPCK_KERNEL_AUTO too. */
#define TCPCK_PARAM_RECEIVE_TWO_PASS (1 << 30)
int tcpck_batch_fixed_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena,
                         uint64_t stride, uint32_t len, uint64_t count, void *d_out,
                         int kernel, int param, tcpck_stream stream);
/* tcpck_batch_segment (tcpck.h) with param = variant | (grid << 16).  Variant 0
 * (+ 8: default block order, else XCD-chunked) is AUTO's form: segments below
 * 8 KiB one run of whole images per wave, 4 steps in flight, default-policy
 * loads and stores, M x the resident grid with M the power of two nearest runs
 * of 3 KiB of output (grid bits: M instead); segments of 8 KiB and more one
 * block of 4 (16 KiB and more: 16) waves per image, up to 64 x the resident
 * grid (grid bits: that multiple instead).  Variants 1-7 and 0x40 / 0x80 (store
 * and load policies, 8 steps in flight, waves per image) are in
 * libtcpck_probe.so only. */
int tcpck_batch_segment_ex(tcpck_ctx *ctx, int mode, const void *d_payload, uint64_t payload_bytes,
                           uint32_t seg, const void *hdr, uint32_t seq0, void *d_images, uint64_t stride,
                           uint16_t *d_out, int param, tcpck_stream stream);

int tcpck_batch_var_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena,
                       const uint64_t *d_offsets, const uint32_t *d_lengths,
                       uint64_t count, void *d_out, const tcpck_layout *layout,
                       int kernel, int param, tcpck_stream stream);

/* tcpck_batch_receive (tcpck.h) with an explicit kernel / param for the VERIFY
 * pass (param may carry TCPCK_PARAM_RECEIVE_TWO_PASS). */
int tcpck_batch_receive_ex(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                           const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                           void *d_hdr, const tcpck_layout *layout, int kernel, int param, tcpck_stream stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* TCPCK_TUNING_H_ */
