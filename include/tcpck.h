/*
 * tcpck.h -- C-ABI of the MI355X (gfx950) TCP checksum library, libtcpck.so.
 *
 * Drop-in boundary for the one per-byte hot path of filixi/TCP-stack:
 *
 *   friend uint16_t CalculateChecksum(const TcpPacket &)   include/tcp-header.h:252-263
 *
 * and its three call sites:
 *
 *   send, insert   src/socket-manager.cc:9-10, include/socket-manager.h:259-260
 *                  (zero TcpHeader::Checksum(), compute, store raw)
 *   receive,verify include/socket-manager.h:182   (CalculateChecksum(pkt) == 0)
 *
 * Plain pointers and sizes only.  Every entry point returns an int status
 * (TCPCK_OK = 0, negative on error) and never throws.  The reference has no
 * error path (odd sizes are an out-of-bounds read, tcp-header.h:259-260); here
 * odd lengths are rejected with TCPCK_EINVAL where the host can see them, and
 * documented as a precondition for device-resident descriptor arrays.
 *
 * Arithmetic (mode TCPCK_MODE_REF, the default and the parity mode):
 *     checksum = ~(sum of little-endian u16 words of the image mod 2^16) & 0xFFFF
 * i.e. the reference's u32 accumulation with no end-around-carry fold.  The
 * opt-in TCPCK_MODE_RFC1071 folds carries (one's complement, RFC 1071); it is
 * NOT what the reference computes.
 *
 * An "image" is the 32-byte TcpHeader (12-byte pseudo-header + 20-byte TCP
 * header, tcp-header.h:188-190) followed by the payload, contiguous, exactly the
 * bytes of TcpPacket::GetBuffer() (tcp-header.h:265-267).  The checksum field is
 * bytes 28-29 (TcpHeader::Checksum(), tcp-header.h:177), stored raw (host order,
 * no htons), as the reference does.
 */
#ifndef TCPCK_H_
#define TCPCK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCPCK_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define TCPCK_OK 0
#define TCPCK_EINVAL (-22)   /* bad argument: odd length/offset, null, overflow */
#define TCPCK_ENOMEM (-12)   /* host or device allocation failed               */
#define TCPCK_ENODEV (-19)   /* no such HIP device                             */
#define TCPCK_EHIP (-1000)   /* HIP runtime error e: returned as TCPCK_EHIP - e */

/* ---- arithmetic modes --------------------------------------------------- */
#define TCPCK_MODE_REF 0     /* bit-exact to tcp-header.h:252-263 (mod 2^16)   */
#define TCPCK_MODE_RFC1071 1 /* opt-in one's complement, end-around carry      */

/* ---- batch operations --------------------------------------------------- */
#define TCPCK_OP_CHECKSUM 0  /* out[k] (u16) = checksum of image k              */
#define TCPCK_OP_FILL 1      /* zero bytes 28-29 of image k, compute, store the
                                result there in place (send path); out[k] (u16)
                                also receives it unless out == NULL.  len >= 30.
                                Only bytes 28-29 change; for packed images of
                                <= 128 B the kernel may store the image's other
                                16-B chunks back unchanged (never bytes outside
                                an image)                                       */
#define TCPCK_OP_VERIFY 2    /* out[k] (u8) = (checksum of image k == 0)
                                (receive path, socket-manager.h:182)            */
#define TCPCK_OP_RECEIVE 3   /* ReceivePacket's front half (socket-manager.h:
                                182-184): out[k] (u8) as VERIFY, on the network-
                                order image; then image k's 32-B header is
                                converted to host order in place (TcpHeaderN2H,
                                see tcpck_batch_header_swap).  Images >= 32 B.
                                The VERIFY pass, then the header pass, on the
                                stream.  Device batches only (not
                                tcpck_host_batch_*).  tcpck_batch_receive can
                                write the headers to a dense array instead. */

/* ---- layout hints (tcpck_layout.flags) ---------------------------------- */
#define TCPCK_LAYOUT_PACKED 1u /* images are back to back in index order:
                                  offsets[k+1] == offsets[k] + lengths[k]      */
#define TCPCK_LAYOUT_SORTED 2u /* images in index order, apart: offsets[k+1] >=
                                  offsets[k] + lengths[k] (receive slots, rings);
                                  a wrong SORTED hint costs speed, never
                                  correctness                                  */

/* Optional description of a variable-length batch.  Zero fields = unknown.
 * Used only to choose a kernel; a wrong hint never changes results, except
 * that TCPCK_LAYOUT_PACKED must be true when set. */
typedef struct tcpck_layout {
  uint64_t total_bytes; /* sum of lengths                                     */
  uint32_t min_len;     /* smallest image length                              */
  uint32_t max_len;     /* largest image length                               */
  uint32_t flags;       /* TCPCK_LAYOUT_*                                     */
  uint32_t reserved;
} tcpck_layout;

typedef struct tcpck_ctx tcpck_ctx;
typedef void *tcpck_stream; /* a hipStream_t; NULL = the device's null stream */

/* ---- library ------------------------------------------------------------ */
int tcpck_abi_version(void);
const char *tcpck_strerror(int status);
/* 1 when the library's gfx950 code object can run on `device`, else 0. */
int tcpck_device_supported(int device);

/* ---- context: one per device; owns no hidden global HIP state ------------
 * A FILL without a results buffer (the reference's call shape,
 * socket-manager.cc:9-10 stores into the packet only) whose AUTO form reads
 * the results back writes them to one of the context's 4 results-scratch
 * slots of 16 MiB (8M images per launch chunk), allocated on the first such
 * call, so it runs the same two-pass forms as a FILL with a buffer.  FILLs
 * on different streams take different slots and overlap; a slot's reuse waits
 * (on the caller's stream, asynchronously) for its previous user's work.  On a
 * stream under capture (HIP graphs), or when the slots cannot be allocated,
 * such a FILL runs AUTO's in-stream form instead (same bytes, no slot, no
 * event); a refused allocation is tried again 64 out-less FILLs later.
 * Context creation allocates nothing on the device. */
int tcpck_ctx_create(int device, tcpck_ctx **out);
int tcpck_ctx_destroy(tcpck_ctx *ctx);
int tcpck_ctx_device(const tcpck_ctx *ctx);

/* ---- single image, host memory (the per-packet drop-in) ------------------
 * Replaces CalculateChecksum(const TcpPacket&) (tcp-header.h:252-263) for one
 * packet at a time: one image is far below a kernel launch in cost, so it is
 * computed on the calling thread.  Reentrant, no allocation. */
int tcpck_checksum16(const void *image, size_t len, int mode, uint16_t *out);
/* Send-side insertion on one host image (socket-manager.cc:9-10). */
int tcpck_fill16(void *image, size_t len, int mode, uint16_t *out);
/* Incremental update of a stored checksum when one aligned u16 word of the
 * image changes from old_word to new_word (retransmit ACK rewrite,
 * socket-internal.h:376-377), exact in the selected mode. */
uint16_t tcpck_update16(uint16_t checksum, uint16_t old_word, uint16_t new_word, int mode);

/* ---- batched, device-resident: the hot path ------------------------------
 * Fixed stride: image k is d_arena[k*stride, k*stride + len).
 * d_arena even (the u16 words of an image sit at even addresses, as in any
 * malloc'd TcpPacket buffer); stride and len even (stride >= len); count images.
 * d_out: u16[count] (CHECKSUM/FILL) or u8[count] (VERIFY); FILL takes NULL
 * (the results then go to the context's scratch, see tcpck_ctx_create).
 * Asynchronous on `stream`; nothing is allocated; no host synchronisation. */
int tcpck_batch_fixed(tcpck_ctx *ctx, int op, int mode, void *d_arena,
                      uint64_t stride, uint32_t len, uint64_t count, void *d_out,
                      tcpck_stream stream);

/* Variable length: image k is d_arena[d_offsets[k], d_offsets[k] + d_lengths[k]).
 * d_arena even; offsets and lengths must be even (precondition: the device
 * arrays are not read by the host).  `layout` may be NULL. */
int tcpck_batch_var(tcpck_ctx *ctx, int op, int mode, void *d_arena,
                    const uint64_t *d_offsets, const uint32_t *d_lengths,
                    uint64_t count, void *d_out, const tcpck_layout *layout,
                    tcpck_stream stream);

/* ---- batched retransmit: ACK rewrite, incremental checksum update --------
 * The resend path: ResendPredicate rewrites the ACK number of each queued
 * packet (include/socket-internal.h:376-377, AcknowledgementNumber() =
 * htonl(rcv_nxt)) and SendPacket then recomputes the whole checksum
 * (src/socket-manager.cc:9-10).  Here, for every image k: bytes 20-23
 * (TCPCK_ACK_OFFSET, AcknowledgementNumber) := htonl(ack_k), and the stored
 * checksum (bytes 28-29) is updated from the two old and new u16 words --
 * C' = ~(~C - old + new) mod 2^16 (TCPCK_MODE_REF) or RFC 1624 eqn. 3
 * (TCPCK_MODE_RFC1071) -- which equals the full recompute whenever C was the
 * valid checksum of the old image (e.g. written by TCPCK_OP_FILL).
 * d_offsets == NULL: image k at k * stride (stride even, >= 30); else image k
 * at d_offsets[k] (precondition: even, image >= 30 B).  d_acks: u32[count],
 * host order; NULL: every image gets `ack`.  d_out: u16[count] receiving C'
 * (may be NULL).  Asynchronous on `stream`. */
#define TCPCK_ACK_OFFSET 20
int tcpck_batch_set_ack(tcpck_ctx *ctx, int mode, void *d_arena, const uint64_t *d_offsets,
                        uint64_t stride, uint64_t count, const uint32_t *d_acks, uint32_t ack,
                        uint16_t *d_out, tcpck_stream stream);

/* ---- batched header byte order: TcpHeaderN2H / TcpHeaderH2N -------------
 * ReceivePacket verifies the network-order image and then converts its header
 * to host order (include/socket-manager.h:182-184); TcpHeaderN2H and
 * TcpHeaderH2N (include/tcp-header.h:193-221) are the same permutation: u32
 * byte swaps of bytes 0-3, 4-7, 16-19, 20-23 (addresses, seq, ack) and u16
 * swaps of 10-11, 12-13, 14-15, 26-27, 30-31 (TcpLength, ports, window,
 * urgent pointer); bytes 8-9, 24-25, 28-29 and the payload are untouched.
 * Applied in place to the first 32 bytes of every image: image k at
 * k * stride (d_offsets == NULL; stride even, >= 32) or at d_offsets[k]
 * (precondition: even, image >= 32 B).  d_arena even.  A receive batch is
 * tcpck_batch_*(TCPCK_OP_VERIFY) then this call on the same stream.
 * Asynchronous on `stream`. */
#define TCPCK_HEADER_BYTES 32
int tcpck_batch_header_swap(tcpck_ctx *ctx, void *d_arena, const uint64_t *d_offsets,
                            uint64_t stride, uint64_t count, tcpck_stream stream);

/* ---- batched receive: verdicts + host-order headers -----------------------
 * ReceivePacket's front half (include/socket-manager.h:181-185) for a batch:
 * d_ok[k] (u8) = (CalculateChecksum(image k) == 0) on the network-order
 * image, and image k's header in host order (TcpHeaderN2H).  Layout: image k
 * at k * stride, `len` bytes (d_offsets == NULL; len >= 32, even) or at
 * d_offsets[k], d_lengths[k] bytes (precondition: >= 32; `layout` as in
 * tcpck_batch_var, may be NULL).  d_arena even.
 *   d_hdr == NULL: headers converted in place (== TCPCK_OP_RECEIVE);
 *   d_hdr != NULL: 4-B aligned, 32 * count bytes: header k in host order at
 *                  d_hdr + 32 k, the arena left as received.  One dense array
 *                  of whole lines instead of one partial-line write per image
 *                  (the cheaper form on this part, profiles/DESIGN_history_r01-r04.md "Receive path").
 * Asynchronous on `stream`. */
int tcpck_batch_receive(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                        const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count,
                        uint8_t *d_ok, void *d_hdr, const tcpck_layout *layout, tcpck_stream stream);

/* ---- batched segmentation: send stream -> checksummed images -------------
 * The data-segment send path in one device pass.  The reference, per segment:
 * TcpSendingBuffer::GetAsTcpPacket(0, window) cuts the next <= window bytes
 * off the send stream into a fresh packet with TcpLength = len
 * (include/tcp-buffer.h:82-98); Estab sets ACK, seq = snd_nxt (then snd_nxt
 * += len) and ack (src/state.cc:167-184); SetSource/SetDestination and
 * TcpHeaderH2N (include/socket-internal.h:186-199); SendPacketsForSending
 * zeroes and stores the checksum (include/socket-manager.h:259-260).  Here:
 *   n = ceil(payload_bytes / seg) images, image k at d_images + k * stride:
 *     bytes 0-31  = hdr (a 32-B network-order header: the connection's fields
 *                   as TcpHeaderH2N leaves them) with TcpLength (10-11) =
 *                   htons(len_k), seq (16-19) = htonl(seq0 + k * seg) and the
 *                   checksum (28-29) of the image (raw, as the reference);
 *     bytes 32..  = d_payload[k * seg, k * seg + len_k), len_k = seg except
 *                   the last (the rest); the slot's bytes after the image = 0.
 * payload_bytes even; seg a multiple of 4 in [4, 65532]; stride a multiple of
 * 16, >= 32 + seg; d_payload 4-B and d_images 16-B aligned; hdr a host pointer
 * (read during the call).  d_out: u16[n] checksums (may be NULL).  Both modes
 * (RFC 1071 folds the same sums).  Asynchronous on `stream`. */
int tcpck_batch_segment(tcpck_ctx *ctx, int mode, const void *d_payload, uint64_t payload_bytes,
                        uint32_t seg, const void *hdr, uint32_t seq0, void *d_images, uint64_t stride,
                        uint16_t *d_out, tcpck_stream stream);

/* ---- batched, host memory (end to end incl. PCIe) ------------------------
 * Segments start and end in host memory (the loopback/socket buffers of
 * network-service.cc / tcp-buffer.h).  The batch is split into chunks that are
 * streamed H2D -> kernel -> D2H on two ctx-owned HIP streams with ctx-owned
 * device staging buffers.  Synchronous: returns when h_out (and, for FILL,
 * h_arena) hold the results.  Host buffers should be pinned
 * (tcpck_host_alloc) for full PCIe rate.  offsets/lengths are host arrays. */
int tcpck_host_batch_fixed(tcpck_ctx *ctx, int op, int mode, void *h_arena,
                           uint64_t stride, uint32_t len, uint64_t count,
                           void *h_out);
int tcpck_host_batch_var(tcpck_ctx *ctx, int op, int mode, void *h_arena,
                         const uint64_t *h_offsets, const uint32_t *h_lengths,
                         uint64_t count, void *h_out);
/* The same host batch over several contexts at once -- one per GPU of the
 * node, each with its own PCIe link (independent segments, no
 * exchange step): contiguous shards, equal image counts (fixed) or balanced by
 * bytes (variable, over h_lengths), each run by tcpck_host_batch_* on its own
 * host thread (the first on the calling thread).  Results land in h_out by
 * index as from one context.  Synchronous; returns the first failing shard's
 * status.  A context listed twice runs its shards one after the other. */
int tcpck_host_batch_fixed_multi(tcpck_ctx *const *ctxs, int n_ctx, int op, int mode, void *h_arena,
                                 uint64_t stride, uint32_t len, uint64_t count, void *h_out);
int tcpck_host_batch_var_multi(tcpck_ctx *const *ctxs, int n_ctx, int op, int mode, void *h_arena,
                               const uint64_t *h_offsets, const uint32_t *h_lengths, uint64_t count,
                               void *h_out);
/* Bytes of device staging per chunk used by the host batch functions. */
int tcpck_ctx_set_chunk_bytes(tcpck_ctx *ctx, uint64_t bytes);

/* ---- memory helpers (for C/C++ callers without another allocator) -------- */
int tcpck_host_alloc(size_t bytes, void **out);   /* pinned host memory   */
int tcpck_host_free(void *p);
int tcpck_device_alloc(tcpck_ctx *ctx, size_t bytes, void **out);
int tcpck_device_free(tcpck_ctx *ctx, void *p);
int tcpck_memcpy_h2d(tcpck_ctx *ctx, void *dst, const void *src, size_t bytes);
int tcpck_memcpy_d2h(tcpck_ctx *ctx, void *dst, const void *src, size_t bytes);
int tcpck_stream_sync(tcpck_ctx *ctx, tcpck_stream stream);

/* ---- synthetic workload generator (benchmarks/tests; not the hot path) ----
 * Writes images with the send path's 32-byte header (127.0.0.1:15500 ->
 * 127.0.0.1:15501, PTCL 6, TcpLength = payload, seq = 1000 + index, ACK,
 * window 1024, network order, checksum 0) and a payload drawn from splitmix64
 * keyed by (seed, first_index + k) -- any shard is reproducible on its own.
 * kind: 0 random payload, 1 all-zero payload, 2 all-0xFF payload. */
int tcpck_synth_fixed(void *d_arena, uint64_t stride, uint32_t len, uint64_t count,
                      uint64_t seed, uint64_t first_index, int kind, tcpck_stream stream);
int tcpck_synth_var(void *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                    uint32_t max_len, uint64_t count, uint64_t seed, uint64_t first_index,
                    int kind, tcpck_stream stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* TCPCK_H_ */
