// tcpck_internal.h -- private interface between the C-ABI layer (tcpck_api.hip)
// and the gfx950 kernels (tcpck_kernels.hip, tcpck_rstream.hip, tcpck_vvstream.hip).
// Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tcpck {

enum Op : int { kChecksum = 0, kFill = 1, kVerify = 2 };
enum Mode : int { kRef = 0, kRfc1071 = 1 };

// ---- seg kernel: any layout, G lanes per image, U loads of 16 B in flight ----
enum SegShape : int {
  kShapeSmall = 0,   // G = 8,  U = 2  : images up to ~256 B
  kShapeMss = 1,     // G = 16, U = 6  : images up to ~4 KiB (Ethernet MSS)
  kShapeJumbo = 2,   // G = 64, U = 4  : 4-6 KiB images
  kShapeWave2 = 3,   // G = 64, U = 2  : tuning
  kShapeG32 = 4,     // G = 32, U = 3  : tuning
  kShapeG4 = 5,      // G = 4,  U = 8  : tuning
  kShapeW4 = 6,      // 4 waves per image, U = 4  : jumbo images
  kShapeW8 = 7,      // 8 waves per image, U = 4  : jumbo images
  kShapeW16 = 8,     // 16 waves per image, U = 2 : jumbo images
  kShapeW16U4 = 9,   // 16 waves per image, U = 4 : tuning
  kShapeW2 = 10,     // 2 waves per image, U = 4  : jumbo images
  kNumShapes = 11
};

struct SegArgs {
  uint8_t *arena;            // image bytes (device)
  const uint64_t *offsets;   // variable layout: byte offset of image k (device)
  const uint32_t *lengths;   // variable layout: byte length of image k (device)
  uint64_t stride;           // fixed layout: image k at k*stride
  uint64_t base;             // subtracted from offsets[k] (chunked host batches)
  uint64_t count;            // images
  void *out;                 // u16[count] or u8[count] (verify); may be null for fill
  uint32_t len;              // fixed layout: image length
  uint32_t oversub;          // grid = resident blocks x this (0/1: one block per resident slot)
  uint32_t order;            // block order (dev::ordered_block; 0xFF default)
  uint32_t rot;              // W-wave shapes: image k's chunks read from chunk ((k rot) mod (n / 64)) 64 on,
                             // wrapping (0: from chunk 0) -- concurrent blocks at different offsets
};

SegShape shape_for_len(uint64_t typical_len);
hipError_t launch_seg(int op, int mode, bool fixed, SegShape shape, const SegArgs &a,
                      uint32_t num_cus, hipStream_t stream);

// ---- run kernels: one contiguous run of whole images per wave ---------------
// Packed and fixed layouts for vvstream (tcpck_vvstream.hip).
struct RunArgs {
  uint8_t *arena;
  const uint64_t *offsets;   // variable layout (packed: offsets[k+1] == offsets[k] + lengths[k])
  const uint32_t *lengths;
  uint64_t stride;           // fixed layouts: image k at k * stride
  uint32_t len;              // fixed layouts: image length (<= stride)
  uint64_t base;             // subtracted from offsets[k] (chunked host batches)
  uint64_t count;
  void *out;
  uint32_t oversub;          // grid = resident blocks x this (0 = by size)
  uint64_t total_bytes;      // batch byte span hint (0 = unknown)
  uint32_t blocks_per_cu;    // vvstream: occupancy cap (LDS padding) and grid base, 0 = by resources
  int mode;                  // vvstream: kRef or kRfc1071
  uint8_t *hdr;              // sstream VERIFY: host-order header k also to hdr + 32 k (receive)
  uint64_t *dbg;             // vvstream, probe library only: 8 x u64 of time stamps per wave (tcpck_probe.h)
};

// Fixed stride == len for rstream (tcpck_rstream.hip).
struct FixedStreamArgs {
  uint8_t *arena;
  uint64_t stride;  // == image length
  uint64_t count;
  void *out;
  uint64_t *dbg;    // optional per-wave {start, end} s_memrealtime stamps (timing builds)
  uint32_t blocks_per_cu;  // optional occupancy cap (0 = as many as fit)
  uint32_t oversub;        // grid = resident blocks x this (0 = by size, 1 = none)
  uint64_t per_wave;       // run split, set by the launcher: count = per_wave * waves + rem,
  uint64_t rem;            // wave w owns per_wave + (w < rem) images (no 64-bit division on device)
  uint32_t order;          // block order (dev::ordered_block; 0xFF default)
  int mode;                // kRef, or kRfc1071 (variant 20 only)
  uint32_t defer_field;    // kFill: results to out only, the fields left for launch_patch_fields
  uint8_t *side;           // probe variants 33 / 34 (kFill): each field's 64-B block, checksum in place, to
                           // side[64 k, 64 k + 64) for launch_side_copy (nullptr otherwise)
  uint32_t side_nt;        // ... those side stores nt (else the default policy)
};

// Fixed stride == len == S, S a power of two in [32, 1024], 16-B aligned arena
// (tcpck_gstream.hip): G = S / 16 lanes per image.
struct GroupStreamArgs {
  uint8_t *arena;
  uint32_t len;      // == stride
  uint64_t count;
  void *out;
  uint32_t oversub;  // grid = resident blocks x this (0 = by size)
  uint32_t order;    // block order, set by launch_gstream
  uint64_t per_wave; // step split, set by the launcher: steps = per_wave * waves + rem
  uint64_t rem;
};
bool gstream_applies(const uint8_t *arena, uint64_t stride, uint32_t len);
// variant: 0 = 4 steps in flight, 1 = 8, 2 = 2; + 4: default block order
// (else XCD-chunked, groups of 16 blocks); kGstreamDefaultLoads: 4 in flight,
// loads with the default cache policy instead of nt (AUTO for FILL <= 256 B);
// tuning: 0x10 / 0x20 / 0x40 results through a buffer resource with the
// default / nt / sc1 policy, 0x100 default-policy loads + 0x10, 0x200-0x202
// FILL with default-policy loads for the field lines only (U4 / U8 / U2);
// FILL only: 0x400 / 0x800 / 0xC00 every chunk written back whole with the
// nt / default / sc1 store policy (U4), kGstreamWriteBack: nt, U8 (AUTO for
// FILL <= 128 B)
constexpr int kGstreamDefaultLoads = 0x80;
constexpr int kGstreamWriteBack = 0x401;
hipError_t launch_gstream(int op, int variant, const GroupStreamArgs &a, uint32_t num_cus, hipStream_t stream);

// ---- rstream (fixed stride == len): one run per wave, scalar boundary walk.
// variant: 0 = 4 loads in flight, 1 = 2, 2 = 8, 3 = 4 with per-wave time stamps,
// 4-8 issue-priority experiments, 9-13 v_dot2 sums and/or buffer loads (10 = policy)
hipError_t launch_rstream(int op, int variant, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream);
// ---- vvstream (prefix table), MODE_REF, all ops: packed variable layouts
// (fixed = false) or fixed strides (fixed = true: a.stride >= a.len).
// variant 0 U4 byte split, 1 U8, 2 U4 count split, 3 U8 (fixed: 0/2 U4, 1/3 U8),
// 4 = policy (oversubscription, split and loads in flight by size)
hipError_t launch_vvstream(int op, int variant, bool fixed, const RunArgs &a, uint32_t num_cus, hipStream_t stream);
// Packed offset lists with rstream's scalar boundary walk (tcpck_rvstream.hip):
// CHECKSUM / VERIFY, reference mode; variant 0 = the policy.
hipError_t launch_rvstream(int op, int variant, const RunArgs &a, uint32_t num_cus, hipStream_t stream);
// ---- sstream (compacted slot stream), MODE_REF, all ops: images anywhere in
// the arena -- fixed slots (fixed = true: stride % 16 == 0, stride >= len) or
// offsets + lengths (fixed = false; runs of <= 128 images).  variant: 0 policy
// (U4, scattered block order), 1 U4, 2 U8; + 4: default block order, + 8:
// scattered (else XCD-chunked); + 16 (with a.hdr): the stream read with the
// default cache policy.  a.hdr (VERIFY only): the run's headers in host order
// to the dense array after its verdicts (tcpck_batch_receive).  a.oversub: 0 = by size; a.total_bytes: image bytes hint.
bool sstream_fixed_applies(uint64_t stride, uint32_t len);
hipError_t launch_sstream(int op, int variant, bool fixed, const RunArgs &a, uint32_t num_cus, hipStream_t stream);
// ---- segment (tcpck_segment.hip): send stream -> checksummed images ------
struct SegmentArgs {
  const uint8_t *payload;    // the send stream (4-B aligned)
  uint8_t *images;           // output: image k at k * stride (16-B aligned)
  uint64_t payload_bytes;    // even
  uint64_t count;            // images: ceil(payload_bytes / seg)
  uint16_t *out;             // checksums (may be null)
  uint64_t per_wave, rem;    // run split, set by the launcher
  uint32_t seg;              // payload bytes per image (the last: the rest); % 4 == 0
  uint32_t stride;           // % 16 == 0, >= 32 + seg
  uint32_t nchunk, magic, shift;  // set by the launcher: chunks per slot and q / nchunk
  uint32_t hdr[8];           // 32-B network-order header template (TcpLength, seq, checksum ignored)
  uint32_t seq0;             // sequence number of image 0 (host order)
  uint32_t order;            // block order, set by the launcher
};
// variant: 0 policy (U4, nt stores), 1 U8, 2 default-policy stores, 3 sc1
// stores; + 8 default block order (else XCD-chunked).  oversub: 0 = by size
hipError_t launch_segment(int mode, int variant, SegmentArgs a, uint32_t oversub, uint32_t num_cus,
                          hipStream_t stream);
// ---- retransmit ACK rewrite with incremental checksum update (tcpck_resend.hip) ----
struct AckArgs {
  uint8_t *arena;
  const uint64_t *offsets;  // null: image k at k * stride
  uint64_t stride;
  uint64_t count;
  const uint32_t *acks;     // per-image ACK numbers (host order); null: `ack` for all
  uint32_t ack;
  uint16_t *out;            // new checksums (may be null)
};
hipError_t launch_set_ack(int mode, const AckArgs &a, uint32_t num_cus, hipStream_t stream);

// ---- header byte-order conversion, TcpHeaderN2H == TcpHeaderH2N (tcpck_header.hip) ----
struct HeaderArgs {
  uint8_t *arena;
  const uint64_t *offsets;  // null: image k at k * stride
  uint64_t stride;
  uint64_t count;
  uint8_t *out;             // null: convert in place; else header k -> out[32k, 32k + 32), arena untouched
  uint32_t store_bits;      // probe builds (tcpck_probe_receive_ex), EXTRACT: 1 = write-through
                            // (sc0 sc1 nt) array stores; 2 = two lanes per image, 16-B loads with
                            // cache bits form (bits 4-5); bits 8-9: the array form's image order
};
hipError_t launch_header_swap(const HeaderArgs &a, uint32_t num_cus, hipStream_t stream);

// ---- FILL's field stores as a second pass (tcpck_header.hip) ----
// One lane per image writes bytes 28-29 with a write-through streaming 2-B
// store (nothing else in the arena is read or written).
//   fixed stride (offsets == null): stride >= 30;
//   offset lists: image k at offsets[k] - base, images < 30 B skipped.
// update == 0: sums[k] is the checksum to store (the stream zeroed the field).
// update == 1 (REF mode only): sums[k] is the checksum of image k as it stands,
// field included (a CHECKSUM pass), so the zero-field checksum follows exactly
// from the old field f: c = ~(~C - f) mod 2^16 (tcp-header.h:252-263 is a sum
// mod 2^16); c goes to the field and back to sums[k].  Images < 30 B keep
// their plain checksum and are not written (seg's FILL does the same).
struct PatchArgs {
  uint8_t *arena;
  uint64_t stride;          // image k at k * stride
  const uint64_t *offsets;  // or image k at offsets[k] - base, lengths[k] bytes
  const uint32_t *lengths;
  uint64_t base;
  uint64_t count;
  uint16_t *sums;
  uint64_t lo, hi;          // probe block forms: byte range (relative to arena) their writes may cover
  uint32_t update;          // 1: sums hold CHECKSUM results, derive FILL's from the old field
  uint32_t packed;          // offset lists: the PACKED contract holds (unused by the 2-B pass)
  uint32_t probe_form;      // probe builds (TCPCK_KERNEL_PATCH): a timing form chosen by store_bits
  uint32_t store_bits;      // probe forms: 1 + store cache bits (sc0 1, nt 2, sc1 4; 0 plain) | granularity << 4
  uint32_t reverse;         // the fields in reverse index order (the stream's last lines first)
};
hipError_t launch_patch_fields(const PatchArgs &a, uint32_t num_cus, hipStream_t stream);
// Probe (round 6): FILL's field blocks from a dense side buffer -- image k's
// 64-B block (the stream's bytes, checksum in place; rstream variants 33 / 34)
// copied from side[64 k] to its place, a whole-block write-through store that
// needs no merge read; a block starting before the arena takes the 2-B store
// of sums[k] instead.  Fixed stride >= 128.
hipError_t launch_side_copy(uint8_t *arena, uint64_t stride, uint64_t count, const uint8_t *side,
                            const uint16_t *sums, uint32_t num_cus, hipStream_t stream);


// timing-only streaming micro-kernels (tcpck_diag.hip)
hipError_t launch_diag_stream(int variant, const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus,
                              hipStream_t s);

}  // namespace tcpck
