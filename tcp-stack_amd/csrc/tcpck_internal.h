// tcpck_internal.h -- private interface between the C-ABI layer (tcpck_api.hip)
// and the gfx950 kernels (tcpck_kernels.hip).  Not installed, not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tcpck {

enum Op : int { kChecksum = 0, kFill = 1, kVerify = 2 };
enum Mode : int { kRef = 0, kRfc1071 = 1 };

// Kernel shapes for the image-per-group kernel: G lanes cooperate on one
// image, each lane keeps U 16-byte loads in flight per step.
enum SegShape : int {
  kShapeSmall = 0,   // G = 8,  U = 2  : images up to ~256 B
  kShapeMss = 1,     // G = 16, U = 6  : images up to ~2 KiB (Ethernet MSS)
  kShapeJumbo = 2,   // G = 64, U = 4  : larger images (64 KiB jumbo)
  kNumShapes = 3
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
};

// Chooses the shape from a representative image length.
SegShape shape_for_len(uint64_t typical_len);

// Launches the image-per-group kernel.  `max_blocks` caps the grid (the
// kernel grid-strides over images).
hipError_t launch_seg(int op, int mode, bool fixed, SegShape shape, const SegArgs &a,
                      uint32_t max_blocks, hipStream_t stream);

}  // namespace tcpck
