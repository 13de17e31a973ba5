// tcpck_diag.hip -- streaming micro-kernels for timing experiments only (their
// outputs are not checksums).  Each wave reads one contiguous, 128-B aligned
// run of the buffer, LPB 16-byte chunks per lane per step (a lane's chunks are
// adjacent: lane l covers bytes [16 LPB l, 16 LPB (l+1)) of the step), U steps
// in flight, optionally with the per-step 64-lane DPP scan the checksum
// kernels need.  Answers: how much does per-step (scalar + scan) overhead cost,
// and what does a wider per-lane stride do to the memory pipeline?
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

template <int LPB, int U, bool SCAN>
__global__ void __launch_bounds__(kBlock) diag_stream_kernel(const uint8_t *buf, uint64_t bytes, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  const uint64_t lines = bytes >> 7;
  const uint64_t b0 = (wid * lines / W) << 7;
  const uint64_t b1 = ((wid + 1) * lines / W) << 7;
  if (b0 >= b1) return;
  constexpr uint32_t kStep = 1024u * LPB;
  const uint32_t nsteps = static_cast<uint32_t>((b1 - b0 + kStep - 1) / kStep);
  const uint32_t last_chunk = static_cast<uint32_t>((b1 - b0) >> 4) - 1;
  const uint8_t *base = buf + b0;
  auto ld = [&](uint32_t st, int i) -> u32x4 {
    const uint32_t ci = min(st * (64u * LPB) + lane * LPB + static_cast<uint32_t>(i), last_chunk);
    return dev::load16_nt(base + 16 * static_cast<uint64_t>(ci));
  };
  u32x4 ring[U][LPB];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < LPB; ++i) ring[u][i] = ld(static_cast<uint32_t>(u), i);
  uint32_t carry = 0;
  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t t = 0;
#pragma unroll
      for (int i = 0; i < LPB; ++i) t += dev::ref_chunk_sum(ring[u][i]);
      if constexpr (SCAN) {
        const uint32_t incl = dev::wave_inclusive_scan(t);
        carry += dev::read_lane(incl, 63);
      } else {
        carry += t;
      }
#pragma unroll
      for (int i = 0; i < LPB; ++i) ring[u][i] = ld(g + u + U, i);
    }
  }
  if (lane == 0) out[wid] = carry;
}

template <int LPB, int U, bool SCAN>
hipError_t launch_one(const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(diag_stream_kernel<LPB, U, SCAN>);
  hipLaunchKernelGGL((diag_stream_kernel<LPB, U, SCAN>), dim3(per_cu * num_cus), dim3(kBlock), 0, s, buf, bytes, out);
  return hipGetLastError();
}

}  // namespace

// variant: LPB x U x scan: 0 = 1x4 scan, 1 = 1x4 no scan, 2 = 2x2 scan, 3 = 2x2 no scan,
// 4 = 4x1 scan, 5 = 2x4 scan, 6 = 4x2 scan, 7 = 1x2 scan
hipError_t launch_diag_stream(int variant, const uint8_t *buf, uint64_t bytes, uint32_t *out, uint32_t num_cus,
                              hipStream_t s) {
  switch (variant) {
    case 0: return launch_one<1, 4, true>(buf, bytes, out, num_cus, s);
    case 1: return launch_one<1, 4, false>(buf, bytes, out, num_cus, s);
    case 2: return launch_one<2, 2, true>(buf, bytes, out, num_cus, s);
    case 3: return launch_one<2, 2, false>(buf, bytes, out, num_cus, s);
    case 4: return launch_one<4, 1, true>(buf, bytes, out, num_cus, s);
    case 5: return launch_one<2, 4, true>(buf, bytes, out, num_cus, s);
    case 6: return launch_one<4, 2, true>(buf, bytes, out, num_cus, s);
    case 7: return launch_one<1, 2, true>(buf, bytes, out, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
