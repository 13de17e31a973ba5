// tcpck_synth.hip -- synthetic segment batches written straight into HBM.
//
// Workload generator for the benchmark and the parity tests (not on the
// checksum path).  Every image is the 32-byte header the reference's send
// path produces, followed by a payload:
//   * header (filixi/TCP-stack tcp-header.h:52-191 layout, after TcpHeaderH2N
//     tcp-header.h:193-206): src 127.0.0.1, dst 127.0.0.1, zero, PTCL 6,
//     TcpLength = payload bytes (tcp-buffer.h:96), sport 15500, dport 15501
//     (main.cc demo ports), seq = first_seq + index, ack 77, flags ACK
//     (bit 107 of the TCP field -> image byte 25 = 0x08, tcp-header.h:129-134),
//     window 1024 (state.cc:43), checksum 0 (bytes 28-29), urgent 0;
//   * payload: splitmix64 keyed by (seed, image index, word index), so any
//     shard of a batch is reproducible on its own, or all-zero /
//     all-0xFF adversarial payloads.
// One thread writes one u16 word; images may start at any even offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcpck.h"

namespace {

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ inline uint16_t bswap16(uint16_t v) { return static_cast<uint16_t>((v >> 8) | (v << 8)); }

// u16 word m (byte 2m) of the 32-byte network-order header.
__device__ inline uint16_t header_word(int m, uint32_t payload, uint32_t seq) {
  switch (m) {
    case 0: return bswap16(0x7F00);           // 127.0  (src 127.0.0.1, htonl)
    case 1: return bswap16(0x0001);           // 0.1
    case 2: return bswap16(0x7F00);           // dst
    case 3: return bswap16(0x0001);
    case 4: return 0x0600;                    // byte 8 zero, byte 9 PTCL = 6
    case 5: return bswap16(static_cast<uint16_t>(payload));  // TcpLength (htons)
    case 6: return bswap16(15500);            // source port
    case 7: return bswap16(15501);            // destination port
    case 8: return bswap16(static_cast<uint16_t>(seq >> 16));
    case 9: return bswap16(static_cast<uint16_t>(seq));
    case 10: return bswap16(0);               // ack 77 = 0x0000004D
    case 11: return bswap16(77);
    case 12: return 0x0800;                   // byte 24 data offset (never set), byte 25 flags = ACK
    case 13: return bswap16(1024);            // window
    default: return 0;                        // checksum (28-29), urgent pointer (30-31)
  }
}

__device__ inline uint16_t payload_word(uint64_t key, uint64_t m, int kind) {
  if (kind == 1) return 0;
  if (kind == 2) return 0xFFFF;
  return static_cast<uint16_t>(splitmix64(key + (m >> 2)) >> (16 * (m & 3)));
}

__global__ void synth_kernel(uint8_t *arena, const uint64_t *offsets, const uint32_t *lengths,
                             uint64_t stride, uint32_t flen, uint64_t count, uint64_t seed,
                             uint64_t first_index, int kind, uint32_t words_per_image) {
  // grid: x over word index within an image (strided), y/z over images
  const uint64_t k = static_cast<uint64_t>(blockIdx.y) + static_cast<uint64_t>(blockIdx.z) * gridDim.y;
  if (k >= count) return;
  const uint64_t off = offsets ? offsets[k] : k * stride;
  const uint32_t len = offsets ? lengths[k] : flen;
  const uint64_t idx = first_index + k;
  const uint64_t key = splitmix64(seed ^ (idx * 0xD1B54A32D192ED03ull));
  const uint32_t payload = len >= 32 ? len - 32 : 0;
  const uint32_t seq = static_cast<uint32_t>(1000 + idx);
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < len / 2 && m < words_per_image;
       m += gridDim.x * blockDim.x) {
    const uint16_t w = m < 16 ? header_word(static_cast<int>(m), payload, seq)
                              : payload_word(key, m - 16, kind);
    *reinterpret_cast<uint16_t *>(arena + off + 2ull * m) = w;
  }
}

int launch(void *d_arena, const uint64_t *d_off, const uint32_t *d_len, uint64_t stride, uint32_t flen,
           uint32_t max_len, uint64_t count, uint64_t seed, uint64_t first, int kind,
           tcpck_stream stream) {
  if (count == 0) return TCPCK_OK;
  const uint32_t words = (max_len + 1) / 2;
  const uint32_t threads = 256;
  uint32_t gx = (words + threads - 1) / threads;
  if (gx == 0) gx = 1;
  const uint64_t gy = count < 65535 ? count : 65535;
  const uint64_t gz = (count + gy - 1) / gy;
  if (gz > 65535) return TCPCK_EINVAL;
  (void)hipGetLastError();  // a stale error from an earlier failed call is not this launch's
  hipLaunchKernelGGL(synth_kernel, dim3(gx, static_cast<uint32_t>(gy), static_cast<uint32_t>(gz)),
                     dim3(threads), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint8_t *>(d_arena), d_off, d_len, stride, flen, count, seed, first,
                     kind, words);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? TCPCK_OK : TCPCK_EHIP - static_cast<int>(e);
}

}  // namespace

extern "C" {

// Fixed-stride synthetic batch (all images `len` bytes at k*stride).
// kind: 0 random payload, 1 zero payload, 2 all-0xFF payload.
int tcpck_synth_fixed(void *d_arena, uint64_t stride, uint32_t len, uint64_t count, uint64_t seed,
                      uint64_t first_index, int kind, tcpck_stream stream) {
  if (!d_arena || (len & 1) || (stride & 1)) return TCPCK_EINVAL;
  return launch(d_arena, nullptr, nullptr, stride, len, len, count, seed, first_index, kind, stream);
}

// Variable-length synthetic batch over device offsets/lengths; max_len bounds lengths[k].
int tcpck_synth_var(void *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                    uint32_t max_len, uint64_t count, uint64_t seed, uint64_t first_index, int kind,
                    tcpck_stream stream) {
  if (!d_arena || !d_offsets || !d_lengths) return TCPCK_EINVAL;
  return launch(d_arena, d_offsets, d_lengths, 0, 0, max_len, count, seed, first_index, kind, stream);
}

}  // extern "C"
