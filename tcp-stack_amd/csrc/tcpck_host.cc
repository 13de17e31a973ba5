// tcpck_host.cc -- the host single-image word sum behind tcpck_checksum16 /
// tcpck_fill16 (include/tcpck.h): the per-packet drop-in's CalculateChecksum
// (reference include/tcp-header.h:252-263), called on the caller's thread for
// every packet the stack sends or receives one at a time (C1, the loopback
// path: socket-manager.cc:9-10, socket-manager.h:182).
//
// Plain host C++ (no HIP): built with clang++ into libtcpck.so beside the HIP
// translation units.  Returns the exact sum of the image's little-endian u16
// words; tcpck_api.hip finishes it (REF: ~sum mod 2^16; RFC 1071: folded).
//
//   * AVX2 (chosen once at run time, __builtin_cpu_supports): 64 B per
//     iteration into two sets of eight u32 lanes -- each 32-bit lane holds two
//     u16 words, split by a mask and a shift and added; 2^14 iterations add at
//     most 2^14 * 2 * 0xFFFF < 2^32 per lane, so the lanes are widened into a
//     u64 total every 2^14 iterations.  1492-B image: ~51-70 ns against
//     ~154-189 ns for the SWAR form on the build container's core.
//   * SWAR fallback (and the tail below 64 B): 8 bytes per step as two u32
//     lanes in a u64, folded every 2^14 steps.
#include <immintrin.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace tcpck {
namespace host {

namespace {

uint64_t word_sum_swar(const uint8_t *p, size_t n) {
  constexpr uint64_t kLo = 0x0000FFFF0000FFFFull;
  uint64_t total = 0;
  size_t i = 0;
  while (n - i >= 8) {
    uint64_t a = 0;
    const size_t stop = i + std::min<size_t>((n - i) & ~size_t{7}, size_t{8} << 14);
    for (; i < stop; i += 8) {
      uint64_t x;
      std::memcpy(&x, p + i, 8);
      a += (x & kLo) + ((x >> 16) & kLo);
    }
    total += (a & 0xFFFFFFFFull) + (a >> 32);
  }
  for (; i + 1 < n; i += 2) {
    uint16_t w;
    std::memcpy(&w, p + i, 2);
    total += w;
  }
  return total;
}

__attribute__((target("avx2"))) uint64_t word_sum_avx2(const uint8_t *p, size_t n) {
  const __m256i lo = _mm256_set1_epi32(0xFFFF);
  const __m256i zero = _mm256_setzero_si256();
  uint64_t total = 0;
  size_t i = 0;
  while (n - i >= 64) {
    __m256i a0 = zero, a1 = zero;
    const size_t stop = i + std::min<size_t>((n - i) & ~size_t{63}, size_t{64} << 14);
    for (; i < stop; i += 64) {
      const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(p + i));
      const __m256i y = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(p + i + 32));
      a0 = _mm256_add_epi32(a0, _mm256_add_epi32(_mm256_and_si256(x, lo), _mm256_srli_epi32(x, 16)));
      a1 = _mm256_add_epi32(a1, _mm256_add_epi32(_mm256_and_si256(y, lo), _mm256_srli_epi32(y, 16)));
    }
    __m256i s = _mm256_add_epi64(_mm256_unpacklo_epi32(a0, zero), _mm256_unpackhi_epi32(a0, zero));
    s = _mm256_add_epi64(s, _mm256_add_epi64(_mm256_unpacklo_epi32(a1, zero), _mm256_unpackhi_epi32(a1, zero)));
    alignas(32) uint64_t t[4];
    _mm256_store_si256(reinterpret_cast<__m256i *>(t), s);
    total += t[0] + t[1] + t[2] + t[3];
  }
  return total + word_sum_swar(p + i, n - i);
}

using WordSum = uint64_t (*)(const uint8_t *, size_t);

WordSum pick() { return __builtin_cpu_supports("avx2") ? word_sum_avx2 : word_sum_swar; }

}  // namespace

uint64_t word_sum(const uint8_t *p, size_t n) {
  static const WordSum impl = pick();  // thread-safe static init; reentrant afterwards
  return impl(p, n);
}

}  // namespace host
}  // namespace tcpck
