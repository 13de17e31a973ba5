// abi_host_test.cc -- the C ABI's host logic under AddressSanitizer + UBSan
// (VERDICT r05 item 5).  Linked against tcp-stack_amd/libtcpck_asan.so, whose
// HOST code -- argument validation, the host-batch layout scans and chunking,
// the results-scratch bookkeeping past 8M images, the layout-hint sub-ranges,
// the receive/segment/set_ack launchers' arithmetic -- is compiled with
// -fsanitize=address,undefined (tcp-stack_amd/Makefile `asan`; the device code
// is not sanitized).  The error contract it checks is SURVEY §8b's, derived
// from include/tcp-header.h:259-260 (an odd length is an out-of-bounds read in
// the reference; here TCPCK_EINVAL).
//
//   abi_host_test cpu   no device needed: validation of every entry point,
//                       the host single-image paths against a scalar sum
//   abi_host_test gpu   device 0: every batch entry point, incl. the scratch
//                       chunks past 8M images, host batches in many chunks,
//                       several threads; results checked on the host
//
// Prints "ok <n checks>" and exits 0, or names the first failed check.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "tcpck.h"

namespace {

long g_checks = 0;

#define CHECK(cond)                                                                  \
  do {                                                                               \
    ++g_checks;                                                                      \
    if (!(cond)) {                                                                   \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)
#define CHECK_RC(expr, want)                                                          \
  do {                                                                                \
    ++g_checks;                                                                       \
    const int rc_ = (expr);                                                           \
    if (rc_ != (want)) {                                                              \
      std::fprintf(stderr, "FAILED %s:%d: %s = %d (%s), want %d\n", __FILE__, __LINE__, #expr, rc_, \
                   tcpck_strerror(rc_), (want));                                      \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

// The reference arithmetic (tcp-header.h:252-263), restated scalar: the sum of
// little-endian u16 words mod 2^16, complemented; mode 1 folds the carries.
uint16_t scalar16(const uint8_t *p, size_t n, int mode) {
  uint64_t s = 0;
  for (size_t i = 0; i + 1 < n; i += 2) s += static_cast<uint64_t>(p[i]) | (static_cast<uint64_t>(p[i + 1]) << 8);
  if (mode == TCPCK_MODE_RFC1071)
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
  return static_cast<uint16_t>(~s);
}

uint16_t field(const uint8_t *img) { return static_cast<uint16_t>(img[28] | (img[29] << 8)); }

std::vector<uint8_t> random_bytes(size_t n, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<uint8_t> v(n);
  for (auto &b : v) b = static_cast<uint8_t>(rng());
  return v;
}

// ---- no device ----------------------------------------------------------------

void cpu_checks() {
  CHECK(tcpck_abi_version() == TCPCK_ABI_VERSION);
  for (int st : {TCPCK_OK, TCPCK_EINVAL, TCPCK_ENOMEM, TCPCK_ENODEV, TCPCK_EHIP - 1, 5, -7})
    CHECK(tcpck_strerror(st) != nullptr && std::strlen(tcpck_strerror(st)) > 0);

  // single images at every alignment, every even length up to 300 and a few large ones
  const auto buf = random_bytes(70000 + 16, 1);
  for (int mode : {TCPCK_MODE_REF, TCPCK_MODE_RFC1071}) {
    for (size_t a = 0; a < 8; ++a) {
      std::vector<size_t> lens;
      for (size_t n = 0; n <= 300; n += 2) lens.push_back(n);
      for (size_t n : {1490, 1492, 4096, 9000, 65534, 65536, 70000}) lens.push_back(n);
      for (size_t n : lens) {
        // a heap copy of exactly n bytes: ASan reports any read past it
        std::vector<uint8_t> img(buf.begin() + a, buf.begin() + a + n);
        uint16_t c = 0;
        CHECK_RC(tcpck_checksum16(img.data(), n, mode, &c), TCPCK_OK);
        CHECK(c == scalar16(img.data(), n, mode));
      }
    }
  }
  uint16_t c = 0;
  CHECK_RC(tcpck_checksum16(nullptr, 0, 0, &c), TCPCK_OK);
  CHECK(c == 0xFFFF);
  CHECK_RC(tcpck_checksum16(buf.data(), 59, 0, &c), TCPCK_EINVAL);  // odd: tcp-header.h:259-260
  CHECK_RC(tcpck_checksum16(nullptr, 2, 0, &c), TCPCK_EINVAL);
  CHECK_RC(tcpck_checksum16(buf.data(), 2, 0, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_checksum16(buf.data(), 2, 7, &c), TCPCK_EINVAL);

  // fill16: a rejected call leaves the image untouched
  for (size_t n : {28, 29, 31}) {
    std::vector<uint8_t> img(buf.begin(), buf.begin() + n);
    const auto before = img;
    CHECK_RC(tcpck_fill16(img.data(), n, 0, &c), TCPCK_EINVAL);
    CHECK(img == before);
  }
  for (int mode : {TCPCK_MODE_REF, TCPCK_MODE_RFC1071}) {
    for (size_t n : {30, 32, 96, 1492, 65536}) {
      std::vector<uint8_t> img(buf.begin() + 3, buf.begin() + 3 + n);
      auto zero = img;
      zero[28] = zero[29] = 0;
      CHECK_RC(tcpck_fill16(img.data(), n, mode, &c), TCPCK_OK);
      CHECK(c == scalar16(zero.data(), n, mode) && field(img.data()) == c);
      CHECK_RC(tcpck_fill16(img.data(), n, mode, nullptr), TCPCK_OK);
      CHECK(field(img.data()) == c);
    }
  }

  // update16 == recomputation whenever C was the image's valid checksum
  std::mt19937_64 rng(3);
  for (int mode : {TCPCK_MODE_REF, TCPCK_MODE_RFC1071}) {
    for (int t = 0; t < 2000; ++t) {
      std::vector<uint8_t> img(64);
      for (auto &b : img) b = static_cast<uint8_t>(rng());
      img[0] |= 1;  // never the all-zero image (RFC 1071's -0 corner)
      CHECK_RC(tcpck_fill16(img.data(), img.size(), mode, &c), TCPCK_OK);
      const size_t w = 2 * (rng() % 32);
      if (w == 28) continue;
      const uint16_t old_w = static_cast<uint16_t>(img[w] | (img[w + 1] << 8));
      const uint16_t new_w = static_cast<uint16_t>(rng());
      img[w] = static_cast<uint8_t>(new_w);
      img[w + 1] = static_cast<uint8_t>(new_w >> 8);
      const uint16_t upd = tcpck_update16(c, old_w, new_w, mode);
      auto zero = img;
      zero[28] = zero[29] = 0;
      const uint16_t full = scalar16(zero.data(), zero.size(), mode);
      if (mode == TCPCK_MODE_REF)
        CHECK(upd == full);
      else  // one's complement: +0 and -0 (0x0000 / 0xFFFF) are the same checksum
        CHECK(upd == full || ((upd == 0 || upd == 0xFFFF) && (upd ^ full) == 0xFFFF));
    }
  }

  // every entry point with a NULL context (or list) is EINVAL, nothing else touched
  uint8_t dummy[64] = {};
  uint64_t off[2] = {0, 32};
  uint32_t len[2] = {32, 32};
  tcpck_ctx *none[2] = {nullptr, nullptr};
  CHECK_RC(tcpck_batch_fixed(nullptr, 0, 0, dummy, 32, 32, 1, dummy, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_var(nullptr, 0, 0, dummy, off, len, 2, dummy, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_set_ack(nullptr, 0, dummy, nullptr, 32, 1, nullptr, 1, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_header_swap(nullptr, dummy, nullptr, 32, 1, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_receive(nullptr, 0, dummy, 32, 32, nullptr, nullptr, 1, dummy, nullptr, nullptr, nullptr),
           TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_segment(nullptr, 0, dummy, 64, 16, dummy, 1, dummy, 64, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_fixed(nullptr, 0, 0, dummy, 32, 32, 2, dummy), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_var(nullptr, 0, 0, dummy, off, len, 2, dummy), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_fixed_multi(nullptr, 1, 0, 0, dummy, 32, 32, 2, dummy), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_fixed_multi(none, 2, 0, 0, dummy, 32, 32, 2, dummy), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_var_multi(none, 0, 0, 0, dummy, off, len, 2, dummy), TCPCK_EINVAL);
  CHECK_RC(tcpck_ctx_set_chunk_bytes(nullptr, 1 << 20), TCPCK_EINVAL);
  CHECK_RC(tcpck_ctx_device(nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_ctx_destroy(nullptr), TCPCK_EINVAL);
  void *p = dummy;
  CHECK_RC(tcpck_device_alloc(nullptr, 16, &p), TCPCK_EINVAL);
  CHECK_RC(tcpck_device_free(nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_memcpy_h2d(nullptr, dummy, dummy, 2), TCPCK_EINVAL);
  CHECK_RC(tcpck_memcpy_d2h(nullptr, dummy, dummy, 2), TCPCK_EINVAL);
  CHECK_RC(tcpck_stream_sync(nullptr, nullptr), TCPCK_EINVAL);
  tcpck_ctx *ctx = reinterpret_cast<tcpck_ctx *>(&dummy);
  CHECK_RC(tcpck_ctx_create(0, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_ctx_create(-1, &ctx), TCPCK_ENODEV);
  CHECK(ctx == nullptr);
  CHECK_RC(tcpck_ctx_create(1 << 20, &ctx), TCPCK_ENODEV);
  CHECK(tcpck_device_supported(-1) == 0 && tcpck_device_supported(1 << 20) == 0);
}

// ---- device 0 -------------------------------------------------------------------

struct Dev {
  tcpck_ctx *ctx;
  template <typename T>
  T *alloc(size_t n) {
    void *p = nullptr;
    CHECK_RC(tcpck_device_alloc(ctx, n * sizeof(T) + 16, &p), TCPCK_OK);
    return static_cast<T *>(p);
  }
  template <typename T>
  void put(T *d, const std::vector<T> &h) {
    CHECK_RC(tcpck_memcpy_h2d(ctx, d, h.data(), h.size() * sizeof(T)), TCPCK_OK);
  }
  template <typename T>
  std::vector<T> get(const T *d, size_t n) {
    std::vector<T> h(n);
    CHECK_RC(tcpck_stream_sync(ctx, nullptr), TCPCK_OK);
    CHECK_RC(tcpck_memcpy_d2h(ctx, h.data(), d, n * sizeof(T)), TCPCK_OK);
    return h;
  }
  void free(void *p) { CHECK_RC(tcpck_device_free(ctx, p), TCPCK_OK); }
};

// images of lengths `lens` packed from offset 0 (or in `slot`-byte slots)
std::vector<uint64_t> offsets_of(const std::vector<uint32_t> &lens, uint64_t slot = 0) {
  std::vector<uint64_t> o(lens.size());
  uint64_t at = 0;
  for (size_t k = 0; k < lens.size(); ++k) {
    o[k] = slot ? k * slot : at;
    at += lens[k];
  }
  return o;
}

void device_validation(Dev &d) {
  uint8_t *a = d.alloc<uint8_t>(4096);
  uint16_t *o = d.alloc<uint16_t>(64);
  tcpck_ctx *c = d.ctx;
  CHECK_RC(tcpck_batch_fixed(c, 9, 0, a, 32, 32, 2, o, nullptr), TCPCK_EINVAL);        // bad op
  CHECK_RC(tcpck_batch_fixed(c, 0, 5, a, 32, 32, 2, o, nullptr), TCPCK_EINVAL);        // bad mode
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a + 1, 32, 32, 2, o, nullptr), TCPCK_EINVAL);    // odd arena
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 33, 32, 2, o, nullptr), TCPCK_EINVAL);        // odd stride
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 32, 31, 2, o, nullptr), TCPCK_EINVAL);        // odd len
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 30, 32, 2, o, nullptr), TCPCK_EINVAL);        // stride < len
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 32, 32, 2, nullptr, nullptr), TCPCK_EINVAL);  // CHECKSUM needs out
  CHECK_RC(tcpck_batch_fixed(c, 1, 0, a, 28, 28, 2, o, nullptr), TCPCK_EINVAL);        // FILL < 30 B
  CHECK_RC(tcpck_batch_fixed(c, 3, 0, a, 30, 30, 2, o, nullptr), TCPCK_EINVAL);        // RECEIVE < 32 B
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 1ull << 40, 32, 1ull << 30, o, nullptr), TCPCK_EINVAL);  // overflow
  CHECK_RC(tcpck_batch_fixed(c, 0, 0, a, 32, 32, 0, o, nullptr), TCPCK_OK);            // empty
  CHECK_RC(tcpck_batch_var(c, 0, 0, a, nullptr, nullptr, 2, o, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_receive(c, 0, a, 32, 32, nullptr, nullptr, 2, nullptr, nullptr, nullptr, nullptr),
           TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_receive(c, 0, a, 32, 32, nullptr, nullptr, 2, a, a + 2, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_receive(c, 0, a, 32, 32, nullptr, nullptr, ~0ull, a, a, nullptr, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_header_swap(c, a, nullptr, 30, 2, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_header_swap(c, a, nullptr, 32, ~0ull, nullptr), TCPCK_EINVAL);
  CHECK_RC(tcpck_batch_set_ack(c, 0, a, nullptr, 28, 2, nullptr, 1, nullptr, nullptr), TCPCK_EINVAL);
  const uint8_t hdr[32] = {};
  CHECK_RC(tcpck_batch_segment(c, 0, a, 64, 18, hdr, 1, a, 64, nullptr, nullptr), TCPCK_EINVAL);   // seg % 4
  CHECK_RC(tcpck_batch_segment(c, 0, a, 64, 16, hdr, 1, a, 40, nullptr, nullptr), TCPCK_EINVAL);   // stride % 16
  CHECK_RC(tcpck_batch_segment(c, 0, a, 63, 16, hdr, 1, a, 64, nullptr, nullptr), TCPCK_EINVAL);   // odd bytes
  CHECK_RC(tcpck_batch_segment(c, 0, a + 2, 64, 16, hdr, 1, a, 64, nullptr, nullptr), TCPCK_EINVAL);  // align
  CHECK_RC(tcpck_ctx_set_chunk_bytes(c, 100), TCPCK_EINVAL);
  // host batches: odd offsets / FILL below 30 B are found by the host scan
  std::vector<uint8_t> h(256, 1);
  std::vector<uint64_t> ho = {0, 65};
  std::vector<uint32_t> hl = {64, 64};
  std::vector<uint16_t> hr(2);
  CHECK_RC(tcpck_host_batch_var(c, 0, 0, h.data(), ho.data(), hl.data(), 2, hr.data()), TCPCK_EINVAL);
  ho = {0, 64};
  hl = {64, 28};
  CHECK_RC(tcpck_host_batch_var(c, 1, 0, h.data(), ho.data(), hl.data(), 2, hr.data()), TCPCK_EINVAL);
  CHECK_RC(tcpck_host_batch_fixed(c, 1, 0, h.data(), 28, 28, 2, hr.data()), TCPCK_EINVAL);
  d.free(a);
  d.free(o);
}

// Fixed and packed-variable batches: CHECKSUM, FILL with and without results,
// VERIFY, RECEIVE, header swap, set_ack -- checked image by image on the host.
void device_small(Dev &d) {
  const uint64_t n = 3001;
  const uint32_t L = 1492;
  auto h = random_bytes(n * L, 11);
  uint8_t *a = d.alloc<uint8_t>(n * L);
  uint16_t *o = d.alloc<uint16_t>(n);
  uint8_t *ok = d.alloc<uint8_t>(n);
  d.put(a, h);
  for (int mode : {0, 1}) {
    CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_CHECKSUM, mode, a, L, L, n, o, nullptr), TCPCK_OK);
    auto r = d.get(o, n);
    for (uint64_t k = 0; k < n; ++k) CHECK(r[k] == scalar16(&h[k * L], L, mode));
  }
  for (int with_out : {1, 0}) {
    d.put(a, h);
    CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_FILL, 0, a, L, L, n, with_out ? o : nullptr, nullptr), TCPCK_OK);
    auto got = d.get(a, n * L);
    auto r = d.get(o, n);
    for (uint64_t k = 0; k < n; ++k) {
      std::vector<uint8_t> z(&h[k * L], &h[k * L] + L);
      z[28] = z[29] = 0;
      const uint16_t want = scalar16(z.data(), L, 0);
      CHECK(field(&got[k * L]) == want);
      if (with_out) CHECK(r[k] == want);
      CHECK(std::memcmp(&got[k * L], z.data(), 28) == 0);
    }
  }
  CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_VERIFY, 0, a, L, L, n, ok, nullptr), TCPCK_OK);
  for (uint8_t v : d.get(ok, n)) CHECK(v == 1);
  // retransmit: ACK rewritten, checksum updated incrementally -> still verifies
  CHECK_RC(tcpck_batch_set_ack(d.ctx, 0, a, nullptr, L, n, nullptr, 0x12345678u, o, nullptr), TCPCK_OK);
  CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_VERIFY, 0, a, L, L, n, ok, nullptr), TCPCK_OK);
  for (uint8_t v : d.get(ok, n)) CHECK(v == 1);
  auto acked = d.get(a, n * L);
  for (uint64_t k = 0; k < n; ++k) CHECK(acked[k * L + 20] == 0x12 && acked[k * L + 23] == 0x78);
  // header swap twice is the identity; RECEIVE into an array = verdicts + swapped headers
  CHECK_RC(tcpck_batch_header_swap(d.ctx, a, nullptr, L, n, nullptr), TCPCK_OK);
  CHECK_RC(tcpck_batch_header_swap(d.ctx, a, nullptr, L, n, nullptr), TCPCK_OK);
  CHECK(d.get(a, n * L) == acked);
  uint8_t *hdr = d.alloc<uint8_t>(32 * n);
  CHECK_RC(tcpck_batch_receive(d.ctx, 0, a, L, L, nullptr, nullptr, n, ok, hdr, nullptr, nullptr), TCPCK_OK);
  auto hh = d.get(hdr, 32 * n);
  for (uint8_t v : d.get(ok, n)) CHECK(v == 1);
  for (uint64_t k = 0; k < n; ++k) {
    const uint8_t *src = &acked[k * L], *dst = &hh[32 * k];
    for (int w : {0, 4, 16, 20})
      for (int b = 0; b < 4; ++b) CHECK(dst[w + b] == src[w + 3 - b]);
    for (int w : {10, 12, 14, 26, 30}) CHECK(dst[w] == src[w + 1] && dst[w + 1] == src[w]);
    for (int w : {8, 9, 24, 25, 28, 29}) CHECK(dst[w] == src[w]);
  }
  d.free(hdr);

  // a packed 96/608/1492 mix: FILL without results (AUTO's update form through
  // a scratch slot), then CHECKSUM with a wrong-but-harmless SORTED hint
  std::mt19937_64 rng(12);
  std::vector<uint32_t> lens(20011);
  for (auto &l : lens) l = std::vector<uint32_t>{96, 608, 1492}[rng() % 3];
  auto offs = offsets_of(lens);
  const uint64_t total = offs.back() + lens.back();
  auto hv = random_bytes(total, 13);
  uint8_t *av = d.alloc<uint8_t>(total);
  uint64_t *doff = d.alloc<uint64_t>(lens.size());
  uint32_t *dlen = d.alloc<uint32_t>(lens.size());
  d.put(av, hv);
  d.put(doff, offs);
  d.put(dlen, lens);
  tcpck_layout lay{total, 96, 1492, TCPCK_LAYOUT_PACKED, 0};
  CHECK_RC(tcpck_batch_var(d.ctx, TCPCK_OP_FILL, 0, av, doff, dlen, lens.size(), nullptr, &lay, nullptr), TCPCK_OK);
  auto gv = d.get(av, total);
  for (size_t k = 0; k < lens.size(); ++k) {
    std::vector<uint8_t> z(&hv[offs[k]], &hv[offs[k]] + lens[k]);
    z[28] = z[29] = 0;
    CHECK(field(&gv[offs[k]]) == scalar16(z.data(), lens[k], 0));
  }
  uint16_t *ov = d.alloc<uint16_t>(lens.size());
  tcpck_layout sorted{total, 96, 1492, TCPCK_LAYOUT_SORTED, 0};
  CHECK_RC(tcpck_batch_var(d.ctx, TCPCK_OP_CHECKSUM, 0, av, doff, dlen, lens.size(), ov, &sorted, nullptr),
           TCPCK_OK);
  auto rv = d.get(ov, lens.size());
  for (size_t k = 0; k < lens.size(); ++k) CHECK(rv[k] == scalar16(&gv[offs[k]], lens[k], 0));
  d.free(av);
  d.free(doff);
  d.free(dlen);
  d.free(ov);
  d.free(a);
  d.free(o);
  d.free(ok);
}

// FILL without results past 8M images (the scratch slot's 8M-image chunks, and
// for an offset list the scaled layout hint of each chunk), checked by VERIFY
// over every image and by the host on a sample.
void device_past_8m(Dev &d) {
  const uint64_t n = (8ull << 20) + 5;
  const uint32_t L = 512;  // rstream's deferred fields (fixed) / the update form (offset list)
  uint8_t *a = d.alloc<uint8_t>(n * L);
  uint8_t *ok = d.alloc<uint8_t>(n);
  std::vector<uint64_t> sample;
  for (uint64_t k = 0; k < n; k += 999983) sample.push_back(k);
  sample.push_back(n - 1);
  for (int var = 0; var < 2; ++var) {
    CHECK_RC(tcpck_synth_fixed(a, L, L, n, 77 + var, 0, 0, nullptr), TCPCK_OK);
    uint64_t *doff = nullptr;
    uint32_t *dlen = nullptr;
    if (!var) {
      CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_FILL, 0, a, L, L, n, nullptr, nullptr), TCPCK_OK);
      CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_VERIFY, 0, a, L, L, n, ok, nullptr), TCPCK_OK);
    } else {
      std::vector<uint64_t> offs(n);
      for (uint64_t k = 0; k < n; ++k) offs[k] = k * L;
      std::vector<uint32_t> lens(n, L);
      doff = d.alloc<uint64_t>(n);
      dlen = d.alloc<uint32_t>(n);
      d.put(doff, offs);
      d.put(dlen, lens);
      tcpck_layout lay{n * L, L, L, TCPCK_LAYOUT_PACKED, 0};
      CHECK_RC(tcpck_batch_var(d.ctx, TCPCK_OP_FILL, 0, a, doff, dlen, n, nullptr, &lay, nullptr), TCPCK_OK);
      CHECK_RC(tcpck_batch_var(d.ctx, TCPCK_OP_VERIFY, 0, a, doff, dlen, n, ok, &lay, nullptr), TCPCK_OK);
    }
    auto v = d.get(ok, n);
    CHECK(std::all_of(v.begin(), v.end(), [](uint8_t x) { return x == 1; }));
    for (uint64_t k : sample) {
      std::vector<uint8_t> img(L);
      CHECK_RC(tcpck_stream_sync(d.ctx, nullptr), TCPCK_OK);
      CHECK_RC(tcpck_memcpy_d2h(d.ctx, img.data(), a + k * L, L), TCPCK_OK);
      CHECK(scalar16(img.data(), L, 0) == 0);
    }
    if (doff) d.free(doff);
    if (dlen) d.free(dlen);
  }
  d.free(a);
  d.free(ok);
}

// Host batches in many small chunks (64-KiB staging) on one and two contexts.
void host_batches(Dev &d, tcpck_ctx *second) {
  CHECK_RC(tcpck_ctx_set_chunk_bytes(d.ctx, 64 << 10), TCPCK_OK);
  CHECK_RC(tcpck_ctx_set_chunk_bytes(second, 48 << 10), TCPCK_OK);
  const uint64_t n = 2003;
  const uint32_t L = 1492;
  auto h = random_bytes(n * L, 21);
  std::vector<uint16_t> r(n);
  CHECK_RC(tcpck_host_batch_fixed(d.ctx, TCPCK_OP_CHECKSUM, 0, h.data(), L, L, n, r.data()), TCPCK_OK);
  for (uint64_t k = 0; k < n; ++k) CHECK(r[k] == scalar16(&h[k * L], L, 0));
  tcpck_ctx *both[2] = {d.ctx, second};
  std::vector<uint16_t> r2(n);
  CHECK_RC(tcpck_host_batch_fixed_multi(both, 2, TCPCK_OP_CHECKSUM, 0, h.data(), L, L, n, r2.data()), TCPCK_OK);
  CHECK(r2 == r);
  auto f = h;
  CHECK_RC(tcpck_host_batch_fixed(d.ctx, TCPCK_OP_FILL, 0, f.data(), L, L, n, nullptr), TCPCK_OK);
  for (uint64_t k = 0; k < n; ++k) CHECK(scalar16(&f[k * L], L, 0) == 0);

  // slots with gaps (SORTED), then unordered offsets
  std::mt19937_64 rng(22);
  std::vector<uint32_t> lens(4001);
  for (auto &l : lens) l = std::vector<uint32_t>{96, 608, 1492}[rng() % 3];
  auto offs = offsets_of(lens, 2048);
  auto hv = random_bytes(lens.size() * 2048, 23);
  std::vector<uint16_t> rv(lens.size()), rv2(lens.size());
  CHECK_RC(tcpck_host_batch_var(d.ctx, TCPCK_OP_CHECKSUM, 0, hv.data(), offs.data(), lens.data(), lens.size(),
                                rv.data()),
           TCPCK_OK);
  for (size_t k = 0; k < lens.size(); ++k) CHECK(rv[k] == scalar16(&hv[offs[k]], lens[k], 0));
  CHECK_RC(tcpck_host_batch_var_multi(both, 2, TCPCK_OP_CHECKSUM, 0, hv.data(), offs.data(), lens.data(),
                                      lens.size(), rv2.data()),
           TCPCK_OK);
  CHECK(rv2 == rv);
  std::vector<size_t> perm(lens.size());
  for (size_t k = 0; k < perm.size(); ++k) perm[k] = k;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<uint64_t> po(lens.size());
  std::vector<uint32_t> pl(lens.size());
  for (size_t k = 0; k < perm.size(); ++k) {
    po[k] = offs[perm[k]];
    pl[k] = lens[perm[k]];
  }
  CHECK_RC(tcpck_host_batch_var(d.ctx, TCPCK_OP_CHECKSUM, 1, hv.data(), po.data(), pl.data(), pl.size(), rv2.data()),
           TCPCK_OK);
  for (size_t k = 0; k < pl.size(); ++k) CHECK(rv2[k] == scalar16(&hv[po[k]], pl[k], 1));
  CHECK_RC(tcpck_ctx_set_chunk_bytes(d.ctx, 64ull << 20), TCPCK_OK);
}

// The send stream cut into images (tcpck_batch_segment): every image verifies.
void device_segment(Dev &d) {
  const uint64_t P = 1000002;
  const uint32_t seg = 1460, stride = 1504;
  const uint64_t n = (P + seg - 1) / seg;
  auto payload = random_bytes(P, 31);
  uint8_t *dp = d.alloc<uint8_t>(P);
  uint8_t *di = d.alloc<uint8_t>(n * stride);
  uint16_t *o = d.alloc<uint16_t>(n);
  d.put(dp, payload);
  uint8_t hdr[32] = {127, 0, 0, 1, 127, 0, 0, 1};
  hdr[25] = 0x10;
  for (int mode : {0, 1}) {
    CHECK_RC(tcpck_batch_segment(d.ctx, mode, dp, P, seg, hdr, 1001, di, stride, o, nullptr), TCPCK_OK);
    auto img = d.get(di, n * stride);
    auto r = d.get(o, n);
    for (uint64_t k = 0; k < n; ++k) {
      const uint32_t lk = static_cast<uint32_t>(std::min<uint64_t>(seg, P - k * seg));
      CHECK(std::memcmp(&img[k * stride + 32], &payload[k * seg], lk) == 0);
      CHECK(field(&img[k * stride]) == r[k]);
      uint16_t c = 0;
      CHECK_RC(tcpck_checksum16(&img[k * stride], 32 + lk, mode, &c), TCPCK_OK);
      CHECK(c == 0);
    }
  }
  d.free(dp);
  d.free(di);
  d.free(o);
}

// Out-less FILLs from 4 threads on 4 streams at once (the scratch slots' mutexes
// and events), 10 calls each, then every image verifies.
void device_threads(Dev &d) {
  const uint64_t n = 1 << 16;
  const uint32_t L = 1492;
  std::vector<uint8_t *> arenas(4);
  std::vector<hipStream_t> streams(4);
  for (int t = 0; t < 4; ++t) {
    arenas[t] = d.alloc<uint8_t>(n * L);
    CHECK_RC(tcpck_synth_fixed(arenas[t], L, L, n, 40 + t, 0, 0, nullptr), TCPCK_OK);
    CHECK(hipStreamCreateWithFlags(&streams[t], hipStreamNonBlocking) == hipSuccess);
  }
  CHECK_RC(tcpck_stream_sync(d.ctx, nullptr), TCPCK_OK);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < 10; ++i)
        if (tcpck_batch_fixed(d.ctx, TCPCK_OP_FILL, 0, arenas[t], L, L, n, nullptr, streams[t]) != TCPCK_OK) ++bad;
      if (tcpck_stream_sync(d.ctx, streams[t]) != TCPCK_OK) ++bad;
    });
  for (auto &x : th) x.join();
  CHECK(bad.load() == 0);
  uint8_t *ok = d.alloc<uint8_t>(n);
  for (int t = 0; t < 4; ++t) {
    CHECK_RC(tcpck_batch_fixed(d.ctx, TCPCK_OP_VERIFY, 0, arenas[t], L, L, n, ok, nullptr), TCPCK_OK);
    auto v = d.get(ok, n);
    CHECK(std::all_of(v.begin(), v.end(), [](uint8_t x) { return x == 1; }));
    d.free(arenas[t]);
    CHECK(hipStreamDestroy(streams[t]) == hipSuccess);
  }
  d.free(ok);
}

}  // namespace

int main(int argc, char **argv) {
  const std::string what = argc > 1 ? argv[1] : "cpu";
  cpu_checks();
  if (what == "gpu") {
    Dev d{nullptr};
    CHECK_RC(tcpck_ctx_create(0, &d.ctx), TCPCK_OK);
    CHECK(tcpck_ctx_device(d.ctx) == 0);
    tcpck_ctx *second = nullptr;
    CHECK_RC(tcpck_ctx_create(0, &second), TCPCK_OK);
    device_validation(d);
    device_small(d);
    device_segment(d);
    host_batches(d, second);
    device_threads(d);
    device_past_8m(d);
    CHECK_RC(tcpck_ctx_destroy(second), TCPCK_OK);
    CHECK_RC(tcpck_ctx_destroy(d.ctx), TCPCK_OK);
  }
  std::printf("ok %ld checks\n", g_checks);
  return 0;
}
