/*
 * oracle/ref16.c -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A plain-C restatement of the reference TCP checksum, used by tests/,
 * __graft_entry__.smoke() and bench.py's `cpu_baseline` leg as the CHECKER.
 * Nothing in the product (tcp-stack_amd/, include/) links, loads or calls this
 * file; the product path is the HIP library `libtcpck.so`.
 *
 * Pinned by: tests/golden/ (vectors produced by the reference header itself,
 * tests/golden/gen_golden.cc) and by oracle/_ref (the reference's own
 * CalculateChecksum compiled from /root/reference/include/tcp-header.h).
 *
 * Reference algorithm (filixi/TCP-stack, include/tcp-header.h:252-263):
 *
 *     uint32_t checksum = 0;
 *     uint16_t *buffer = (uint16_t *)packet.buff_;
 *     for (i = 0; i < size/2; ++i) checksum += buffer[i];   // :257-258
 *     if (size % 2) checksum += buffer[size-1];              // :259-260 (OOB read: UB)
 *     return (uint16_t)~checksum;                           // :262
 *
 * i.e. ~(sum of little-endian u16 words mod 2^16) -- NOT RFC 1071 (no
 * end-around carry).  Odd sizes read out of bounds in the reference, so no
 * parity exists for them; the oracle reports them as an error (-1) from the
 * checked entry points.  The RFC 1071 variant (opt-in mode 1 of the product)
 * is restated here too, as its own oracle; the reference does not compute
 * it, so it is pinned instead by RFC 1071 section 3's worked example
 * (00 01 f2 03 f4 f5 f6 f7 -> 0x0d22 here; tests/test_oracle.py).
 */
#include <stddef.h>
#include <stdint.h>
#include <pthread.h>
#include <string.h>

/* include/tcp-header.h:252-263, word-at-a-time exactly as written. */
uint16_t oracle_ref16(const uint8_t *buf, size_t size) {
  uint32_t checksum = 0;
  size_t i;
  for (i = 0; i < size / 2; ++i) {
    uint16_t w;
    memcpy(&w, buf + 2 * i, 2); /* little-endian host, like the reference */
    checksum += w;
  }
  return (uint16_t)~checksum;
}

/* RFC 1071 one's-complement sum over the same LE words, stored raw (mode 1). */
uint16_t oracle_rfc1071(const uint8_t *buf, size_t size) {
  uint64_t s = 0;
  size_t i;
  for (i = 0; i < size / 2; ++i) {
    uint16_t w;
    memcpy(&w, buf + 2 * i, 2);
    s += w;
  }
  while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
  return (uint16_t)~s;
}

/* Send-side insertion, include/socket-manager.h:259-260 and
 * src/socket-manager.cc:9-10: zero bytes 28-29 (TcpHeader::Checksum(),
 * tcp-header.h:177 -> field_ byte 16 -> image byte 12+16), compute, store raw. */
uint16_t oracle_fill(uint8_t *buf, size_t size, int mode) {
  uint16_t c;
  buf[28] = 0;
  buf[29] = 0;
  c = mode ? oracle_rfc1071(buf, size) : oracle_ref16(buf, size);
  memcpy(buf + 28, &c, 2);
  return c;
}

typedef struct {
  const uint8_t *arena;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride, flen;
  size_t lo, hi;
  uint16_t *out;
  int mode;
} job_t;

static void *run_job(void *p) {
  job_t *j = (job_t *)p;
  size_t k;
  for (k = j->lo; k < j->hi; ++k) {
    const uint8_t *b = j->off ? j->arena + j->off[k] : j->arena + k * j->stride;
    size_t n = j->len ? j->len[k] : j->flen;
    j->out[k] = j->mode ? oracle_rfc1071(b, n) : oracle_ref16(b, n);
  }
  return NULL;
}

/* Batch over (offsets, lengths) or, when off == NULL, a fixed stride.
 * Returns -1 on any odd length (no parity defined, tcp-header.h:259-260). */
int oracle_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                 uint64_t stride, uint64_t flen, size_t n, uint16_t *out,
                 int mode, int nthreads) {
  pthread_t th[256];
  job_t jobs[256];
  size_t k;
  int t;
  if (len) {
    for (k = 0; k < n; ++k)
      if (len[k] & 1) return -1;
  } else if (flen & 1) {
    return -1;
  }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  for (t = 0; t < nthreads; ++t) {
    jobs[t].arena = arena;
    jobs[t].off = off;
    jobs[t].len = len;
    jobs[t].stride = stride;
    jobs[t].flen = flen;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
    jobs[t].out = out;
    jobs[t].mode = mode;
  }
  if (nthreads == 1) {
    run_job(&jobs[0]);
    return 0;
  }
  for (t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
  for (t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}
