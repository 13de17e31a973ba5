// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// Binds the reference's OWN checksum (filixi/TCP-stack,
// include/tcp-header.h:252-263, `friend uint16_t CalculateChecksum(const
// TcpPacket&)`) to a C ABI so tests and bench.py's cpu_baseline leg can run
// the real reference code.  The reference header is #included by path from
// /root/reference at build time (oracle/Makefile); its source is never copied
// into this repo.  Output goes to oracle/_ref/ (git-ignored, travels to the GPU
// box as a prebuilt .so).  Nothing in the product links this.
//
// Packets are built with MakeNetPacket (tcp-header.h:310-315), which copies
// every byte of the image; MakeTcpPacket(size) would leave the payload
// uninitialised (tcp-header.h:270-273), see SURVEY.md section 8c.
#include "tcp-header.h"

#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using tcp_stack::TcpPacket;

extern "C" {

// One image -> reference checksum (the receive path's computation,
// include/socket-manager.h:182, before the ==0 test).
uint16_t ref_calculate_checksum(const char *buf, size_t n) {
  auto p = tcp_stack::MakeNetPacket(buf, n);
  return CalculateChecksum(*p);
}

// Send-side insertion exactly as src/socket-manager.cc:9-10: zero the field,
// compute, store; the filled image is copied back into buf.
uint16_t ref_fill(char *buf, size_t n) {
  auto p = tcp_stack::MakeNetPacket(buf, n);
  p->GetHeader().Checksum() = 0;
  p->GetHeader().Checksum() = CalculateChecksum(*p);
  auto bs = p->GetBuffer();
  std::memcpy(buf, bs.first, bs.second);
  return p->GetHeader().Checksum();
}

// Receive-side verification, include/socket-manager.h:182.
int ref_verify(const char *buf, size_t n) {
  auto p = tcp_stack::MakeNetPacket(buf, n);
  return CalculateChecksum(*p) == 0;
}

// Builds a structured 32-B header the way the send path does
// (socket-internal.h header builders + TcpHeaderH2N, tcp-header.h:193-206),
// with the checksum field left 0.  Used by the golden-vector generator.
void ref_make_header(char *out32, uint32_t src, uint32_t dst, uint16_t tcplen,
                     uint16_t sport, uint16_t dport, uint32_t seq, uint32_t ack,
                     uint16_t win, uint16_t urg, int flag_ack, int flag_syn,
                     int flag_fin, int flag_rst, int flag_psh, int flag_urg) {
  auto p = tcp_stack::MakeTcpPacket(0);
  auto &h = p->GetHeader();
  h.SourceAddress() = src;
  h.DestinationAddress() = dst;
  h.PTCL() = 6;
  h.TcpLength() = tcplen;
  h.SourcePort() = sport;
  h.DestinationPort() = dport;
  h.SequenceNumber() = seq;
  h.AcknowledgementNumber() = ack;
  h.Window() = win;
  h.UrgentPointer() = urg;
  h.SetAck(flag_ack);
  h.SetSyn(flag_syn);
  h.SetFin(flag_fin);
  h.SetRst(flag_rst);
  h.SetPsh(flag_psh);
  h.SetUrg(flag_urg);
  tcp_stack::TcpHeaderH2N(h);
  h.Checksum() = 0;
  std::memcpy(out32, p->GetBuffer().first, 32);
}

// ---- CPU baseline harness: packets are materialised once (outside the
// timed region), then CalculateChecksum runs over all of them on `nthreads`
// std::threads.  Returns elapsed seconds of the timed region.
struct RefPackets {
  std::vector<std::shared_ptr<TcpPacket>> pkts;
};

void *ref_packets_make(const char *arena, const uint64_t *off,
                       const uint32_t *len, uint64_t stride, uint64_t flen,
                       size_t n) {
  auto *h = new RefPackets;
  h->pkts.reserve(n);
  for (size_t k = 0; k < n; ++k) {
    const char *b = off ? arena + off[k] : arena + k * stride;
    const size_t l = len ? len[k] : flen;
    h->pkts.push_back(tcp_stack::MakeNetPacket(b, l));
  }
  return h;
}

double ref_packets_checksum(void *handle, uint16_t *out, int nthreads) {
  auto *h = static_cast<RefPackets *>(handle);
  const size_t n = h->pkts.size();
  if (nthreads < 1) nthreads = 1;
  auto t0 = std::chrono::steady_clock::now();
  auto body = [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) out[k] = CalculateChecksum(*h->pkts[k]);
  };
  if (nthreads == 1) {
    body(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back(body, n * t / nthreads, n * (t + 1) / nthreads);
    for (auto &x : th) x.join();
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// Same, `reps` passes over all packets in one timed region: the threads start
// once, each runs its share `reps` times, so thread start-up stays out of a
// pass over a DRAM-sized packet set (bench.py's median-of-5 baseline).
double ref_packets_checksum_reps(void *handle, uint16_t *out, int nthreads, int reps) {
  auto *h = static_cast<RefPackets *>(handle);
  const size_t n = h->pkts.size();
  if (nthreads < 1) nthreads = 1;
  if (reps < 1) reps = 1;
  auto body = [&](size_t lo, size_t hi) {
    for (int r = 0; r < reps; ++r)
      for (size_t k = lo; k < hi; ++k) out[k] = CalculateChecksum(*h->pkts[k]);
  };
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(body, n * t / nthreads, n * (t + 1) / nthreads);
  body(0, n / nthreads);
  for (auto &x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

void ref_packets_free(void *handle) { delete static_cast<RefPackets *>(handle); }

}  // extern "C"
