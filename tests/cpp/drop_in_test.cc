// drop_in_test.cc -- exercises the drop-in C++ header (include/tcp_stack/) the
// way the reference's call sites use it.  Driven by tests/test_drop_in.py.
//
//   drop_in_test golden <blob> <manifest>   one output line per manifest case
//       manifest line: <kind> <off> <len>; kind checksum|fill|verify
//       checksum -> CalculateChecksum(*MakeNetPacket(image))        (tcp-header.h:252-263)
//       fill     -> Checksum()=0; Checksum()=CalculateChecksum(...)  (socket-manager.cc:9-10)
//                   prints the stored value, then CalculateChecksum of the result
//       verify   -> CalculateChecksum(...) == 0                      (socket-manager.h:182)
//   drop_in_test layout                      header field layout / H2N / flags / operator<<
//   drop_in_test batch <n> <seed> [ctxs]     PacketBatch (GPU, ctxs contexts on device 0) vs per-packet
//                                            CalculateChecksum
//   drop_in_test segment <bytes> <win> <seed> tcpck_batch_segment (GPU) vs the per-packet send path
//   drop_in_test receive <n> <slot> <seed>    tcpck_batch_receive (GPU) vs ReceivePacket's verdict + N2H
#include <tcp_stack/packet-batch.h>
#include <tcp_stack/tcp-header.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <vector>

using namespace tcp_stack;

static int Golden(const char *blob_path, const char *manifest) {
  std::ifstream bf(blob_path, std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(bf)), std::istreambuf_iterator<char>());
  std::ifstream mf(manifest);
  std::string kind;
  size_t off, len;
  while (mf >> kind >> off >> len) {
    if (off + len > blob.size()) return 2;
    auto pkt = MakeNetPacket(blob.data() + off, len);
    if (kind == "checksum") {
      std::printf("%u\n", CalculateChecksum(*pkt));
    } else if (kind == "fill") {
      auto &h = pkt->GetHeader();
      h.Checksum() = 0;
      h.Checksum() = CalculateChecksum(*pkt);
      std::printf("%u %u\n", h.Checksum(), CalculateChecksum(*pkt));
    } else if (kind == "verify") {
      std::printf("%d\n", CalculateChecksum(*pkt) == 0 ? 1 : 0);
    } else {
      return 3;
    }
  }
  return 0;
}

static int Layout() {
  // The structured header of SURVEY.md §8c / tests/golden (struct_hdr/32).
  auto pkt = MakeTcpPacket(0);
  TcpHeader &h = pkt->GetHeader();
  h.SourceAddress() = 0x7f000001u;       // 127.0.0.1
  h.DestinationAddress() = 0x0a000002u;  // 10.0.0.2
  h.PTCL() = 6;
  h.TcpLength() = 0x1234;
  h.SourcePort() = 0xabcd;
  h.DestinationPort() = 10;
  h.SequenceNumber() = 0x11223344u;
  h.AcknowledgementNumber() = 0x55667788u;
  h.Window() = 1024;
  h.UrgentPointer() = 0x0102;
  h.SetAck(true);
  h.SetSyn(true);
  std::ostringstream text;
  text << h;
  std::printf("text %s\n", text.str().c_str());
  TcpHeaderH2N(h);
  h.Checksum() = 0;
  const auto buf = pkt->GetBuffer();
  std::printf("size %zu\nbytes", buf.second);
  for (size_t i = 0; i < buf.second; ++i) std::printf(" %02x", static_cast<unsigned char>(buf.first[i]));
  std::printf("\n");
  h.Checksum() = CalculateChecksum(*pkt);
  std::printf("checksum %u\nreverify %u\n", h.Checksum(), CalculateChecksum(*pkt));
  {
    // retransmit ACK rewrite (socket-internal.h:376-377): incremental == full recompute
    auto rp = MakeNetPacket(pkt->GetBuffer().first, pkt->GetBuffer().second);
    TcpHeader &r = rp->GetHeader();
    const uint32_t old_ack = r.AcknowledgementNumber();
    r.AcknowledgementNumber() = htonl(0xdeadbeefu);
    const uint16_t inc = UpdateChecksum32(r.Checksum(), old_ack, r.AcknowledgementNumber());
    r.Checksum() = 0;
    const uint16_t full = CalculateChecksum(*rp);
    std::printf("update %u %u\n", inc, full);
  }
  TcpHeaderN2H(h);
  std::printf("n2h %x %x %u %x\n", h.SourceAddress(), h.SequenceNumber(), h.Window(), h.TcpLength());
  // flag bits land in byte 25 exactly as the reference's bit positions 106..111
  auto p2 = MakeTcpPacket(0);
  const unsigned char *b = reinterpret_cast<const unsigned char *>(p2->GetBuffer().first);
  TcpHeader &g = p2->GetHeader();
  g.SetUrg(true); std::printf("urg %02x\n", b[25]); g.SetUrg(false);
  g.SetAck(true); std::printf("ack %02x\n", b[25]); g.SetAck(false);
  g.SetPsh(true); std::printf("psh %02x\n", b[25]); g.SetPsh(false);
  g.SetRst(true); std::printf("rst %02x\n", b[25]); g.SetRst(false);
  g.SetSyn(true); std::printf("syn %02x\n", b[25]); g.SetSyn(false);
  g.SetFin(true); std::printf("fin %02x\n", b[25]); g.SetFin(false);
  std::printf("cleared %02x\n", b[25]);
  // payload constructor: zeroed header + copied payload
  const char payload[6] = {1, 2, 3, 4, 5, 6};
  auto p3 = MakeTcpPacket(payload, sizeof(payload));
  std::printf("payload %zu %d %d\n", p3->GetBuffer().second, p3->begin()[0], p3->end()[-1]);
  // odd length: defined here (zero-padded last word), verifies after fill
  const char odd[5] = {9, 8, 7, 6, 5};
  auto p4 = MakeTcpPacket(odd, sizeof(odd));
  p4->GetHeader().Checksum() = 0;
  p4->GetHeader().Checksum() = CalculateChecksum(*p4);
  std::printf("odd %u %u\n", p4->GetHeader().Checksum(), CalculateChecksum(*p4));
  return 0;
}

static int Batch(size_t n, unsigned seed, size_t ctxs) {
  std::mt19937_64 rng(seed);
  const size_t lens[] = {0, 64, 576, 1460, 1461, 7, 4000};
  std::vector<std::shared_ptr<TcpPacket>> pkts, copy;
  for (size_t k = 0; k < n; ++k) {
    const size_t pl = lens[rng() % (sizeof(lens) / sizeof(lens[0]))];
    std::vector<char> payload(pl);
    for (auto &c : payload) c = static_cast<char>(rng());
    auto p = MakeTcpPacket(payload.data(), pl);
    TcpHeader &h = p->GetHeader();
    h.SourceAddress() = 0x7f000001u;
    h.DestinationAddress() = 0x7f000001u;
    h.PTCL() = 6;
    h.TcpLength() = static_cast<uint16_t>(pl);
    h.SourcePort() = 15500;
    h.DestinationPort() = 15501;
    h.SequenceNumber() = static_cast<uint32_t>(1000 + k);
    h.SetAck(true);
    h.Window() = 1024;
    TcpHeaderH2N(h);
    h.Checksum() = static_cast<uint16_t>(rng());  // stale field: fill must ignore it
    auto b = p->GetBuffer();
    copy.push_back(MakeNetPacket(b.first, b.second));
    pkts.push_back(std::move(p));
  }
  PacketBatch batch(std::vector<int>(ctxs, 0), PacketBatch::Thresholds{1, 1});
  // checksums as-is
  const std::vector<uint16_t> sums = batch.Checksums(pkts);
  size_t bad = 0;
  for (size_t k = 0; k < n; ++k) bad += sums[k] != CalculateChecksum(*copy[k]);
  const size_t gpu_images = batch.last_gpu_images();
  // send path: fill in place, compare with the per-packet reference sequence
  batch.Fill(pkts);
  for (size_t k = 0; k < n; ++k) {
    TcpHeader &h = copy[k]->GetHeader();
    h.Checksum() = 0;
    h.Checksum() = CalculateChecksum(*copy[k]);
    bad += pkts[k]->GetHeader().Checksum() != h.Checksum();
  }
  // receive path: every filled packet verifies; a flipped payload byte does not
  std::vector<uint8_t> ok = batch.Verify(pkts);
  for (size_t k = 0; k < n; ++k) bad += ok[k] != 1;
  for (size_t k = 0; k < n; k += 3) {
    auto b = pkts[k]->GetBuffer();
    b.first[b.second - 1] ^= 0x10;
  }
  ok = batch.Verify(pkts);
  for (size_t k = 0; k < n; ++k) bad += ok[k] != (k % 3 != 0);
  std::printf("batch n=%zu gpu_images=%zu mismatches=%zu\n", n, gpu_images, bad);
  return bad == 0 ? 0 : 1;
}

// The send path of INTEGRATION.md section 2 in C++: the header template built
// with the drop-in, one tcpck_batch_segment call on a device-resident stream,
// and every image compared byte for byte with the per-packet reference
// sequence (MakeTcpPacket + payload, TcpLength, Estab's ACK/seq/ack,
// addresses, TcpHeaderH2N, zero + CalculateChecksum) built with the drop-in.
static int Segment(size_t bytes, uint32_t window, unsigned seed) {
  std::mt19937_64 rng(seed);
  std::vector<char> stream(bytes);
  for (auto &c : stream) c = static_cast<char>(rng());
  const uint32_t host_ip = 0x0A000001u, peer_ip = 0x0A000002u, snd_nxt = 0xFFFFF000u, rcv_nxt = 4242;
  const uint16_t host_port = 15500, peer_port = 15501;
  TcpHeader hdr;  // INTEGRATION.md section 2, verbatim
  hdr.SetAck(true);
  hdr.AcknowledgementNumber() = rcv_nxt;
  hdr.SourceAddress() = host_ip;  hdr.SourcePort() = host_port;
  hdr.DestinationAddress() = peer_ip;  hdr.DestinationPort() = peer_port;
  TcpHeaderH2N(hdr);
  const uint64_t n = (bytes + window - 1) / window;
  const uint64_t stride = (32 + window + 15) / 16 * 16;
  tcpck_ctx *ctx = nullptr;
  if (tcpck_ctx_create(0, &ctx) != TCPCK_OK) return 3;
  void *d_stream = nullptr, *d_slots = nullptr, *d_sums = nullptr;
  if (tcpck_device_alloc(ctx, bytes, &d_stream) || tcpck_device_alloc(ctx, n * stride, &d_slots) ||
      tcpck_device_alloc(ctx, n * 2, &d_sums) || tcpck_memcpy_h2d(ctx, d_stream, stream.data(), bytes))
    return 3;
  int st = tcpck_batch_segment(ctx, TCPCK_MODE_REF, d_stream, bytes, window, &hdr, snd_nxt, d_slots, stride,
                               static_cast<uint16_t *>(d_sums), nullptr);
  if (st == TCPCK_OK) st = tcpck_stream_sync(ctx, nullptr);
  std::vector<uint8_t> slots(n * stride);
  std::vector<uint16_t> sums(n);
  if (st || tcpck_memcpy_d2h(ctx, slots.data(), d_slots, slots.size()) ||
      tcpck_memcpy_d2h(ctx, sums.data(), d_sums, n * 2)) {
    std::fprintf(stderr, "segment: %s\n", tcpck_strerror(st));
    return 3;
  }
  size_t bad = 0;
  uint32_t seq = snd_nxt;
  for (uint64_t k = 0; k < n; ++k) {
    const size_t len = std::min<size_t>(window, bytes - k * window);
    auto p = MakeTcpPacket(stream.data() + k * window, len);  // GetAsTcpPacket (tcp-buffer.h:82-98)
    TcpHeader &h = p->GetHeader();
    h.TcpLength() = static_cast<uint16_t>(len);
    h.SetAck(true);                                           // Estab (state.cc:178-182)
    h.SequenceNumber() = seq;
    h.AcknowledgementNumber() = rcv_nxt;
    seq += h.TcpLength();
    h.SourceAddress() = host_ip;  h.SourcePort() = host_port; // socket-internal.h:52-60
    h.DestinationAddress() = peer_ip;  h.DestinationPort() = peer_port;
    TcpHeaderH2N(h);
    h.Checksum() = 0;                                         // socket-manager.h:259-260
    h.Checksum() = CalculateChecksum(*p);
    auto b = p->GetBuffer();
    bad += std::memcmp(b.first, slots.data() + k * stride, b.second) != 0;
    bad += sums[k] != h.Checksum();
    for (size_t t = b.second; t < stride; ++t) bad += slots[k * stride + t] != 0;
  }
  tcpck_device_free(ctx, d_stream);
  tcpck_device_free(ctx, d_slots);
  tcpck_device_free(ctx, d_sums);
  tcpck_ctx_destroy(ctx);
  std::printf("segment bytes=%zu window=%u images=%llu mismatches=%zu\n", bytes, window,
              static_cast<unsigned long long>(n), bad);
  return bad == 0 ? 0 : 1;
}

// The receive path of INTEGRATION.md section 2 in C++: datagrams in the slots
// of a device ring, one tcpck_batch_receive call (verdicts + host-order
// headers into a dense array, then in place), against ReceivePacket's front
// half per packet with the drop-in (MakeNetPacket, CalculateChecksum == 0,
// TcpHeaderN2H; socket-manager.h:181-184).
static int Receive(size_t n, uint32_t slot, unsigned seed) {
  std::mt19937_64 rng(seed);
  std::vector<uint8_t> ring(n * slot, 0);
  std::vector<uint64_t> offsets(n);
  std::vector<uint32_t> lengths(n);
  for (size_t k = 0; k < n; ++k) {
    const size_t len = (rng() % ((slot - 32) / 2 + 1)) * 2;  // even payloads, 0 .. slot - 32
    auto p = MakeTcpPacket(len);
    for (char *c = p->begin(); c != p->end(); ++c) *c = static_cast<char>(rng());
    TcpHeader &h = p->GetHeader();
    h.SourceAddress() = static_cast<uint32_t>(rng());
    h.DestinationAddress() = static_cast<uint32_t>(rng());
    h.PTCL() = 6;
    h.TcpLength() = static_cast<uint16_t>(len);
    h.SourcePort() = static_cast<uint16_t>(rng());
    h.DestinationPort() = static_cast<uint16_t>(rng());
    h.SequenceNumber() = static_cast<uint32_t>(rng());
    h.AcknowledgementNumber() = static_cast<uint32_t>(rng());
    h.SetAck(k & 1);
    h.SetSyn(k % 5 == 0);
    h.Window() = static_cast<uint16_t>(rng());
    TcpHeaderH2N(h);
    h.Checksum() = 0;
    h.Checksum() = CalculateChecksum(*p);
    auto b = p->GetBuffer();
    offsets[k] = k * slot;
    lengths[k] = static_cast<uint32_t>(b.second);
    std::memcpy(ring.data() + offsets[k], b.first, b.second);
    if (k % 7 == 3) ring[offsets[k] + rng() % b.second] ^= 0x04;  // a damaged datagram
  }
  tcpck_ctx *ctx = nullptr;
  if (tcpck_ctx_create(0, &ctx) != TCPCK_OK) return 3;
  void *d_ring = nullptr, *d_off = nullptr, *d_len = nullptr, *d_ok = nullptr, *d_hdr = nullptr;
  if (tcpck_device_alloc(ctx, ring.size(), &d_ring) || tcpck_device_alloc(ctx, n * 8, &d_off) ||
      tcpck_device_alloc(ctx, n * 4, &d_len) || tcpck_device_alloc(ctx, n, &d_ok) ||
      tcpck_device_alloc(ctx, n * 32, &d_hdr) || tcpck_memcpy_h2d(ctx, d_ring, ring.data(), ring.size()) ||
      tcpck_memcpy_h2d(ctx, d_off, offsets.data(), n * 8) || tcpck_memcpy_h2d(ctx, d_len, lengths.data(), n * 4))
    return 3;
  uint64_t bytes = 0;
  for (auto l : lengths) bytes += l;
  tcpck_layout lay = {bytes, 32, slot, TCPCK_LAYOUT_SORTED, 0};
  auto *off = static_cast<const uint64_t *>(d_off);
  auto *len = static_cast<const uint32_t *>(d_len);
  auto *okp = static_cast<uint8_t *>(d_ok);
  std::vector<uint8_t> ok(n), ok2(n), hdrs(n * 32), after(ring.size());
  int st = tcpck_batch_receive(ctx, TCPCK_MODE_REF, d_ring, 0, 0, off, len, n, okp, d_hdr, &lay, nullptr);
  if (st == TCPCK_OK) st = tcpck_stream_sync(ctx, nullptr);
  if (st || tcpck_memcpy_d2h(ctx, ok.data(), d_ok, n) || tcpck_memcpy_d2h(ctx, hdrs.data(), d_hdr, n * 32) ||
      tcpck_memcpy_d2h(ctx, after.data(), d_ring, ring.size()))
    return 3;
  size_t bad = after != ring;  // the header array leaves the ring as received
  st = tcpck_batch_receive(ctx, TCPCK_MODE_REF, d_ring, 0, 0, off, len, n, okp, nullptr, &lay, nullptr);
  if (st == TCPCK_OK) st = tcpck_stream_sync(ctx, nullptr);
  if (st || tcpck_memcpy_d2h(ctx, ok2.data(), d_ok, n) || tcpck_memcpy_d2h(ctx, after.data(), d_ring, ring.size())) {
    std::fprintf(stderr, "receive: %s\n", tcpck_strerror(st));
    return 3;
  }
  size_t damaged = 0;
  for (size_t k = 0; k < n; ++k) {
    // ReceivePacket (socket-manager.h:181-184), per packet, with the drop-in
    auto p = MakeNetPacket(reinterpret_cast<const char *>(ring.data() + offsets[k]), lengths[k]);
    const bool valid = CalculateChecksum(*p) == 0;
    TcpHeaderN2H(p->GetHeader());
    damaged += !valid;
    bad += ok[k] != valid;
    bad += ok2[k] != valid;
    bad += std::memcmp(hdrs.data() + 32 * k, &p->GetHeader(), 32) != 0;
    auto b = p->GetBuffer();
    bad += std::memcmp(after.data() + offsets[k], b.first, b.second) != 0;
    for (size_t t = b.second; t < slot; ++t) bad += after[offsets[k] + t] != 0;
  }
  for (void *d : {d_ring, d_off, d_len, d_ok, d_hdr}) tcpck_device_free(ctx, d);
  tcpck_ctx_destroy(ctx);
  std::printf("receive n=%zu slot=%u damaged=%zu mismatches=%zu\n", n, slot, damaged, bad);
  return bad == 0 && (damaged > 0 || n <= 3) ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc >= 5 && !std::strcmp(argv[1], "receive"))
    return Receive(std::strtoull(argv[2], nullptr, 10), static_cast<uint32_t>(std::atoi(argv[3])), std::atoi(argv[4]));
  if (argc >= 5 && !std::strcmp(argv[1], "segment"))
    return Segment(std::strtoull(argv[2], nullptr, 10), static_cast<uint32_t>(std::atoi(argv[3])), std::atoi(argv[4]));
  if (argc >= 4 && !std::strcmp(argv[1], "golden")) return Golden(argv[2], argv[3]);
  if (argc >= 2 && !std::strcmp(argv[1], "layout")) return Layout();
  if (argc >= 4 && !std::strcmp(argv[1], "batch"))
    return Batch(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]),
                 argc >= 5 ? std::strtoull(argv[4], nullptr, 10) : 1);
  std::fprintf(stderr, "usage: %s golden <blob> <manifest> | layout | batch <n> <seed> [ctxs] | segment <bytes> <window> <seed> | receive <n> <slot> <seed>\n",
               argv[0]);
  return 2;
}
