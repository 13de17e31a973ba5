// tests/golden/gen_segment.cc -- generates the committed segmentation fixtures
// (segment_golden.bin + segment_golden.json) by running the REFERENCE's own
// data-segment send path on known send streams:
//
//   TcpSendingBuffer::Push / GetAsTcpPacket(0, window)  include/tcp-buffer.h:70-98
//     (MakeTcpPacket(len), the payload copied out of the deque, TcpLength = len)
//   Estab, Event::kSend                                   src/state.cc:167-184
//     (SetAck(true), SequenceNumber = snd_nxt, AcknowledgementNumber = rcv_nxt,
//      snd_nxt += TcpLength) -- restated here: state.cc needs the whole stack
//   SetSource / SetDestination                            include/socket-internal.h:52-60
//   TcpHeaderH2N                                          include/tcp-header.h:193-206
//   Checksum() = 0; Checksum() = CalculateChecksum(*p)    include/socket-manager.h:259-260
//
// Built and run only in the build container, where /root/reference exists:
//     sh tests/golden/make_golden.sh
// The reference headers are #included by path; no reference source is copied.
// Output = data only: the send streams, the header templates the batched op
// takes, and the reference's images and checksums.
#include "tcp-buffer.h"
#include "tcp-header.h"

#include <arpa/inet.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

using namespace tcp_stack;

namespace {

std::vector<uint8_t> blob;
std::string json = "{\n  \"blob\": \"segment_golden.bin\",\n  \"cases\": [\n";
bool first_case = true;

uint64_t rng = 0x9E3779B97F4A7C15ull;  // fixed seed
uint8_t next_byte() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return static_cast<uint8_t>(rng >> 32);
}

size_t put(const void *p, size_t n) {
  while (blob.size() % 16) blob.push_back(0);
  const size_t off = blob.size();
  const auto *b = static_cast<const uint8_t *>(p);
  blob.insert(blob.end(), b, b + n);
  return off;
}

struct Conn {
  uint32_t src_ip, dst_ip;
  uint16_t sport, dport;
  uint32_t snd_nxt, rcv_nxt;
};

// The per-connection header fields of a data segment, as GetPacketForSending
// leaves them, with TcpLength and the sequence number 0: the template the
// batched op fills per segment (network order, checksum 0).
std::vector<uint8_t> header_template(const Conn &c) {
  TcpHeader h;  // zero-filled (tcp-header.h:18)
  h.SetAck(true);
  h.AcknowledgementNumber() = c.rcv_nxt;
  h.SourceAddress() = c.src_ip;
  h.SourcePort() = c.sport;
  h.DestinationAddress() = c.dst_ip;
  h.DestinationPort() = c.dport;
  TcpHeaderH2N(h);
  const auto *p = reinterpret_cast<const uint8_t *>(&h);
  return std::vector<uint8_t>(p, p + sizeof(TcpHeader));
}

void add_case(const std::string &name, const std::vector<uint8_t> &payload, uint32_t window, Conn c) {
  const size_t pay_off = put(payload.data(), payload.size());
  const auto tmpl = header_template(c);
  const size_t tmpl_off = put(tmpl.data(), tmpl.size());
  const uint32_t seq0 = c.snd_nxt;

  TcpSendingBuffer buf;
  buf.InitializeAckNumber(seq0);
  buf.Push(reinterpret_cast<const char *>(payload.data()), payload.size());
  std::vector<uint8_t> images;
  std::vector<size_t> lens;
  std::vector<unsigned> sums;
  while (!buf.Empty()) {
    auto pkt = buf.GetAsTcpPacket(0, window);           // tcp-buffer.h:82-98
    TcpHeader &h = pkt->GetHeader();
    h.SetAck(true);                                     // state.cc:178-180
    h.SequenceNumber() = c.snd_nxt;
    h.AcknowledgementNumber() = c.rcv_nxt;
    c.snd_nxt += h.TcpLength();                         // state.cc:182
    h.SourceAddress() = c.src_ip;                       // socket-internal.h:52-55
    h.SourcePort() = c.sport;
    h.DestinationAddress() = c.dst_ip;                  // socket-internal.h:57-60
    h.DestinationPort() = c.dport;
    TcpHeaderH2N(h);                                    // socket-internal.h:196
    h.Checksum() = 0;                                   // socket-manager.h:259-260
    h.Checksum() = CalculateChecksum(*pkt);
    auto [p, n] = pkt->GetBuffer();
    images.insert(images.end(), p, p + n);
    lens.push_back(n);
    sums.push_back(h.Checksum());
  }
  const size_t img_off = put(images.data(), images.size());

  char head[512];
  std::snprintf(head, sizeof head,
                "%s    {\"name\": \"%s\", \"payload_off\": %zu, \"payload_len\": %zu, \"seg\": %u, "
                "\"seq0\": %u, \"template_off\": %zu, \"images_off\": %zu, \"lengths\": [",
                first_case ? "" : ",\n", name.c_str(), pay_off, payload.size(), window, seq0, tmpl_off, img_off);
  first_case = false;
  json += head;
  for (size_t i = 0; i < lens.size(); ++i) json += (i ? ", " : "") + std::to_string(lens[i]);
  json += "], \"checksums\": [";
  for (size_t i = 0; i < sums.size(); ++i) json += (i ? ", " : "") + std::to_string(sums[i]);
  json += "]}";
}

std::vector<uint8_t> random_bytes(size_t n) {
  std::vector<uint8_t> v(n);
  for (auto &b : v) b = next_byte();
  return v;
}

}  // namespace

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const uint32_t lo = 0x7F000001u;  // 127.0.0.1, host order (main.cc:19-22)
  const Conn demo{lo, lo, 15500, 15501, 1001, 7777};
  // the reference's own window: every segment 1024 B (state.cc:43, 60)
  add_case("window1024_5000", random_bytes(5000), 1024, demo);
  add_case("window1024_exact4", random_bytes(4096), 1024, demo);
  add_case("short_single", random_bytes(100), 1024, demo);
  add_case("two_bytes", random_bytes(2), 1024, demo);
  // Ethernet MSS payloads, a 2-B last segment
  add_case("mss1460_tail2", random_bytes(3 * 1460 + 2), 1460, Conn{0x0A000002u, 0xC0A80101u, 443, 51000, 123456, 99});
  add_case("mss1448_ff", std::vector<uint8_t>(3000, 0xFF), 1448, Conn{lo, 0x0A000001u, 80, 40000, 0xFFFFFF00u, 5});
  add_case("mss1448_zero", std::vector<uint8_t>(2896, 0x00), 1448, Conn{lo, lo, 1, 2, 0, 0});
  // jumbo segments and the sequence number wrapping past 2^32
  add_case("jumbo65532", random_bytes(2 * 65532 + 8), 65532, Conn{lo, lo, 9000, 9001, 0xFFFF0000u, 0x12345678u});
  add_case("jumbo9000_wrap", random_bytes(5 * 9000 + 100), 9000, Conn{0xC0A80001u, 0xC0A80002u, 2049, 2050, 0xFFFFC000u, 3});
  // tiny segments
  add_case("seg4", random_bytes(40), 4, demo);
  add_case("seg16_odd_tail", random_bytes(16 * 9 + 6), 16, demo);
  add_case("seg100", random_bytes(1000), 100, demo);
  add_case("seg1000_random_fields", random_bytes(7777 + 1), 1000, Conn{0xDEADBEEFu, 0x01020304u, 0xABCD, 0x1234, 0x80000000u, 0xFFFFFFFFu});
  json += "\n  ],\n  \"blob_bytes\": " + std::to_string(blob.size()) + "\n}\n";

  FILE *f = std::fopen((dir + "/segment_golden.bin").c_str(), "wb");
  if (!f || std::fwrite(blob.data(), 1, blob.size(), f) != blob.size()) return 1;
  std::fclose(f);
  f = std::fopen((dir + "/segment_golden.json").c_str(), "w");
  if (!f) return 1;
  std::fputs(json.c_str(), f);
  std::fclose(f);
  std::printf("wrote %zu bytes of segment fixtures\n", blob.size());
  return 0;
}
