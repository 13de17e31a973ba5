// tests/golden/gen_golden.cc -- generates the committed golden fixtures
// (golden.bin + golden.json) by running the REFERENCE's own checksum
// (filixi/TCP-stack include/tcp-header.h:252-263) on known inputs.
//
// Built and run only in the build container, where /root/reference exists:
//     sh tests/golden/make_golden.sh
// The reference header is #included by path (-I/root/reference/include); no
// reference source is copied.  Output = data only: image bytes and the
// reference's answers.
//
// Every image is materialised with MakeNetPacket (tcp-header.h:310-315), which
// copies all bytes (MakeTcpPacket(size) leaves the payload uninitialised,
// tcp-header.h:270-273).
#include "tcp-header.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace tcp_stack;

namespace {

struct Case {
  std::string name, kind;  // kind: checksum | fill | verify
  size_t off, len;
  unsigned expected;       // checksum value, or 0/1 for verify
  size_t fill_off;         // for kind==fill: offset of the reference-filled image
};

std::vector<uint8_t> blob;
std::vector<Case> cases;

uint64_t rng = 0x243F6A8885A308D3ull;  // fixed seed
uint8_t next_byte() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return static_cast<uint8_t>(rng >> 24);
}

// Append an image at an offset with the requested residue mod 16 (even), so
// the fixtures also exercise unaligned segment starts in a packed arena.
size_t place(const std::vector<uint8_t> &img, unsigned mis) {
  while (blob.size() % 16 != mis) blob.push_back(0xA5);
  size_t off = blob.size();
  blob.insert(blob.end(), img.begin(), img.end());
  return off;
}

unsigned ref_checksum(const std::vector<uint8_t> &img) {
  auto p = MakeNetPacket(reinterpret_cast<const char *>(img.data()), img.size());
  return CalculateChecksum(*p);
}

unsigned mis_cycle = 0;
void add_checksum(const std::string &name, const std::vector<uint8_t> &img) {
  unsigned mis = (mis_cycle++ * 2) % 16;
  size_t off = place(img, mis);
  cases.push_back({name, "checksum", off, img.size(), ref_checksum(img), 0});
}

// send path, src/socket-manager.cc:9-10
void add_fill(const std::string &name, const std::vector<uint8_t> &img) {
  unsigned mis = (mis_cycle++ * 2) % 16;
  size_t off = place(img, mis);
  auto p = MakeNetPacket(reinterpret_cast<const char *>(img.data()), img.size());
  p->GetHeader().Checksum() = 0;
  p->GetHeader().Checksum() = CalculateChecksum(*p);
  auto bs = p->GetBuffer();
  std::vector<uint8_t> filled(bs.first, bs.first + bs.second);
  size_t foff = place(filled, 0);
  cases.push_back({name, "fill", off, img.size(), p->GetHeader().Checksum(), foff});
  // receive path, include/socket-manager.h:182: the filled image verifies
  auto q = MakeNetPacket(bs.first, bs.second);
  cases.push_back({name + "/verify", "verify", foff, filled.size(),
                   CalculateChecksum(*q) == 0 ? 1u : 0u, 0});
  // one flipped payload/header byte must fail verification
  std::vector<uint8_t> bad = filled;
  bad[bad.size() / 2] ^= 0x5A;
  size_t boff = place(bad, (mis_cycle++ * 2) % 16);
  auto r = MakeNetPacket(reinterpret_cast<const char *>(bad.data()), bad.size());
  cases.push_back({name + "/corrupt", "verify", boff, bad.size(),
                   CalculateChecksum(*r) == 0 ? 1u : 0u, 0});
}

std::vector<uint8_t> structured_header(uint32_t src, uint32_t dst, uint16_t tcplen,
                                       uint16_t sport, uint16_t dport, uint32_t seq,
                                       uint32_t ack, uint16_t win, uint16_t urg,
                                       bool fack, bool fsyn, bool ffin, bool frst) {
  auto p = MakeTcpPacket(0);  // header-only, zero-initialised (tcp-header.h:18,270-273)
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
  h.SetAck(fack);
  h.SetSyn(fsyn);
  h.SetFin(ffin);
  h.SetRst(frst);
  TcpHeaderH2N(h);
  h.Checksum() = 0;
  auto bs = p->GetBuffer();
  return std::vector<uint8_t>(bs.first, bs.first + bs.second);
}

}  // namespace

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const size_t sizes[] = {32, 96, 608, 1492, 65536};

  // Known-answer patterns.
  for (size_t n : sizes) {
    std::vector<uint8_t> v(n);
    for (size_t i = 0; i < n; ++i) v[i] = static_cast<uint8_t>((i * 7 + 1) & 0xFF);
    add_checksum("pattern7/" + std::to_string(n), v);
  }
  for (size_t n : sizes) add_checksum("ones/" + std::to_string(n), std::vector<uint8_t>(n, 0xFF));
  for (size_t n : sizes) add_checksum("zeros/" + std::to_string(n), std::vector<uint8_t>(n, 0x00));

  // Every even length 0..256 with random bytes (short images come from
  // MakeNetPacket of short datagrams, network-service.cc:49-56).
  for (size_t n = 0; n <= 256; n += 2) {
    std::vector<uint8_t> v(n);
    for (auto &b : v) b = next_byte();
    add_checksum("rand/" + std::to_string(n), v);
  }
  // Lengths around the configs, including 2 mod 4.
  const size_t odd4[] = {94, 98, 606, 610, 1490, 1494, 4094, 4098, 65534};
  for (size_t n : odd4) {
    std::vector<uint8_t> v(n);
    for (auto &b : v) b = next_byte();
    add_checksum("rand/" + std::to_string(n), v);
  }
  // Adversarial: words of 0xFFFF / 0x0001 mixes that wrap the u16 many times.
  for (size_t n : {1492, 65536}) {
    std::vector<uint8_t> v(n);
    for (size_t i = 0; i < n; i += 2) {
      v[i] = (i / 2) % 3 ? 0xFF : 0x01;
      v[i + 1] = (i / 2) % 3 ? 0xFF : 0x00;
    }
    add_checksum("wrapmix/" + std::to_string(n), v);
  }

  // Structured header of SURVEY.md 8c: 127.0.0.1 -> 10.0.0.2, TcpLength 0x1234,
  // 0xabcd -> 10, seq 0x11223344, ack 0x55667788, win 1024, urg 0x0102, ACK+SYN.
  auto hdr = structured_header(0x7F000001u, 0x0A000002u, 0x1234, 0xabcd, 10,
                               0x11223344u, 0x55667788u, 1024, 0x0102, true, true,
                               false, false);
  add_checksum("struct_hdr/32", hdr);
  add_fill("struct_hdr/32", hdr);

  // Data segments the way the send path builds them (tcp-buffer.h:82-98 sets
  // TcpLength = payload; state.cc Estab sets ACK; H2N; checksum zeroed), with
  // random payloads at the config payload sizes.
  const size_t payloads[] = {0, 64, 576, 1023, 1024, 1460, 65504};
  uint32_t seq = 1000;
  for (size_t pl : payloads) {
    if (pl % 2) continue;  // odd images have no parity (tcp-header.h:259-260)
    auto h = structured_header(0x7F000001u, 0x7F000001u, static_cast<uint16_t>(pl),
                               15500, 15501, seq, 77, 1024, 0, true, false, false,
                               false);
    seq += static_cast<uint32_t>(pl);
    std::vector<uint8_t> img = h;
    for (size_t i = 0; i < pl; ++i) img.push_back(next_byte());
    add_fill("segment/" + std::to_string(pl), img);
  }
  // Garbage in the checksum field before fill must not matter.
  {
    auto img = structured_header(0x0A000001u, 0x0A000002u, 1460, 80, 443, 7, 9,
                                 1024, 0, true, false, true, false);
    for (size_t i = 0; i < 1460; ++i) img.push_back(next_byte());
    img[28] = 0xDE;
    img[29] = 0xAD;
    add_fill("segment_dirty_field/1460", img);
  }

  while (blob.size() % 16) blob.push_back(0);
  FILE *f = std::fopen((dir + "/golden.bin").c_str(), "wb");
  std::fwrite(blob.data(), 1, blob.size(), f);
  std::fclose(f);
  f = std::fopen((dir + "/golden.json").c_str(), "w");
  std::fprintf(f, "{\n  \"source\": \"filixi/TCP-stack include/tcp-header.h:252-263 via "
                  "MakeNetPacket+CalculateChecksum (tests/golden/gen_golden.cc)\",\n");
  std::fprintf(f, "  \"blob\": \"golden.bin\",\n  \"blob_bytes\": %zu,\n  \"cases\": [\n",
               blob.size());
  for (size_t i = 0; i < cases.size(); ++i) {
    const auto &c = cases[i];
    std::fprintf(f,
                 "    {\"name\": \"%s\", \"kind\": \"%s\", \"off\": %zu, \"len\": %zu, "
                 "\"expected\": %u, \"fill_off\": %zu}%s\n",
                 c.name.c_str(), c.kind.c_str(), c.off, c.len, c.expected, c.fill_off,
                 i + 1 < cases.size() ? "," : "");
  }
  std::fprintf(f, "  ]\n}\n");
  std::fclose(f);
  std::printf("wrote %zu cases, %zu bytes\n", cases.size(), blob.size());
  return 0;
}
