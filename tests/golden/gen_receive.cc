// tests/golden/gen_receive.cc -- generates the committed receive-path fixtures
// (receive_golden.bin + receive_golden.json) by running the REFERENCE's own
// code on both ends of the wire:
//
//   send:    MakeTcpPacket(len), header fields through TcpHeader's accessors
//            (tcp-header.h:52-191), TcpHeaderH2N (tcp-header.h:193-206),
//            Checksum() = 0; Checksum() = CalculateChecksum(*p)
//            (socket-manager.h:259-260) -- then, for some packets, a flipped
//            byte or a wrong checksum (a damaged packet)
//   receive: MakeNetPacket(wire, n) (tcp-header.h:310-315), the verdict
//            CalculateChecksum(*packet) == 0 and TcpHeaderN2H
//            (ReceivePacket, socket-manager.h:181-184; tcp-header.h:208-221)
//
// Built and run only in the build container, where /root/reference exists:
//     sh tests/golden/make_golden.sh
// The reference headers are #included by path; no reference source is copied.
// Output = data only: one arena of wire images (network order) at even
// offsets, the same arena after the receive path, the verdicts and the
// host-order header fields the accessors read after TcpHeaderN2H.
#include "tcp-header.h"

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

using namespace tcp_stack;

namespace {

uint64_t rng = 0xD1B54A32D192ED03ull;  // fixed seed
uint32_t next32() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return static_cast<uint32_t>(rng >> 32);
}

std::string list(const std::vector<uint64_t> &v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
  return s + "]";
}

}  // namespace

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const size_t payloads[] = {0, 2, 4, 14, 100, 1024, 1460, 1448, 536, 8, 2000, 64, 9000, 30, 6, 1200};
  std::vector<uint8_t> wire, host;
  std::vector<uint64_t> offsets, lengths, ok, damage;
  std::vector<uint64_t> f_src, f_dst, f_len, f_sport, f_dport, f_seq, f_ack, f_win, f_urg, f_flags;
  const int n = 96;
  for (int k = 0; k < n; ++k) {
    const size_t len = payloads[k % 16] + 2 * (k / 16 % 3);
    auto p = MakeTcpPacket(len);
    for (char *c = p->begin(); c != p->end(); ++c) *c = static_cast<char>(next32());
    TcpHeader &h = p->GetHeader();
    h.SourceAddress() = next32();
    h.DestinationAddress() = k % 5 ? next32() : 0x7F000001u;
    h.PTCL() = 6;
    h.TcpLength() = static_cast<uint16_t>(len);
    h.SourcePort() = static_cast<uint16_t>(next32());
    h.DestinationPort() = static_cast<uint16_t>(next32());
    h.SequenceNumber() = next32();
    h.AcknowledgementNumber() = next32();
    h.SetAck(k % 2);
    h.SetSyn(k % 7 == 0);
    h.SetFin(k % 11 == 0);
    h.SetRst(k % 13 == 0);
    h.SetPsh(k % 3 == 0);
    h.SetUrg(k % 17 == 0);
    h.Window() = static_cast<uint16_t>(next32());
    h.UrgentPointer() = static_cast<uint16_t>(next32());
    TcpHeaderH2N(h);
    h.Checksum() = 0;
    h.Checksum() = CalculateChecksum(*p);
    auto [buf, size] = p->GetBuffer();
    std::vector<uint8_t> w(buf, buf + size);
    // damage: 0 none; 1 a payload or header byte flipped; 2 checksum off by one
    const uint64_t dmg = k % 4 == 3 ? 1 + (k / 4) % 2 : 0;
    if (dmg == 1) w[(next32() % (size / 2)) * 2 + (k & 1)] ^= static_cast<uint8_t>(1u << (k % 8));
    if (dmg == 2) w[28] ^= 1;
    while (wire.size() % 2 || (k % 3 == 1 && wire.size() % 16 != 6)) wire.push_back(0xA5);
    offsets.push_back(wire.size());
    lengths.push_back(size);
    damage.push_back(dmg);
    wire.insert(wire.end(), w.begin(), w.end());
  }
  while (wire.size() % 16) wire.push_back(0xA5);
  host = wire;
  for (int k = 0; k < n; ++k) {
    // ReceivePacket (socket-manager.h:181-184) on the wire bytes
    auto p = MakeNetPacket(reinterpret_cast<const char *>(wire.data() + offsets[k]), lengths[k]);
    ok.push_back(CalculateChecksum(*p) == 0);
    TcpHeaderN2H(p->GetHeader());
    const TcpHeader &h = p->GetHeader();
    f_src.push_back(h.SourceAddress());
    f_dst.push_back(h.DestinationAddress());
    f_len.push_back(h.TcpLength());
    f_sport.push_back(h.SourcePort());
    f_dport.push_back(h.DestinationPort());
    f_seq.push_back(h.SequenceNumber());
    f_ack.push_back(h.AcknowledgementNumber());
    f_win.push_back(h.Window());
    f_urg.push_back(h.UrgentPointer());
    f_flags.push_back(h.Urg() | h.Ack() << 1 | h.Psh() << 2 | h.Rst() << 3 | h.Syn() << 4 | h.Fin() << 5);
    auto [buf, size] = p->GetBuffer();
    std::copy(buf, buf + size, host.begin() + offsets[k]);
  }
  std::vector<uint8_t> blob = wire;
  blob.insert(blob.end(), host.begin(), host.end());

  std::string json = "{\n  \"blob\": \"receive_golden.bin\", \"blob_bytes\": " + std::to_string(blob.size()) +
                     ",\n  \"wire_off\": 0, \"host_off\": " + std::to_string(wire.size()) +
                     ", \"arena_bytes\": " + std::to_string(wire.size()) +
                     ",\n  \"offsets\": " + list(offsets) + ",\n  \"lengths\": " + list(lengths) +
                     ",\n  \"damage\": " + list(damage) + ",\n  \"ok\": " + list(ok) +
                     ",\n  \"fields\": {\n    \"src\": " + list(f_src) + ",\n    \"dst\": " + list(f_dst) +
                     ",\n    \"tcp_length\": " + list(f_len) + ",\n    \"sport\": " + list(f_sport) +
                     ",\n    \"dport\": " + list(f_dport) + ",\n    \"seq\": " + list(f_seq) +
                     ",\n    \"ack\": " + list(f_ack) + ",\n    \"window\": " + list(f_win) +
                     ",\n    \"urgent\": " + list(f_urg) + ",\n    \"flags\": " + list(f_flags) + "\n  }\n}\n";
  FILE *f = std::fopen((dir + "/receive_golden.bin").c_str(), "wb");
  if (!f || std::fwrite(blob.data(), 1, blob.size(), f) != blob.size()) return 1;
  std::fclose(f);
  f = std::fopen((dir + "/receive_golden.json").c_str(), "w");
  if (!f) return 1;
  std::fputs(json.c_str(), f);
  std::fclose(f);
  std::printf("wrote %zu bytes of receive fixtures\n", blob.size());
  return 0;
}
