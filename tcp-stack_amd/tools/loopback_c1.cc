// loopback_c1.cc -- BASELINE config C1: one 1460-B segment at a time over UDP
// loopback, checksummed on the CPU through the tcp-header API (plumbing, no GPU).
//
// Mirrors the reference's per-packet path without its control plane:
//   send     TcpSendingBuffer::GetAsTcpPacket (tcp-buffer.h:82-98: new image,
//            TcpLength = payload), header fields + TcpHeaderH2N
//            (socket-internal.h:52-60, tcp-header.h:193-206), then
//            SocketManager::SendPacket: Checksum() = 0; Checksum() =
//            CalculateChecksum(*packet) (socket-manager.cc:9-10) and sendto
//            (network-service.h:61-65);
//   receive  recvfrom into a reused buffer (network-service.cc:39,49-50),
//            MakeNetPacket (tcp-header.h:310-315), then
//            CalculateChecksum(*packet) == 0 (socket-manager.h:182).
//
// Source-compatible with both headers: built against include/tcp_stack/
// (this library, -ltcpck) by tcp-stack_amd/Makefile, and against the
// reference's own include/tcp-header.h by oracle/Makefile (`make ref`, this
// container only) -- the same program is the drop-in check.
//
//   loopback_c1 [segments] [payload]   -> one JSON line
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "tcp-header.h"

using namespace tcp_stack;

int main(int argc, char **argv) {
  const size_t segments = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000;
  const size_t payload = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1460;
  const uint16_t sport = 15500, dport = 15501;  // main.cc:19-22

  const int rx = socket(AF_INET, SOCK_DGRAM, 0);
  const int tx = socket(AF_INET, SOCK_DGRAM, 0);
  if (rx < 0 || tx < 0) return 2;
  sockaddr_in ra{};
  ra.sin_family = AF_INET;
  ra.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  ra.sin_port = 0;  // any free port: the demo's fixed ports may be taken
  if (bind(rx, reinterpret_cast<sockaddr *>(&ra), sizeof(ra)) != 0) return 3;
  socklen_t rl = sizeof(ra);
  getsockname(rx, reinterpret_cast<sockaddr *>(&ra), &rl);
  int big = 8 << 20;
  setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));

  std::vector<char> data(payload);
  for (size_t i = 0; i < payload; ++i) data[i] = static_cast<char>((i * 131u + 7u) & 0xFF);
  std::vector<char> rbuf(102400);  // network-service.cc:39

  size_t verified = 0, received = 0;
  double send_ck_ns = 0, recv_ck_ns = 0;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (size_t k = 0; k < segments; ++k) {
    auto pkt = MakeTcpPacket(data.data(), payload);
    TcpHeader &h = pkt->GetHeader();
    h.SourceAddress() = INADDR_LOOPBACK;
    h.DestinationAddress() = INADDR_LOOPBACK;
    h.PTCL() = 6;
    h.TcpLength() = static_cast<uint16_t>(payload);
    h.SourcePort() = sport;
    h.DestinationPort() = dport;
    h.SequenceNumber() = static_cast<uint32_t>(1000 + k * payload);
    h.AcknowledgementNumber() = 77;
    h.SetAck(true);
    h.Window() = 1024;
    TcpHeaderH2N(h);
    const auto c0 = clk::now();
    h.Checksum() = 0;
    h.Checksum() = CalculateChecksum(*pkt);
    send_ck_ns += std::chrono::duration<double, std::nano>(clk::now() - c0).count();
    auto buf = pkt->GetBuffer();
    if (sendto(tx, buf.first, buf.second, 0, reinterpret_cast<sockaddr *>(&ra), sizeof(ra)) !=
        static_cast<ssize_t>(buf.second))
      return 4;
    const ssize_t n = recvfrom(rx, rbuf.data(), rbuf.size(), 0, nullptr, nullptr);
    if (n <= 0) return 5;
    ++received;
    auto in = MakeNetPacket(rbuf.data(), static_cast<size_t>(n));
    const auto c1 = clk::now();
    const bool ok = CalculateChecksum(*in) == 0;
    recv_ck_ns += std::chrono::duration<double, std::nano>(clk::now() - c1).count();
    verified += ok;
  }
  const double total_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
  std::printf(
      "{\"config\": \"C1\", \"segments\": %zu, \"payload\": %zu, \"image_bytes\": %zu, \"received\": %zu, "
      "\"verified\": %zu, \"us_per_segment\": %.3f, \"send_checksum_ns\": %.1f, \"recv_checksum_ns\": %.1f}\n",
      segments, payload, payload + sizeof(TcpHeader), received, verified, total_us / segments,
      send_ck_ns / segments, recv_ck_ns / segments);
  close(rx);
  close(tx);
  return verified == segments ? 0 : 1;
}
