// recv_burst.cc -- SURVEY.md §8f rank 2: batched receive-side verification.
//
// The reference receives one datagram per poll()/recvfrom() into a reused
// 102400-B buffer (src/network-service.cc:41-61), copies it into a TcpPacket
// (MakeNetPacket, include/tcp-header.h:310-315) and verifies it in
// SocketManager::ReceivePacket (include/socket-manager.h:182:
// CalculateChecksum(*packet) == 0), one packet at a time.
//
// Here recvmmsg() lands bursts of datagrams directly in fixed slots of a pinned
// host arena (tcpck_host_alloc).  Once `batch` datagrams (or the end of the
// stream) are in, ONE tcpck_host_batch_var(TCPCK_OP_VERIFY) call checks them
// all on the GPU (chunked H2D -> kernel -> u8 verdicts D2H), and each packet is
// handed on with its verdict: the `check_sum_validate` argument of
// SocketInternal::RecvPacket (socket-manager.h:200).  Odd-length datagrams
// (undefined in the reference, rejected by the C ABI) are verified on the CPU
// through the drop-in CalculateChecksum instead of poisoning the batch.
//
// A sender thread plays the peer.  It builds segments as the send path does
// (header fields + TcpHeaderH2N, Checksum() = 0, Checksum() =
// CalculateChecksum: socket-manager.cc:9-10), corrupts one payload byte of
// every C-th segment after the checksum, and sendmmsg()s them over 127.0.0.1,
// at most `window` datagrams ahead of the receiver (loopback UDP drops what
// does not fit the socket buffer).
//
// Every GPU verdict is checked against CalculateChecksum on the same received
// bytes, and the flagged segments against the corrupted sequence numbers.
//
//   recv_burst [segments] [payload] [batch] [corrupt_every] [--cpu-only]
//   -> one JSON line; exit 0 iff nothing was lost and every verdict matches
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "tcp-header.h"
#include "tcpck.h"

using namespace tcp_stack;
using clk = std::chrono::steady_clock;

namespace {

constexpr size_t kBurst = 32;       // datagrams per sendmmsg / recvmmsg call
constexpr size_t kMaxSlot = 65536;  // largest arena slot per datagram

double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

struct Stats {
  size_t received = 0, truncated = 0, odd = 0, batches = 0;
  size_t mismatches = 0, flagged = 0, flagged_wrong = 0;
  double gpu_ms = 0, cpu_ms = 0, deliver_ms = 0;
  uint64_t bytes = 0;
};

// Sender: the peer's send path (socket-manager.cc:6-12) in bursts of kBurst.
void Sender(int tx, const sockaddr_in &to, size_t segments, size_t payload, size_t corrupt_every, size_t window,
            const std::atomic<size_t> &received, std::atomic<bool> &failed) {
  std::vector<char> data(payload);
  for (size_t i = 0; i < payload; ++i) data[i] = static_cast<char>((i * 131u + 7u) & 0xFF);
  std::vector<std::shared_ptr<TcpPacket>> pkts(kBurst);
  std::vector<mmsghdr> msgs(kBurst);
  std::vector<iovec> iov(kBurst);
  for (size_t k0 = 0; k0 < segments; k0 += kBurst) {
    const size_t n = std::min(kBurst, segments - k0);
    while (k0 + n > received.load(std::memory_order_acquire) + window) std::this_thread::yield();
    for (size_t i = 0; i < n; ++i) {
      const size_t k = k0 + i;
      std::memcpy(data.data(), &k, std::min<size_t>(sizeof(k), payload));  // distinct payloads
      auto pkt = MakeTcpPacket(data.data(), payload);
      TcpHeader &h = pkt->GetHeader();
      h.SourceAddress() = INADDR_LOOPBACK;
      h.DestinationAddress() = INADDR_LOOPBACK;
      h.PTCL() = 6;
      h.TcpLength() = static_cast<uint16_t>(payload);
      h.SourcePort() = 15500;
      h.DestinationPort() = 15501;
      h.SequenceNumber() = static_cast<uint32_t>(k);  // the receiver identifies segments by it
      h.AcknowledgementNumber() = 77;
      h.SetAck(true);
      h.Window() = 1024;
      TcpHeaderH2N(h);
      h.Checksum() = 0;
      h.Checksum() = CalculateChecksum(*pkt);
      if (corrupt_every && k % corrupt_every == corrupt_every - 1 && payload)
        pkt->GetBuffer().first[sizeof(TcpHeader) + k % payload] ^= 0x5A;  // in flight, after the checksum
      auto buf = pkt->GetBuffer();
      iov[i] = {buf.first, buf.second};
      std::memset(&msgs[i], 0, sizeof(mmsghdr));
      msgs[i].msg_hdr.msg_name = const_cast<sockaddr_in *>(&to);
      msgs[i].msg_hdr.msg_namelen = sizeof(to);
      msgs[i].msg_hdr.msg_iov = &iov[i];
      msgs[i].msg_hdr.msg_iovlen = 1;
      pkts[i] = std::move(pkt);
    }
    size_t done = 0;
    while (done < n) {
      const int r = sendmmsg(tx, msgs.data() + done, static_cast<unsigned>(n - done), 0);
      if (r <= 0) {
        failed = true;
        return;
      }
      done += static_cast<size_t>(r);
    }
  }
}

}  // namespace

int main(int argc, char **argv) {
  std::vector<std::string> pos;
  bool cpu_only = false;
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "--cpu-only")
      cpu_only = true;
    else
      pos.emplace_back(argv[i]);
  }
  const size_t segments = pos.size() > 0 ? std::strtoull(pos[0].c_str(), nullptr, 10) : 200000;
  const size_t payload = pos.size() > 1 ? std::strtoull(pos[1].c_str(), nullptr, 10) : 1460;
  const size_t batch = pos.size() > 2 ? std::max<size_t>(1, std::strtoull(pos[2].c_str(), nullptr, 10)) : 65536;
  const size_t corrupt_every = pos.size() > 3 ? std::strtoull(pos[3].c_str(), nullptr, 10) : 97;
  if (payload + sizeof(TcpHeader) > kMaxSlot || payload < 8) {
    std::fprintf(stderr, "payload must be in [8, %zu]\n", kMaxSlot - sizeof(TcpHeader));
    return 2;
  }
  // one arena slot per datagram: the largest image the stack accepts (its MSS +
  // header), rounded up to a 128-B line; a longer datagram comes back MSG_TRUNC
  const size_t kSlot = (payload + sizeof(TcpHeader) + 127) & ~size_t{127};

  const int rx = socket(AF_INET, SOCK_DGRAM, 0);
  const int tx = socket(AF_INET, SOCK_DGRAM, 0);
  if (rx < 0 || tx < 0) return 2;
  sockaddr_in ra{};
  ra.sin_family = AF_INET;
  ra.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  ra.sin_port = 0;
  if (bind(rx, reinterpret_cast<sockaddr *>(&ra), sizeof(ra)) != 0) return 3;
  socklen_t rl = sizeof(ra);
  getsockname(rx, reinterpret_cast<sockaddr *>(&ra), &rl);
  int want_buf = 8 << 20, got_buf = 0;
  setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &want_buf, sizeof(want_buf));
  socklen_t gl = sizeof(got_buf);
  getsockopt(rx, SOL_SOCKET, SO_RCVBUF, &got_buf, &gl);
  // a queued datagram costs ~its size + ~1 KiB of skb overhead in the buffer
  const size_t window = std::max<size_t>(kBurst, std::min<size_t>(1024, static_cast<size_t>(got_buf) / (payload + 33 + 1024)));

  tcpck_ctx *ctx = nullptr;
  char *arena = nullptr;
  const size_t cap = std::min(batch, segments);
  if (!cpu_only) {
    int st = tcpck_ctx_create(0, &ctx);
    if (st != TCPCK_OK) {
      std::fprintf(stderr, "tcpck_ctx_create: %s\n", tcpck_strerror(st));
      return 4;
    }
    void *p = nullptr;
    if (tcpck_host_alloc(cap * kSlot, &p) != TCPCK_OK) return 4;
    arena = static_cast<char *>(p);
    // first use allocates the context's device staging: keep it out of the timing
    std::memset(arena, 0, 64);
    uint64_t o = 0;
    uint32_t l = 64;
    uint8_t v = 0;
    if (tcpck_host_batch_var(ctx, TCPCK_OP_VERIFY, TCPCK_MODE_REF, arena, &o, &l, 1, &v) != TCPCK_OK) return 4;
  } else {
    arena = static_cast<char *>(std::aligned_alloc(4096, cap * kSlot));
  }
  std::vector<uint64_t> offsets(cap);
  std::vector<uint32_t> lengths(cap), gpu_len(cap);
  std::vector<uint8_t> ok(cap);
  for (size_t k = 0; k < cap; ++k) offsets[k] = k * kSlot;

  std::atomic<size_t> received{0};
  std::atomic<bool> send_failed{false};
  Stats st;
  const auto t_start = clk::now();
  std::thread sender(Sender, tx, std::cref(ra), segments, payload, corrupt_every, window, std::cref(received),
                     std::ref(send_failed));

  std::vector<mmsghdr> msgs(kBurst);
  std::vector<iovec> iov(kBurst);
  size_t nb = 0;  // datagrams in the current batch
  bool timed_out = false;
  auto flush = [&]() {
    if (nb == 0) return;
    ++st.batches;
    for (size_t k = 0; k < nb; ++k) gpu_len[k] = (lengths[k] & 1u) ? 0u : lengths[k];  // odd: CPU below
    if (!cpu_only) {
      const auto t0 = clk::now();
      const int rc = tcpck_host_batch_var(ctx, TCPCK_OP_VERIFY, TCPCK_MODE_REF, arena, offsets.data(),
                                          gpu_len.data(), nb, ok.data());
      st.gpu_ms += ms_since(t0);
      if (rc != TCPCK_OK) {
        std::fprintf(stderr, "tcpck_host_batch_var: %s\n", tcpck_strerror(rc));
        std::exit(5);
      }
    }
    for (size_t k = 0; k < nb; ++k) {
      const auto t0 = clk::now();
      auto pkt = MakeNetPacket(arena + offsets[k], lengths[k]);  // network-service.cc:56
      st.deliver_ms += ms_since(t0);
      const auto t1 = clk::now();
      const bool cpu_ok = CalculateChecksum(*pkt) == 0;  // socket-manager.h:182, one packet at a time
      st.cpu_ms += ms_since(t1);
      const bool odd = lengths[k] & 1u;
      st.odd += odd;
      const bool verdict = (cpu_only || odd) ? cpu_ok : ok[k] != 0;
      st.mismatches += verdict != cpu_ok;
      // the verdict travels with the packet: RecvPacket(packet, check_sum_validate)
      const uint32_t seq = ntohl(pkt->GetHeader().SequenceNumber());
      const bool corrupted = corrupt_every && seq % corrupt_every == corrupt_every - 1;
      st.flagged += !verdict;
      st.flagged_wrong += (!verdict) != corrupted;
      st.bytes += lengths[k];
    }
    nb = 0;
  };

  while (st.received < segments) {
    const size_t want = std::min({kBurst, cap - nb, segments - st.received});
    for (size_t i = 0; i < want; ++i) {
      iov[i] = {arena + offsets[nb + i], kSlot};
      std::memset(&msgs[i], 0, sizeof(mmsghdr));
      msgs[i].msg_hdr.msg_iov = &iov[i];
      msgs[i].msg_hdr.msg_iovlen = 1;
    }
    pollfd fds[1] = {{rx, POLLIN, 0}};
    const int pr = poll(fds, 1, 1000);  // network-service.cc:44
    if (pr == 0 || send_failed) {
      timed_out = true;
      break;
    }
    if (pr < 0) continue;
    const int r = recvmmsg(rx, msgs.data(), static_cast<unsigned>(want), MSG_DONTWAIT, nullptr);
    if (r <= 0) continue;
    for (int i = 0; i < r; ++i) {
      lengths[nb + i] = msgs[i].msg_len;
      st.truncated += (msgs[i].msg_hdr.msg_flags & MSG_TRUNC) != 0;
    }
    nb += static_cast<size_t>(r);
    st.received += static_cast<size_t>(r);
    received.store(st.received, std::memory_order_release);
    if (nb == cap || st.received == segments) flush();
  }
  flush();
  const double wall_ms = ms_since(t_start);
  received.store(segments + (1u << 30));  // release a sender still waiting on the window
  sender.join();
  close(rx);
  close(tx);
  if (ctx) {
    tcpck_host_free(arena);
    tcpck_ctx_destroy(ctx);
  } else {
    std::free(arena);
  }

  const size_t expected_bad = corrupt_every ? segments / corrupt_every : 0;
  const double gib = static_cast<double>(st.bytes) / (1u << 30);
  std::printf(
      "{\"config\": \"recv_burst\", \"segments\": %zu, \"payload\": %zu, \"slot\": %zu, \"batch\": %zu, \"window\": %zu, "
      "\"received\": %zu, \"lost\": %zu, \"truncated\": %zu, \"odd\": %zu, \"batches\": %zu, \"gpu\": %s, "
      "\"mismatches\": %zu, \"flagged\": %zu, \"expected_flagged\": %zu, \"flagged_wrong\": %zu, "
      "\"wall_ms\": %.1f, \"recv_GiBs\": %.3f, \"gpu_verify_ms\": %.2f, \"gpu_verify_GiBs\": %.2f, "
      "\"cpu_verify_ms\": %.2f, \"cpu_verify_GiBs\": %.2f, \"make_net_packet_ms\": %.2f}\n",
      segments, payload, kSlot, cap, window, st.received, segments - st.received, st.truncated, st.odd, st.batches,
      cpu_only ? "false" : "true", st.mismatches, st.flagged, expected_bad, st.flagged_wrong, wall_ms,
      gib / (wall_ms / 1e3), st.gpu_ms, st.gpu_ms > 0 ? gib / (st.gpu_ms / 1e3) : 0.0, st.cpu_ms,
      st.cpu_ms > 0 ? gib / (st.cpu_ms / 1e3) : 0.0, st.deliver_ms);
  const bool good = !timed_out && st.received == segments && st.mismatches == 0 && st.flagged_wrong == 0 &&
                    st.truncated == 0 && st.flagged == expected_bad;
  return good ? 0 : 1;
}
