// tcp_stack/packet-batch.h -- batched send-side fill and receive-side verify
// for the reference's call sites, on top of the drop-in tcp_stack/tcp-header.h.
//
// The reference checksums one packet at a time:
//   send     include/socket-manager.h:259-260, src/socket-manager.cc:9-10
//            hdr.Checksum() = 0; hdr.Checksum() = CalculateChecksum(*pkt);
//   receive  include/socket-manager.h:182
//            bool ok = CalculateChecksum(*pkt) == 0;
// PacketBatch does the same for a whole vector of packets (e.g. everything the
// per-socket loop of SendPacketsForSending, socket-manager.h:256-263, drains
// in one tick, or one recvmmsg burst): the images are gathered back to back
// into a pinned host arena, checksummed on the GPU by tcpck_host_batch_var
// (chunked H2D -> kernel -> D2H), and the 2-byte results are scattered back.
// Small batches, and odd-length images, stay on the calling thread, where a
// packet costs ~0.1 us instead of a launch.
//
// Results are identical to calling CalculateChecksum per packet.  Not
// thread-safe: one PacketBatch per thread (each owns its tcpck contexts and a
// staging arena).  Given several devices, a batch is split over all of them
// (tcpck_host_batch_var_multi: contiguous shards balanced by bytes, one host
// thread and PCIe link per GPU).
#ifndef TCP_STACK_AMD_PACKET_BATCH_H_
#define TCP_STACK_AMD_PACKET_BATCH_H_

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "tcp-header.h"

namespace tcp_stack {

// Incremental update of a stored checksum when one aligned u32 field of the
// image (raw, as stored: network order) changes, e.g. the ACK-number rewrite
// of a retransmit (socket-internal.h:376-377), instead of the full recompute
// that SendPacket then does (socket-manager.cc:9-10).  Exact in the
// reference's mod-2^16 arithmetic: C' = ~(~C - old + new).
inline uint16_t UpdateChecksum32(uint16_t checksum, uint32_t old_raw, uint32_t new_raw) {
  uint16_t o[2], n[2];
  std::memcpy(o, &old_raw, 4);
  std::memcpy(n, &new_raw, 4);
  checksum = tcpck_update16(checksum, o[0], n[0], TCPCK_MODE_REF);
  return tcpck_update16(checksum, o[1], n[1], TCPCK_MODE_REF);
}

class PacketBatch {
 public:
  // Batches with fewer images or bytes than these stay on the CPU.
  struct Thresholds {
    size_t min_images = 256;
    size_t min_bytes = 1u << 20;
  };

  explicit PacketBatch(int device = 0) : PacketBatch(device, Thresholds()) {}
  PacketBatch(int device, Thresholds t) : PacketBatch(std::vector<int>{device}, t) {}
  // One context per listed device (a device may appear more than once).
  PacketBatch(const std::vector<int> &devices, Thresholds t) : thresholds_(t) {
    if (devices.empty()) throw std::invalid_argument("PacketBatch: no device");
    for (int d : devices) {
      tcpck_ctx *c = nullptr;
      const int st = tcpck_ctx_create(d, &c);
      if (st != TCPCK_OK) {
        Release();
        Check(st, "tcpck_ctx_create");
      }
      ctxs_.push_back(c);
    }
  }
  ~PacketBatch() { Release(); }
  PacketBatch(const PacketBatch &) = delete;
  PacketBatch &operator=(const PacketBatch &) = delete;

  void set_thresholds(Thresholds t) { thresholds_ = t; }

  // Send side: zero bytes 28-29 of every image, compute, store in place.
  void Fill(const std::vector<std::shared_ptr<TcpPacket>> &pkts) {
    Run(pkts, TCPCK_OP_FILL);
    for (size_t k = 0; k < pkts.size(); ++k) pkts[k]->GetHeader().Checksum() = sums_[k];
  }

  // Receive side: ok[k] = (CalculateChecksum(*pkts[k]) == 0).
  std::vector<uint8_t> Verify(const std::vector<std::shared_ptr<TcpPacket>> &pkts) {
    Run(pkts, TCPCK_OP_CHECKSUM);
    std::vector<uint8_t> ok(pkts.size());
    for (size_t k = 0; k < pkts.size(); ++k) ok[k] = sums_[k] == 0;
    return ok;
  }

  // Plain checksums, as CalculateChecksum would return them.
  const std::vector<uint16_t> &Checksums(const std::vector<std::shared_ptr<TcpPacket>> &pkts) {
    Run(pkts, TCPCK_OP_CHECKSUM);
    return sums_;
  }

  // Images that went to the GPU in the last call (the rest ran on the CPU).
  size_t last_gpu_images() const { return last_gpu_; }

 private:
  static const char *Image(const TcpPacket &p) { return reinterpret_cast<const char *>(&p.GetHeader()); }
  static size_t Size(const TcpPacket &p) { return static_cast<size_t>(p.end() - Image(p)); }

  static void Check(int st, const char *what) {
    if (st != TCPCK_OK) throw std::runtime_error(std::string(what) + ": " + tcpck_strerror(st));
  }

  // Fills sums_ (FILL: the value to store; CHECKSUM: the checksum).  A FILL
  // result equals the checksum of the image with bytes 28-29 zeroed.
  void Run(const std::vector<std::shared_ptr<TcpPacket>> &pkts, int op) {
    const size_t n = pkts.size();
    sums_.assign(n, 0);
    idx_.clear();
    offsets_.clear();
    lengths_.clear();
    uint64_t bytes = 0;
    for (size_t k = 0; k < n; ++k) {
      const size_t len = Size(*pkts[k]);
      if ((len & 1) || len < 32 || len > 0xFFFFFFFFu) continue;  // CPU: odd or short images
      idx_.push_back(k);
      offsets_.push_back(bytes);
      lengths_.push_back(static_cast<uint32_t>(len));
      bytes += len;
    }
    last_gpu_ = 0;
    const bool gpu = idx_.size() >= thresholds_.min_images && bytes >= thresholds_.min_bytes;
    if (gpu) {
      Reserve(bytes);
      for (size_t j = 0; j < idx_.size(); ++j) std::memcpy(arena_ + offsets_[j], Image(*pkts[idx_[j]]), lengths_[j]);
      out_.resize(idx_.size());
      Check(tcpck_host_batch_var_multi(ctxs_.data(), static_cast<int>(ctxs_.size()), op, TCPCK_MODE_REF, arena_,
                                       offsets_.data(), lengths_.data(), idx_.size(), out_.data()),
            "tcpck_host_batch_var_multi");
      for (size_t j = 0; j < idx_.size(); ++j) sums_[idx_[j]] = out_[j];
      last_gpu_ = idx_.size();
    }
    size_t j = 0;
    for (size_t k = 0; k < n; ++k) {
      if (gpu && j < idx_.size() && idx_[j] == k) {
        ++j;
        continue;
      }
      TcpPacket &p = *pkts[k];
      if (op == TCPCK_OP_FILL) p.GetHeader().Checksum() = 0;
      sums_[k] = CalculateChecksum(p);
    }
  }

  void Release() {
    if (arena_) tcpck_host_free(arena_);
    arena_ = nullptr;
    for (tcpck_ctx *c : ctxs_) tcpck_ctx_destroy(c);
    ctxs_.clear();
  }

  void Reserve(uint64_t bytes) {
    if (bytes <= cap_) return;
    if (arena_) tcpck_host_free(arena_);
    arena_ = nullptr;
    cap_ = 0;
    void *p = nullptr;
    Check(tcpck_host_alloc(bytes + (bytes >> 2), &p), "tcpck_host_alloc");
    arena_ = static_cast<char *>(p);
    cap_ = bytes + (bytes >> 2);
  }

  std::vector<tcpck_ctx *> ctxs_;
  Thresholds thresholds_;
  char *arena_ = nullptr;
  uint64_t cap_ = 0;
  size_t last_gpu_ = 0;
  std::vector<size_t> idx_;
  std::vector<uint64_t> offsets_;
  std::vector<uint32_t> lengths_;
  std::vector<uint16_t> out_;
  std::vector<uint16_t> sums_;
};

}  // namespace tcp_stack

#endif  // TCP_STACK_AMD_PACKET_BATCH_H_
