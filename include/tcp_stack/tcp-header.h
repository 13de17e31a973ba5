// tcp_stack/tcp-header.h -- drop-in replacement for the reference's
// include/tcp-header.h (filixi/TCP-stack), backed by libtcpck.so.
//
// Same namespace, type names, member functions, byte layout and call syntax as
// the reference, so socket-manager.h / socket-manager.cc / socket-internal.h
// compile against it unchanged:
//
//   Field<N>                 tcp-header.h:13-50   (bit / byte accessors over N u32)
//   TcpHeader                tcp-header.h:52-191  (32 B: 12-B pseudo-header + 20-B TCP header)
//   TcpHeaderH2N / N2H       tcp-header.h:193-221
//   TcpPacket                tcp-header.h:223-292 (one contiguous [header | payload] image)
//   CalculateChecksum        tcp-header.h:252-263 (hidden friend, found by ADL)
//   operator<<               tcp-header.h:294, src/tcp-header.cc:4-19
//   MakeTcpPacket/MakeNetPacket  tcp-header.h:296-315
//
// CalculateChecksum forwards to tcpck_checksum16 (include/tcpck.h), the host
// single-image entry point: one image is far cheaper than a kernel launch, so
// per-packet calls stay on the calling thread.  Batches go to the GPU through
// tcpck_batch_fixed / tcpck_batch_var; see tcp_stack/packet-batch.h and
// INTEGRATION.md.
//
// Differences from the reference, all outside its defined behaviour:
//  * odd-length images: the reference reads 2 bytes past the end
//    (tcp-header.h:259-260, undefined).  Here the last byte is added as the low
//    byte of a zero-padded word (the RFC 1071 padding rule, in the reference's
//    mod-2^16 arithmetic), so odd payloads checksum and verify consistently.
#ifndef TCP_STACK_AMD_TCP_HEADER_H_
#define TCP_STACK_AMD_TCP_HEADER_H_

#include <arpa/inet.h>

#include <algorithm>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <ostream>
#include <utility>

// tcpck.h sits one directory up; a build that reaches this header through
// another path (e.g. a directory of symlinks) finds it on the include path
#if __has_include("../tcpck.h")
#include "../tcpck.h"
#else
#include "tcpck.h"
#endif

namespace tcp_stack {

// N 32-bit words addressed by bit position.  Bit p is bit p%32 of word p/32
// (the host's word order, as in the reference); byte views start at bit p/8 of
// the word array's memory.
template <size_t N>
class Field {
 public:
  static constexpr size_t kSize = N;

  Field() { std::memset(words_, 0, sizeof(words_)); }

  uint8_t GetAtBit(size_t pos) const {
    assert(pos < 32 * N);
    return static_cast<uint8_t>((words_[pos >> 5] >> (pos & 31)) & 1u);
  }

  void SetAtBit(size_t pos, bool value) {
    assert(pos < 32 * N);
    const uint32_t m = 1u << (pos & 31);
    words_[pos >> 5] = value ? (words_[pos >> 5] | m) : (words_[pos >> 5] & ~m);
  }

  template <class T>
  const T &At(size_t pos) const {
    assert(pos < 32 * N && pos % 8 == 0 && (pos / 8) % alignof(T) == 0);
    const unsigned char *b = reinterpret_cast<const unsigned char *>(words_) + pos / 8;
    return *reinterpret_cast<const T *>(b);
  }
  template <class T>
  T &At(size_t pos) {
    return const_cast<T &>(static_cast<const Field &>(*this).template At<T>(pos));
  }

 private:
  uint32_t words_[N];
};

// The 32-byte image header.  Byte offsets (tcp-header.h:59-185):
//   0 src addr  4 dst addr  8 zero  9 PTCL  10 TcpLength | 12 sport 14 dport
//   16 seq  20 ack  24 data offset (never set)  25 flags  26 window
//   28 checksum  30 urgent pointer
// Flag bits of byte 25 follow the reference (non-standard): URG 0x04, ACK 0x08,
// PSH 0x10, RST 0x20, SYN 0x40, FIN 0x80.
class TcpHeader {
 public:
  static constexpr size_t kChecksumOffset = 28;

#define TCP_STACK_FIELD(Name, T, field, bit)                              \
  T &Name() { return field.At<T>(bit); }                         \
  const T &Name() const { return field.At<T>(bit); }
  TCP_STACK_FIELD(SourceAddress, uint32_t, pseudo_, 0)
  TCP_STACK_FIELD(DestinationAddress, uint32_t, pseudo_, 32)
  TCP_STACK_FIELD(PTCL, uint8_t, pseudo_, 72)
  TCP_STACK_FIELD(TcpLength, uint16_t, pseudo_, 80)
  TCP_STACK_FIELD(SourcePort, uint16_t, tcp_, 0)
  TCP_STACK_FIELD(DestinationPort, uint16_t, tcp_, 16)
  TCP_STACK_FIELD(SequenceNumber, uint32_t, tcp_, 32)
  TCP_STACK_FIELD(AcknowledgementNumber, uint32_t, tcp_, 64)
  TCP_STACK_FIELD(Window, uint16_t, tcp_, 112)
  TCP_STACK_FIELD(Checksum, uint16_t, tcp_, 128)
  TCP_STACK_FIELD(UrgentPointer, uint16_t, tcp_, 144)
#undef TCP_STACK_FIELD

#define TCP_STACK_FLAG(Name, bit)                                         \
  bool Name() const { return tcp_.GetAtBit(bit) != 0; }                   \
  void Set##Name(bool value) { tcp_.SetAtBit(bit, value); }
  TCP_STACK_FLAG(Urg, 106)
  TCP_STACK_FLAG(Ack, 107)
  TCP_STACK_FLAG(Psh, 108)
  TCP_STACK_FLAG(Rst, 109)
  TCP_STACK_FLAG(Syn, 110)
  TCP_STACK_FLAG(Fin, 111)
#undef TCP_STACK_FLAG

 private:
  Field<3> pseudo_;  // 12-byte pseudo-header
  Field<5> tcp_;     // 20-byte TCP header
};

static_assert(sizeof(TcpHeader) == 32, "image header is 32 bytes (tcp-header.h:188-190)");
static_assert(alignof(TcpHeader) == 4, "u32-aligned header");

// Host <-> network order of the multi-byte fields; the checksum, flags and
// PTCL stay as they are (tcp-header.h:193-221).
inline void TcpHeaderH2N(TcpHeader &h) {
  h.SourceAddress() = htonl(h.SourceAddress());
  h.DestinationAddress() = htonl(h.DestinationAddress());
  h.TcpLength() = htons(h.TcpLength());
  h.SourcePort() = htons(h.SourcePort());
  h.DestinationPort() = htons(h.DestinationPort());
  h.SequenceNumber() = htonl(h.SequenceNumber());
  h.AcknowledgementNumber() = htonl(h.AcknowledgementNumber());
  h.Window() = htons(h.Window());
  h.UrgentPointer() = htons(h.UrgentPointer());
}

inline void TcpHeaderN2H(TcpHeader &h) {
  // byte swaps are involutions: ntoh == hton on every host
  TcpHeaderH2N(h);
}

// One segment image [32-B header | payload], owned, move-only.
class TcpPacket {
 public:
  TcpPacket(TcpPacket &&) = default;
  TcpPacket &operator=(TcpPacket &&) = default;

  TcpHeader &GetHeader() { return *reinterpret_cast<TcpHeader *>(buff_.get()); }
  const TcpHeader &GetHeader() const { return *reinterpret_cast<const TcpHeader *>(buff_.get()); }

  char *begin() { return buff_.get() + sizeof(TcpHeader); }
  const char *begin() const { return buff_.get() + sizeof(TcpHeader); }
  char *end() { return buff_.get() + size_; }
  const char *end() const { return buff_.get() + size_; }

  // ~(sum of the image's little-endian u16 words mod 2^16), tcp-header.h:252-263.
  friend uint16_t CalculateChecksum(const TcpPacket &packet) {
    return ImageChecksum(packet.buff_.get(), packet.size_);
  }

  std::pair<char *, size_t> GetBuffer() { return {buff_.get(), size_}; }

  // The single-image checksum used by CalculateChecksum (odd lengths: see the
  // file comment).  Public so batch code can checksum raw images the same way.
  static uint16_t ImageChecksum(const void *image, size_t size) {
    uint16_t c = 0;
    const int st = tcpck_checksum16(image, size & ~static_cast<size_t>(1), TCPCK_MODE_REF, &c);
    assert(st == TCPCK_OK);
    (void)st;
    if (size & 1) c = static_cast<uint16_t>(c - static_cast<const unsigned char *>(image)[size - 1]);
    return c;
  }

 protected:
  // Header-only allocation: the header is zeroed, the payload is not
  // (tcp-header.h:270-273).
  explicit TcpPacket(size_t payload)
      : size_(sizeof(TcpHeader) + payload), buff_(new char[sizeof(TcpHeader) + payload]) {
    new (buff_.get()) TcpHeader;
  }
  // Zeroed header followed by a copy of `payload` bytes (tcp-header.h:275-279).
  TcpPacket(const char *payload, size_t size) : TcpPacket(size) { std::copy(payload, payload + size, begin()); }
  // A raw wire image, header included (tcp-header.h:281-284).
  TcpPacket(const char *first, const char *last)
      : size_(static_cast<size_t>(last - first)), buff_(new char[static_cast<size_t>(last - first)]) {
    std::copy(first, last, buff_.get());
  }

 private:
  TcpPacket(const TcpPacket &) = delete;
  TcpPacket &operator=(const TcpPacket &) = delete;

  size_t size_;
  std::unique_ptr<char[]> buff_;
};

// Same text as src/tcp-header.cc:4-19 prints: flags, ports, seq, ack, length.
inline std::ostream &operator<<(std::ostream &o, const TcpHeader &h) {
  if (h.Ack()) o << "Ack ";
  if (h.Syn()) o << "Syn ";
  if (h.Rst()) o << "Rst ";
  if (h.Fin()) o << "Fin ";
  return o << h.SourcePort() << "->" << h.DestinationPort() << " S" << h.SequenceNumber() << " A"
           << h.AcknowledgementNumber() << " L" << h.TcpLength();
}

namespace detail {
struct PacketAccess : TcpPacket {
  explicit PacketAccess(size_t n) : TcpPacket(n) {}
  PacketAccess(const char *p, size_t n) : TcpPacket(p, n) {}
  PacketAccess(const char *a, const char *b) : TcpPacket(a, b) {}
};
}  // namespace detail

inline std::shared_ptr<TcpPacket> MakeTcpPacket(size_t size) {
  return std::make_shared<detail::PacketAccess>(size);
}
inline std::shared_ptr<TcpPacket> MakeTcpPacket(const char *buff, size_t size) {
  return std::make_shared<detail::PacketAccess>(buff, size);
}
inline std::shared_ptr<TcpPacket> MakeNetPacket(const char *buff, size_t size) {
  return std::make_shared<detail::PacketAccess>(buff, buff + size);
}

}  // namespace tcp_stack

#endif  // TCP_STACK_AMD_TCP_HEADER_H_
