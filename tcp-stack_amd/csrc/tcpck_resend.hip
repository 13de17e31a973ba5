// tcpck_resend.hip -- batched retransmit: ACK-number rewrite with an
// incremental checksum update, one lane per image.
//
// The reference's resend path rewrites the ACK number of every queued packet
// (ResendPredicate, include/socket-internal.h:376-377:
//   packet->GetHeader().AcknowledgementNumber() = htonl(rcv_nxt)
// ) and then recomputes the checksum over the whole image (SendPacket,
// src/socket-manager.cc:9-10).  Only two u16 words of the image change (bytes
// 20-23: TcpHeader::field_ bit 64, tcp-header.h:117, after the 12-byte pseudo
// header), so the stored checksum C (bytes 28-29, tcp-header.h:177) is updated
// from the old and new words instead:
//   REF     (tcp-header.h:252-263, sums mod 2^16):  C' = ~(~C - o0 - o1 + n0 + n1)
//   RFC1071 (opt-in, RFC 1624 eqn. 3):              C' = ~(~C + ~o0 + ~o1 + n0 + n1),
//           end-around carry; a folded +0 becomes 0xFFFF (a TCP image is
//           never all zero: PTCL = 6 in the pseudo header)
// Both equal the full recompute whenever C was the valid checksum of the old
// image (written by FILL / SendPacket).  Per image: 6 bytes read, 6 bytes
// written, no payload bytes touched -- the kernel is bound by scattered
// sub-line accesses (one 128-B line per image), not by streaming bandwidth.
#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;

template <int MODE>
__device__ __forceinline__ uint16_t update_ack(uint16_t c, uint16_t o0, uint16_t o1, uint16_t n0, uint16_t n1) {
  if constexpr (MODE == kRef) {
    const uint32_t s = static_cast<uint16_t>(~c) - o0 - o1 + n0 + n1;
    return static_cast<uint16_t>(~s);
  } else {
    uint32_t s = static_cast<uint32_t>(static_cast<uint16_t>(~c)) + static_cast<uint16_t>(~o0) +
                 static_cast<uint16_t>(~o1) + n0 + n1;
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    if (s == 0) s = 0xFFFFu;
    return static_cast<uint16_t>(~s);
  }
}

template <int MODE, bool FIXED, bool PER_IMAGE>
__global__ void __launch_bounds__(kBlock) set_ack_kernel(AckArgs a) {
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; k < a.count; k += step) {
    const uint64_t start = FIXED ? k * a.stride : a.offsets[k];
    uint16_t *w = reinterpret_cast<uint16_t *>(a.arena + start);  // even offsets: u16-aligned
    const uint16_t o0 = w[10], o1 = w[11], c = w[14];
    // htonl(ack) stored raw: memory bytes 20..23 = ack >> 24, >> 16, >> 8, ack
    const uint32_t net = __builtin_bswap32(PER_IMAGE ? a.acks[k] : a.ack);
    const uint16_t n0 = static_cast<uint16_t>(net), n1 = static_cast<uint16_t>(net >> 16);
    const uint16_t c2 = update_ack<MODE>(c, o0, o1, n0, n1);
    w[10] = n0;
    w[11] = n1;
    w[14] = c2;
    if (a.out) a.out[k] = c2;
  }
}

template <int MODE, bool FIXED, bool PER_IMAGE>
hipError_t launch_one(const AckArgs &a, uint32_t num_cus, hipStream_t s) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(set_ack_kernel<MODE, FIXED, PER_IMAGE>);
  uint64_t blocks = (a.count + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * 8;  // grid-stride beyond 8 resident grids
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((set_ack_kernel<MODE, FIXED, PER_IMAGE>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                     s, a);
  return hipGetLastError();
}

template <int MODE>
hipError_t dispatch(const AckArgs &a, uint32_t num_cus, hipStream_t s) {
  const bool fixed = a.offsets == nullptr, per = a.acks != nullptr;
  if (fixed) return per ? launch_one<MODE, true, true>(a, num_cus, s) : launch_one<MODE, true, false>(a, num_cus, s);
  return per ? launch_one<MODE, false, true>(a, num_cus, s) : launch_one<MODE, false, false>(a, num_cus, s);
}

}  // namespace

hipError_t launch_set_ack(int mode, const AckArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  return mode == kRef ? dispatch<kRef>(a, num_cus, stream) : dispatch<kRfc1071>(a, num_cus, stream);
}

}  // namespace tcpck
