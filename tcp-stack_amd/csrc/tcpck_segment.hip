// tcpck_segment.hip -- the send path's producer, batched: a device-resident
// send stream cut into checksummed TCP images in one pass (segmentation +
// header + checksum fill).
//
// Reference (filixi/TCP-stack), per data segment:
//   TcpSendingBuffer::GetAsTcpPacket(0, window)     include/tcp-buffer.h:82-98
//     MakeTcpPacket(len), the payload copied byte by byte out of a deque
//     (tcp-buffer.h:33-35), TcpLength = len
//   Estab, Event::kSend                             src/state.cc:167-184
//     SetAck, seq = snd_nxt, ack = rcv_nxt, snd_nxt += len
//   SetSource / SetDestination, TcpHeaderH2N        include/socket-internal.h:186-199
//   Checksum() = 0; Checksum() = CalculateChecksum  include/socket-manager.h:259-260
// Here the per-connection fields come as a 32-B network-order header template
// (TcpLength and seq 0); image k = template with TcpLength = htons(len_k) and
// seq = htonl(seq0 + k seg), then payload bytes [k seg, k seg + len_k), its
// checksum in bytes 28-29 (raw, as the reference), written at k * stride of
// the output (stride a multiple of 16: every image starts 16-B aligned; the
// slot's bytes after the image are written 0).
//
// One run of whole images per wave, one output 16-B chunk per lane and step:
//   * chunk q of the run is chunk j = q - i nc of image i = q / nc (nc =
//     stride / 16; multiply-high by a launcher-computed magic number): j = 0, 1
//     are the header (from the template in SGPRs), j >= 2 payload bytes 16 (j -
//     2) .. of the image, loaded from the stream (4-B aligned when seg % 4 ==
//     0), the bytes past the image zeroed;
//   * U steps of loads in flight (buffer loads, out-of-range for header and
//     padding chunks: no traffic); each chunk is stored as it is consumed,
//     except header chunk 1, which holds the checksum;
//   * the image sums come from one 64-lane inclusive scan per step: every image
//     ends at a chunk boundary of the output, so sum(k) = P(end of its last
//     chunk) - P(its start), P read from the scan with one cross-lane pull
//     (ds_bpermute) per ending image, the start by DPP wave_shr:1 from the image
//     before; u32 differences are exact, so RFC 1071 mode folds them;
//   * the lane that resolves image k stores out[k] and the whole header chunk 1
//     (seq, window/flags from the template, checksum, urgent pointer) -- one
//     16-B store, not a 2-B patch.
// The last chunk of the whole stream is read dword by dword inside the stream's
// bytes (the stream may end 2 B into a dword).
#include <algorithm>

#include "tcpck_device.h"
#include "tcpck_internal.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

template <int U, int MODE, int SPOL, int LPOL = 2>
__global__ void __launch_bounds__(kBlock) segment_kernel(SegmentArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint64_t wid = static_cast<uint64_t>(bid) * kWavesPerBlock + wv;
  uint64_t kb, ke;
  dev::count_split(wid, a.per_wave, a.rem, kb, ke);
  if (kb >= ke) return;
  const uint32_t nimg = static_cast<uint32_t>(ke - kb);
  const uint32_t S = a.seg;
  const uint32_t nc = a.nchunk;
  const uint64_t p0 = kb * S;
  // the run's stream bytes, plus up to 16 B of the next run's: the last chunk of
  // an image that ends inside a chunk is read whole and masked (< 2^31, launcher)
  const uint32_t in_ext = static_cast<uint32_t>(min(ke * static_cast<uint64_t>(S) + 16, a.payload_bytes) - p0);
  // image i of the run: payload length (the batch's last image is shorter)
  const bool has_last = ke == a.count;
  const uint32_t last_len = static_cast<uint32_t>(a.payload_bytes - (a.count - 1) * static_cast<uint64_t>(S));
  const auto rin = dev::make_rsrc(a.payload + p0, in_ext);
  const auto rout = dev::make_rsrc(a.images + kb * static_cast<uint64_t>(a.stride), nimg * a.stride);
  const uint32_t T = nimg * nc;  // output chunks of the run
  const uint32_t nsteps = (T + 63) >> 6;
  constexpr uint32_t kNone = 0xFFFFFFF0u;  // out of every buffer range: no traffic, reads 0

  auto image_of = [&](uint32_t q) -> uint32_t {
    return a.magic ? (__umulhi(q, a.magic) >> a.shift) : (q >> a.shift);
  };
  auto len_of = [&](uint32_t i) -> uint32_t { return (has_last && i == nimg - 1) ? last_len : S; };
  // a chunk that would read past the stream's end (the batch's last image, or
  // the run's last image with < 16 B of stream after it) is read dword by
  // dword inside the image (the stream may end inside a dword); every other
  // payload chunk is one whole 16-B load
  auto is_tail = [&](uint32_t i, uint32_t j, uint32_t len) -> bool {
    return j >= 2 && 16 * (j - 2) < len && i * S + 16 * (j - 2) + 16 > in_ext;
  };
  auto load_step = [&](uint32_t t) -> u32x4 {
    const uint32_t q = (t << 6) + lane;
    const uint32_t i = image_of(q);
    const uint32_t j = q - i * nc;
    uint32_t voff = kNone;
    if (i < nimg && j >= 2) {
      const uint32_t pb = 16 * (j - 2);
      const uint32_t len = len_of(i);
      if (pb < len && !is_tail(i, j, len)) voff = i * S + pb;
    }
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rin, static_cast<int>(voff), 0, LPOL);
    return u32x4{v.x, v.y, v.z, v.w};
  };
  auto store16 = [&](uint32_t voff, u32x4 w) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = {w.x, w.y, w.z, w.w};
    // SPOL 0 nt, 1 default, 2 sc1, 3 sc1 nt, 4 sc0 sc1 nt (write-through streaming)
    constexpr int aux = SPOL == 0 ? 2 : (SPOL == 2 ? 16 : (SPOL == 3 ? 18 : (SPOL == 4 ? 19 : 0)));
    __builtin_amdgcn_raw_buffer_store_b128(v, rout, static_cast<int>(voff), 0, aux);
  };
  auto header1 = [&](uint32_t i, uint32_t csum) -> u32x4 {  // bytes 16-31: seq, ack, flags/window, checksum/urgent
    const uint32_t seq = a.seq0 + static_cast<uint32_t>((kb + i) * static_cast<uint64_t>(S));
    return u32x4{bswap32(seq), a.hdr[5], a.hdr[6], (a.hdr[7] & 0xFFFF0000u) | (csum & 0xFFFFu)};
  };

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = load_step(static_cast<uint32_t>(u));

  uint32_t carry = 0, p_last = 0, jn = 0;
  for (uint32_t g = 0; g < nsteps; g += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t st = g + u;
      const uint32_t q = (st << 6) + lane;
      const uint32_t i = image_of(q);
      const uint32_t j = q - i * nc;
      const bool live = q < T;
      u32x4 w = ring[u];
      if (live) {
        const uint32_t len = len_of(i);
        if (j == 0) {  // bytes 0-15: addresses, zero/PTCL, TcpLength (network order), ports
          w = u32x4{a.hdr[0], a.hdr[1], (a.hdr[2] & 0x0000FFFFu) | (bswap16(len) << 16), a.hdr[3]};
        } else if (j == 1) {
          w = header1(i, 0u);  // checksum 0 in the sum (socket-manager.h:259)
        } else {
          const uint32_t pb = 16 * (j - 2);
          if (is_tail(i, j, len)) {
            const uint32_t base = i * S + pb, valid = len - pb;  // even, < 16
            uint32_t d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t b = 4 * k;
              d[k] = b + 4 <= valid ? __builtin_amdgcn_raw_buffer_load_b32(rin, static_cast<int>(base + b), 0, 0)
                                    : (b + 2 <= valid ? static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(
                                                            rin, static_cast<int>(base + b), 0, 0))
                                                      : 0u);
            }
            w = u32x4{d[0], d[1], d[2], d[3]};
          } else if (pb + 16 > len) {
            w = dev::apply_mask(w, dev::word_mask(0, static_cast<int32_t>(pb < len ? len - pb : 0)));
          }
        }
        if (j != 1) store16(q << 4, w);
      } else {
        w = u32x4{0u, 0u, 0u, 0u};
      }
      const uint32_t tot = dev::ref_chunk_sum_dot(w);
      const uint32_t incl = dev::wave_inclusive_scan(tot);
      // images ending in this step: lane l takes image jn + l (at most 22: nc >= 3)
      const uint32_t ie = jn + lane;
      const uint32_t e = ie < nimg ? (ie + 1) * nc - 1 - (st << 6) : ~0u;  // its last chunk, step-relative
      const bool inb = e < 64;
      const uint64_t bal = __ballot(inb);
      const uint32_t pe = carry + static_cast<uint32_t>(__shfl(static_cast<int>(incl), static_cast<int>(e & 63u), 64));
      const uint32_t pprev = static_cast<uint32_t>(
          __builtin_amdgcn_update_dpp(static_cast<int>(p_last), static_cast<int>(pe), 0x138, 0xF, 0xF, false));
      if (inb) {
        const uint16_t c = dev::finish<MODE>(pe - pprev);
        if (a.out) a.out[kb + ie] = c;
        store16((ie * nc + 1) << 4, header1(ie, c));
      }
      if (bal) {
        const uint32_t cnt = static_cast<uint32_t>(__popcll(bal));
        p_last = dev::read_lane(pe, cnt - 1);
        jn += cnt;
      }
      carry += dev::read_lane(incl, 63);
      ring[u] = load_step(st + U);
    }
  }
}

// Jumbo segments: the block's W waves stream ONE image together, wave w taking
// the image's 1 KiB steps w, w + W, ... (so the block reads W KiB of the image
// per round, front to back), lane sums accumulated, the W partial sums met in
// LDS; the block then takes the next image (grid-stride).  With one image per
// wave, 64-KiB segments left few waves and a last round running alone.
template <int W, int U, int MODE>
__global__ void __launch_bounds__(64 * W) segment_wide_kernel(SegmentArgs a) {
  __shared__ uint32_t s_part[W];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
  const uint32_t S = a.seg, nc = a.nchunk;
  const uint32_t nsteps = (nc + 63) >> 6;
  const uint32_t bid = dev::ordered_block(blockIdx.x, gridDim.x, a.order);
  const uint32_t last_len = static_cast<uint32_t>(a.payload_bytes - (a.count - 1) * static_cast<uint64_t>(S));
  for (uint64_t k = bid; k < a.count; k += gridDim.x) {
    const uint64_t p0 = k * S;
    const uint32_t len = k + 1 == a.count ? last_len : S;
    const auto rin = dev::make_rsrc(a.payload + p0, len);  // exactly the image's payload
    const auto rout = dev::make_rsrc(a.images + k * static_cast<uint64_t>(a.stride), a.stride);
    // chunks j >= 2 whose 16 B pass the payload's end are read dword by dword
    auto load_step = [&](uint32_t t) -> u32x4 {
      const uint32_t j = (t << 6) + lane;
      uint32_t voff = 0xFFFFFFF0u;
      if (j >= 2 && j < nc && 16 * (j - 2) + 16 <= len) voff = 16 * (j - 2);
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rin, static_cast<int>(voff), 0, 0);
      return u32x4{v.x, v.y, v.z, v.w};
    };
    u32x4 ring[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ring[u] = load_step(wv + W * u);
    uint32_t acc = 0;
    for (uint32_t g = wv; g < nsteps; g += W * U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t t = g + W * u;
        const uint32_t j = (t << 6) + lane;
        u32x4 w = ring[u];
        if (j < nc) {
          if (j == 0) {
            w = u32x4{a.hdr[0], a.hdr[1], (a.hdr[2] & 0x0000FFFFu) | (bswap16(len) << 16), a.hdr[3]};
          } else if (j == 1) {
            const uint32_t seq = a.seq0 + static_cast<uint32_t>(k * S);
            w = u32x4{bswap32(seq), a.hdr[5], a.hdr[6], a.hdr[7] & 0xFFFF0000u};
          } else {
            const uint32_t pb = 16 * (j - 2);
            if (pb >= len) {
              w = u32x4{0u, 0u, 0u, 0u};
            } else if (pb + 16 > len) {
              const uint32_t valid = len - pb;
              uint32_t d[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const uint32_t b = 4 * q;
                d[q] = b + 4 <= valid ? __builtin_amdgcn_raw_buffer_load_b32(rin, static_cast<int>(pb + b), 0, 0)
                                      : (b + 2 <= valid ? static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(
                                                              rin, static_cast<int>(pb + b), 0, 0))
                                                        : 0u);
              }
              w = u32x4{d[0], d[1], d[2], d[3]};
            }
          }
          if (j != 1) {
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const v4u v = {w.x, w.y, w.z, w.w};
            __builtin_amdgcn_raw_buffer_store_b128(v, rout, static_cast<int>(j << 4), 0, 0);
          }
        } else {
          w = u32x4{0u, 0u, 0u, 0u};
        }
        acc += dev::ref_chunk_sum_dot(w);  // < 2^32 for an image < 128 KiB: exact
        ring[u] = load_step(t + W * U);
      }
    }
    acc = dev::group_sum<64>(acc);
    if (lane == 0) s_part[wv] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t sum = 0;
#pragma unroll
      for (int i = 0; i < W; ++i) sum += s_part[i];
      const uint16_t c = dev::finish<MODE>(sum);
      if (a.out) a.out[k] = c;
      const uint32_t seq = a.seq0 + static_cast<uint32_t>(k * S);
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      const v4u v = {bswap32(seq), a.hdr[5], a.hdr[6], (a.hdr[7] & 0xFFFF0000u) | c};
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, 16, 0, 0);
    }
    __syncthreads();  // s_part is rewritten for the next image
  }
}

template <int W, int U, int MODE>
hipError_t launch_wide(SegmentArgs a, uint32_t oversub, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = [] {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, segment_wide_kernel<W, U, MODE>, 64 * W, 0) != hipSuccess ||
        nb < 1)
      nb = 1;
    return static_cast<uint32_t>(nb);
  }();
  // one block per image up to 64 x the resident grid (grid-stride past it):
  // cold, 1.6 GB of stream, 9000 / 16000 / 65532-B segments ran 65.2 / 63.6 /
  // 66.8 % of the roof (read + write) at the former 4 x, 70.2 / 69.1 / 70.1 % at
  // 64 x (profiles/r05/segment_wide2_s5.log)
  uint64_t blocks = a.count;
  const uint64_t cap = static_cast<uint64_t>(per_cu) * num_cus * (oversub ? oversub : 64);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL((segment_wide_kernel<W, U, MODE>), dim3(static_cast<uint32_t>(blocks)), dim3(64 * W), 0, stream, a);
  return hipGetLastError();
}

template <int U, int MODE, int SPOL, int LPOL = 2>
hipError_t launch_one(SegmentArgs a, uint32_t oversub, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(segment_kernel<U, MODE, SPOL, LPOL>);
  const uint64_t resident = static_cast<uint64_t>(per_cu) * num_cus;
  const uint64_t out_bytes = a.count * static_cast<uint64_t>(a.stride);
  // runs of ~3 KiB of output (two 1.5-KB images): M = the power of two
  // nearest (in ratio) to out_bytes / (resident waves x 3 KiB), up to 1024.
  // Measured cold at 0.40 / 1.58 / 6.6 GB of images, the best M is the power
  // of two giving 3.0-3.2-KiB runs (69.3 % at M 16, 71.0 % at M 64, 68.9 % at
  // M 256 of the roof in read + write traffic; M 56 / 72 at 1.58 GB 69.7 /
  // 69.8 %); rounding DOWN to a power of two put the bench's 1.58 GB at M 32
  // (6-KiB runs, 66.7 %) (scripts/segment_probe.py, profiles/r05/segment_m_*.log)
  uint64_t m = oversub;
  if (!m) {
    const double q = static_cast<double>(out_bytes) / static_cast<double>(resident * kWavesPerBlock * (3u << 10));
    m = 1;
    while (m < 1024 && q >= 1.4142135623730951 * static_cast<double>(m)) m *= 2;
  }
  uint64_t blocks = resident * m;
  const uint64_t need = (a.count + kWavesPerBlock - 1) / kWavesPerBlock;
  // runs below 2^30 bytes of output (u32 run arithmetic)
  const uint64_t per_max = std::max<uint64_t>(1, (uint64_t{1} << 30) / a.stride);
  const uint64_t least = (a.count + per_max * kWavesPerBlock - 1) / (per_max * kWavesPerBlock);
  if (blocks < least) blocks = least;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
  a.per_wave = a.count / (blocks * kWavesPerBlock);
  a.rem = a.count % (blocks * kWavesPerBlock);
  hipLaunchKernelGGL((segment_kernel<U, MODE, SPOL, LPOL>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int U, int SPOL, int LPOL = 2>
hipError_t by_mode(int mode, const SegmentArgs &a, uint32_t m, uint32_t num_cus, hipStream_t s) {
  return mode == kRef ? launch_one<U, kRef, SPOL, LPOL>(a, m, num_cus, s)
                      : launch_one<U, kRfc1071, SPOL, LPOL>(a, m, num_cus, s);
}

}  // namespace

hipError_t launch_segment(int mode, int variant, SegmentArgs a, uint32_t oversub, uint32_t num_cus, hipStream_t stream) {
  if (a.count == 0) return hipSuccess;
  a.nchunk = a.stride / 16;
  uint32_t sh = 0;
  while ((2u << sh) <= a.nchunk) ++sh;  // floor(log2 nchunk)
  a.shift = sh;
  a.magic = (a.nchunk & (a.nchunk - 1)) == 0
                ? 0u
                : static_cast<uint32_t>(((uint64_t{1} << (32 + sh)) + a.nchunk - 1) / a.nchunk);
  a.order = (variant & 8) ? dev::kOrderDefault : 4u;  // groups of 16 blocks per XCD
  // variant & 7: 0 = policy, 1 = U4 nt stores, 2 = U4 default-policy stores,
  // 3 = U4 sc1 stores, 4 = U8 default-policy stores, 5 = U8 nt stores, 6 = 2 with
  // default-policy loads
#ifdef TCPCK_PROBE
  if (variant & 0xC0) {  // the policy's MSS form with write-through stores: 0x40 sc1 nt, 0x80 sc0 sc1 nt
    if (a.seg >= 8192) return hipErrorInvalidValue;
    return (variant & 0x80) ? by_mode<4, 4, 0>(mode, a, oversub, num_cus, stream)
                            : by_mode<4, 3, 0>(mode, a, oversub, num_cus, stream);
  }
#endif
  switch (variant & 7) {  // (bit 3: default block order)
    // policy: default-policy stores (66.6 vs 61.2 % with nt at M = 32) and loads
    // (9000-B segments 64.2 vs 60.6 %; MSS +0.2-0.5 %: the 4-B offset loads of
    // 1460-B segments split lines between steps), profiles/r02/segment_probe4.log
    // jumbo segments stream with W waves per image (segment_probe5.log): 65532 B
    // W16 67.4 % against 60.5 % one image per wave, 16 KiB 68.5 vs 60.9 %, 9000 B
    // W4 65.4 vs 64.1 %; below 8 KiB (MSS) the run kernel (W4 at 1460 B: 35 %)
    case 0:
      if (a.seg >= 16384)
        return mode == kRef ? launch_wide<16, 2, kRef>(a, oversub, num_cus, stream)
                            : launch_wide<16, 2, kRfc1071>(a, oversub, num_cus, stream);
      if (a.seg >= 8192)
        return mode == kRef ? launch_wide<4, 4, kRef>(a, oversub, num_cus, stream)
                            : launch_wide<4, 4, kRfc1071>(a, oversub, num_cus, stream);
      return by_mode<4, 1, 0>(mode, a, oversub, num_cus, stream);
#ifdef TCPCK_PROBE
    // measurement-only variants (libtcpck_probe.so)
    case 1: return by_mode<4, 0>(mode, a, oversub, num_cus, stream);
    case 2: return by_mode<4, 1>(mode, a, oversub, num_cus, stream);
    case 3: return by_mode<4, 2>(mode, a, oversub, num_cus, stream);
    case 4: return by_mode<8, 1>(mode, a, oversub, num_cus, stream);
    case 5: return by_mode<8, 0>(mode, a, oversub, num_cus, stream);
    case 6: return by_mode<4, 1, 0>(mode, a, oversub, num_cus, stream);  // default-policy loads too
    case 7: {  // W waves per image (variant >> 4: 0 -> 4, 1 -> 8, 2 -> 16)
      const int wsel = (variant >> 4) & 3;
      if (wsel == 1) return mode == kRef ? launch_wide<8, 4, kRef>(a, oversub, num_cus, stream)
                                         : launch_wide<8, 4, kRfc1071>(a, oversub, num_cus, stream);
      if (wsel == 2) return mode == kRef ? launch_wide<16, 2, kRef>(a, oversub, num_cus, stream)
                                         : launch_wide<16, 2, kRfc1071>(a, oversub, num_cus, stream);
      return mode == kRef ? launch_wide<4, 4, kRef>(a, oversub, num_cus, stream)
                          : launch_wide<4, 4, kRfc1071>(a, oversub, num_cus, stream);
    }
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
