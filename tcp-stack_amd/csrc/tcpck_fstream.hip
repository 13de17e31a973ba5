// tcpck_fstream.hip -- fixed-stride packed batches (stride == image length):
// the hot path of BASELINE configs C2 / C5 (1,048,576 x 1492-B images per GPU).
//
// Reference semantics: CalculateChecksum, include/tcp-header.h:252-263:
// ~(sum of the image's LE u16 words mod 2^16).  With images back to back at a
// fixed stride S, image k is bytes [kS, (k+1)S), and
//     sum(k) = P((k+1)S) - P(kS)  (mod 2^16),  P(x) = word sum before byte x,
// so the arena is read as a flat stream and never split per image.
//
// Work split: tiles of T images (T*S >= U KiB), wave w takes tiles
// w, w+W, w+2W, ... (W = waves in the grid): all waves sweep the arena together
// as one moving front, every wave has the same number of bytes, and the last
// tile ends within one tile time of the others.
//
// Per wave, steps of 1 KiB: lane l reads the 16 B at 1024 s + 16 l of the
// tile's run, the run start rounded down to a 128-B line (so one step covers
// exactly eight whole lines); U steps are in flight in a register ring that
// rolls across tile boundaries (the refill for step s+U already belongs to the
// wave's next tile when s+U runs past this one), so a wave's load queue never
// drains between tiles.  Per step:
//   * chunk sum of the lane's 8 words (field word zeroed for kFill);
//   * 64-lane inclusive DPP scan + running carry (readlane 63) -> P at every
//     chunk start;
//   * boundaries are found arithmetically: each lane tracks its chunk's
//     position m inside an image (m += 1024 mod S per step), so a boundary
//     lies in the chunk iff m == 0 or m > S - 16; the lane holding it forms
//     P(boundary) = carry + exclusive scan + its words before the boundary;
//   * every boundary lane emits the image that ends there, using the previous
//     boundary's P fetched from the nearest lower boundary lane of the same
//     step (ds_bpermute) or, for the first one, from the step before (SGPR).
// Results are stored as u16 (kFill: also into bytes 28-29, tcp-header.h:177;
// kVerify: u8 checksum == 0).
#include "tcpck_device.h"

namespace tcpck {

namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
using dev::u32x4;

struct TileGeom {
  uint64_t k0;          // first image
  uint64_t a0;          // arena offset of the line-aligned run start (wrapping)
  uint32_t n;           // images
  uint32_t lead;        // bytes before the first image in the first step
  uint32_t span;        // bytes from a0 to the run end
  uint32_t nsteps;      // 1 KiB steps
  uint32_t last_chunk;  // index of the run's last 16-B chunk
};

__device__ __forceinline__ TileGeom tile_geom(const FixedStreamArgs &a, uint64_t t) {
  TileGeom g;
  g.k0 = t * a.tile;
  const uint64_t left = a.count - g.k0;
  g.n = static_cast<uint32_t>(left < a.tile ? left : a.tile);
  const uint64_t s0 = g.k0 * a.stride;
  g.a0 = dev::align128_rel(a.arena, s0);
  g.lead = static_cast<uint32_t>(s0 - g.a0);
  g.span = g.lead + g.n * static_cast<uint32_t>(a.stride);
  g.nsteps = (g.span + 1023) >> 10;
  g.last_chunk = (g.span - 1) >> 4;
  return g;
}

// Sum of the chunk's words before byte r (r even, 0..14), given the per-dword
// sums c0..c2 (w + (w >> 16), low 16 bits meaningful) and the raw dwords.
__device__ __forceinline__ uint32_t head_sum(uint32_t r, u32x4 w, uint32_t c0, uint32_t c1, uint32_t c2) {
  uint32_t h = (r >= 4 ? c0 : 0u) + (r >= 8 ? c1 : 0u) + (r >= 12 ? c2 : 0u);
  const uint32_t q = r >> 2;
  const uint32_t d = q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w));
  return h + ((r & 2u) ? (d & 0xFFFFu) : 0u);
}

template <int U, int OP>
__global__ void __launch_bounds__(kBlock) fstream_kernel(FixedStreamArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t W = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  uint64_t t = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  const uint64_t ntiles = (a.count + a.tile - 1) / a.tile;
  if (t >= ntiles) return;
  const uint32_t S = static_cast<uint32_t>(a.stride);
  const uint32_t D = 1024u % S;  // chunk position advance per step, mod S
  const uint32_t Q = 1024u / S;  // whole images passed per step

  TileGeom cur = tile_geom(a, t);
  bool has_next = t + W < ntiles;
  TileGeom nxt = has_next ? tile_geom(a, t + W) : cur;

  // address of 16-B chunk `lane` of step st of the current run, or -- past the
  // current run -- of the next tile's run (clamped: always a legal address)
  auto chunk_ptr = [&](uint32_t st) -> const uint8_t * {
    if (st < cur.nsteps) {
      const uint32_t ci = min((st << 6) + lane, cur.last_chunk);
      return a.arena + cur.a0 + 16 * static_cast<uint64_t>(ci);
    }
    // value selects, never a reference to one of two structs: that would put
    // both in scratch, and every scratch load waits behind the whole ring
    const uint64_t ga0 = has_next ? nxt.a0 : cur.a0;
    const uint32_t glast = has_next ? nxt.last_chunk : cur.last_chunk;
    const uint32_t sn = has_next ? st - cur.nsteps : 0;
    const uint32_t ci = min((sn << 6) + lane, glast);
    return a.arena + ga0 + 16 * static_cast<uint64_t>(ci);
  };

  // per-lane position of its chunk inside an image: x = q*S + m, 0 <= m < S
  // (x relative to the run's first image; negative for chunks before it)
  uint32_t m;
  int32_t q;
  auto lane_init = [&]() {
    const int32_t x = static_cast<int32_t>(lane << 4) - static_cast<int32_t>(cur.lead);
    if (x >= 0) {
      q = x / static_cast<int32_t>(S);
      m = static_cast<uint32_t>(x) - static_cast<uint32_t>(q) * S;
    } else {  // x in [-127, 0): before the run, possibly several short images back
      q = -static_cast<int32_t>((static_cast<uint32_t>(-x) + S - 1) / S);
      m = static_cast<uint32_t>(x - q * static_cast<int32_t>(S));
    }
  };
  lane_init();

  uint32_t carry = 0;   // P at the current step's start (mod 2^32; low 16 bits meaningful)
  uint32_t p_last = 0;  // P of the latest boundary already passed (run start = 0)
  uint32_t st = 0;      // step within the current run

  u32x4 ring[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ring[u] = dev::load16_nt(chunk_ptr(static_cast<uint32_t>(u)));

  for (;;) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 w = ring[u];
      const uint32_t sb = st << 10;
      if (sb == 0 || sb + 1024 > cur.span) {  // run edge (wave-uniform): mask words outside [lead, span)
        const int32_t crel = static_cast<int32_t>(sb + (lane << 4));
        const int32_t lo = min(max(static_cast<int32_t>(cur.lead) - crel, 0), 16);
        const int32_t hi = min(max(static_cast<int32_t>(cur.span) - crel, 0), 16);
        w = dev::apply_mask(w, dev::word_mask(lo, hi));
      }
      if (OP == kFill && m >= 14 && m <= 28) {  // this chunk holds an image's checksum field: count it as 0
        const uint32_t fw = (28 - m) >> 1;
        w = dev::apply_mask(w, 0xFFu & ~(1u << fw));
      }
      const uint32_t c0 = w.x + (w.x >> 16);
      const uint32_t c1 = w.y + (w.y >> 16);
      const uint32_t c2 = w.z + (w.z >> 16);
      const uint32_t c3 = w.w + (w.w >> 16);
      const uint32_t tot = c0 + c1 + c2 + c3;
      const uint32_t incl = dev::wave_inclusive_scan(tot);

      // boundary in this chunk: at r = 0 (m == 0) or r = S - m (m > S - 16);
      // j = image index (relative to the run) that starts there
      const bool at_start = m == 0;
      const uint32_t r = at_start ? 0u : S - m;
      const int32_t j = q + (at_start ? 0 : 1);
      const bool has = (at_start || m > S - 16) && j >= 1 && j < static_cast<int32_t>(cur.n);
      const uint64_t bal = __ballot(has);
      if (bal) {  // wave-uniform
        const uint32_t P = carry + (incl - tot) + head_sum(r, w, c0, c1, c2);
        // previous boundary: nearest lower boundary lane of this step, else p_last
        const uint64_t below = bal & ((uint64_t{1} << lane) - 1u);
        const int32_t src = below ? 63 - __clzll(below) : 0;
        const uint32_t p_prev_lane = static_cast<uint32_t>(
            __builtin_amdgcn_ds_bpermute(src << 2, static_cast<int>(P)));
        if (has) {
          const uint32_t sum = P - (below ? p_prev_lane : p_last);
          const uint64_t k = cur.k0 + static_cast<uint64_t>(j - 1);  // the image that ends here
          const uint16_t c = static_cast<uint16_t>(~sum);             // tcp-header.h:262
          if constexpr (OP == kVerify) {
            static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
          } else {
            if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
            if (OP == kFill && S >= 30) *reinterpret_cast<uint16_t *>(a.arena + k * S + 28) = c;
          }
        }
        p_last = dev::read_lane(P, 63 - __clzll(bal));
      }
      carry += dev::read_lane(incl, 63);
      // Refill this slot with step st + U only now that its data is dead, so the
      // load can land in the same registers (an earlier refill makes hipcc
      // rotate the slot through other registers and drain the queue to do it).
      ring[u] = dev::load16_nt(chunk_ptr(st + U));
      // advance the lane's chunk position by one step (1024 B)
      m += D;
      q += static_cast<int32_t>(Q);
      if (m >= S) {
        m -= S;
        q += 1;
      }
      ++st;
      if (st == cur.nsteps) {  // wave-uniform: run finished, the last image ends at the run end
        if (lane == 0) {
          const uint64_t k = cur.k0 + cur.n - 1;
          const uint16_t c = static_cast<uint16_t>(~(carry - p_last));
          if constexpr (OP == kVerify) {
            static_cast<uint8_t *>(a.out)[k] = (c == 0) ? 1 : 0;
          } else {
            if (a.out) static_cast<uint16_t *>(a.out)[k] = c;
            if (OP == kFill && S >= 30) *reinterpret_cast<uint16_t *>(a.arena + k * S + 28) = c;
          }
        }
        if (!has_next) return;
        t += W;
        cur = nxt;
        has_next = t + W < ntiles;
        if (has_next) nxt = tile_geom(a, t + W);
        lane_init();
        carry = 0;
        p_last = 0;
        st = 0;
      }
    }
  }
}

template <int U, int OP>
hipError_t launch_one(const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  static const uint32_t per_cu = dev::resident_blocks_per_cu(fstream_kernel<U, OP>);
  const uint64_t ntiles = (a.count + a.tile - 1) / a.tile;
  uint64_t blocks = static_cast<uint64_t>(per_cu) * num_cus;
  const uint64_t need = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > need) blocks = need;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((fstream_kernel<U, OP>), dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int U>
hipError_t dispatch(int op, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t s) {
  switch (op) {
    case kChecksum: return launch_one<U, kChecksum>(a, num_cus, s);
    case kFill: return launch_one<U, kFill>(a, num_cus, s);
    case kVerify: return launch_one<U, kVerify>(a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

uint32_t fstream_min_tile(uint32_t stride, int variant) {
  const uint32_t U = variant == 1 ? 2u : 4u;
  return (U * 1024u + stride - 1) / stride;  // every non-final tile spans >= U steps
}

uint32_t fstream_tile_for_len(uint32_t stride, int variant) {
  uint32_t t = (24u << 10) / stride;  // ~24 KiB per tile
  const uint32_t lo = fstream_min_tile(stride, variant);
  if (t < lo) t = lo;
  return t ? t : 1;
}

hipError_t launch_fstream(int op, int variant, const FixedStreamArgs &a, uint32_t num_cus, hipStream_t stream) {
  if (a.stride < 16 || a.stride > (1u << 20) || a.tile < fstream_min_tile(static_cast<uint32_t>(a.stride), variant) ||
      static_cast<uint64_t>(a.tile) * a.stride > (1u << 30))
    return hipErrorInvalidValue;
  switch (variant) {
    case 0: return dispatch<4>(op, a, num_cus, stream);
    case 1: return dispatch<2>(op, a, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tcpck
