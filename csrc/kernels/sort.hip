// sort.hip — stable LSD radix sort of (key, value) pairs on gfx950, written
// for the engine's two sorts: the rank order of linear-ranking selection
// (every generation, S keys) and the sorted top-k (k keys).  No library sort.
//
// Reduce-then-scan, up to 8-bit digits (the passes split the key bits evenly:
// OneMax-1024's 11-bit keys sort in 6 + 5 bits), three launches per pass:
//   COUNT    a workgroup per TILE of 4096 keys counts its digits into
//            counts[digit * tiles + tile] (digit-major);
//   SCAN     exclusive scan of counts: each entry becomes the global output
//            base of (digit, tile) — one launch of 4096-entry chunks whose
//            totals (up to 256) the scatter folds itself, else two levels;
//   SCATTER  the tile again, every wave its own 1024 consecutive keys in 16
//            rounds of 64: the lanes that share a digit find each other with
//            one ballot per digit bit (a match-any), rank among themselves by
//            popcount below the lane, and bump the wave's LDS digit counter
//            once per group.  Stable by construction (rounds in key order,
//            lanes in key order, waves in key order), no atomics, no look-back
//            chain: every workgroup of a pass is independent.  The ranked tile
//            is staged in LDS in digit order and written out from there, so a
//            store instruction covers consecutive addresses of one digit run.
// The previous onesweep design (decoupled look-back over 512 tiles of 2048
// keys, 4-bit digits) serialised on the look-back: 28 us per pass at 1M keys
// (profiles/rank_roulette_r03.md).
//
// Reference: the reference has no selection but binary tournament
// (src/pga.cu:278-292); linear ranking is the "placeholder" selection enum
// (include/pga.h:36-42) made real.
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"

// dynamic LDS of radix_scatter_wide_kernel (outside the anonymous namespace:
// an extern __shared__ array has no definition to give it internal linkage)
extern __shared__ __align__(16) uint8_t pga_sort_dyn_lds[];

namespace pga {
namespace {

using namespace dev;

constexpr uint32_t kMaxDigitBits = 8;
constexpr uint32_t kMaxDigits = 1u << kMaxDigitBits;
// single-pass mode for small key ranges (u16 keys of integer objectives,
// key_range <= 2048): the digit is the whole key, D = key_range digits
constexpr uint32_t kWideBits = 11;
constexpr uint32_t kWideDigits = 1u << kWideBits;
constexpr uint32_t kWaveKeys = 1024;                   // per wave: 16 rounds of 64
constexpr uint32_t kRounds = kWaveKeys / 64;
constexpr uint32_t kTile = kWaveKeys * (kBlock / 64);  // 4096 keys per workgroup
static_assert(kTile == kRankTile, "the fused rank counts (binary_gen_tp) assume the sort's tile");
// one scan workgroup: 4096 entries.  The rank order of OneMax-1024 at 1M
// keys scans 1025 x 256 counts: 65 workgroups of 256 threads take 4.9 us
// where 17 of 1024 threads took 5.5 (profiles/rank_fused_r06.md)
constexpr uint32_t kScanBlock = 256, kScanPer = 16;
constexpr uint32_t kScanChunk = kScanBlock * kScanPer;
// the scatters fold up to this many chunk totals themselves (fold_chunk_sums)
constexpr uint32_t kScanFold = 256;

// cpre[c] = exclusive prefix of the chunk totals csums[0, nchunks), nchunks
// <= kScanFold: one wave, 4 totals per lane
__device__ __forceinline__ void fold_chunk_sums(const uint32_t* __restrict__ csums, uint32_t nchunks, uint32_t* cpre,
                                                uint32_t lane) {
  uint32_t c[kScanFold / 64], s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanFold / 64; ++j) {
    const uint32_t i = lane * (kScanFold / 64) + j;
    c[j] = i < nchunks ? csums[i] : 0u;
    s += c[j];
  }
  uint32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  uint32_t run = incl - s;
#pragma unroll
  for (uint32_t j = 0; j < kScanFold / 64; ++j) {
    cpre[lane * (kScanFold / 64) + j] = run;
    run += c[j];
  }
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
inline uint64_t tiles_of(uint64_t n) { return (n + kTile - 1) / kTile; }

// workspace: [counts kMaxDigits x tiles][chunk sums][chunk sums of sums][keys W][vals W]
struct RadixWs {
  uint32_t* counts;
  uint32_t* sums;
  uint32_t* sums2;
  uint32_t* k;
  uint32_t* v;
};

RadixWs radix_ws(void* ws, uint64_t n) {
  const uint64_t entries = (uint64_t)kWideDigits * tiles_of(n);
  const uint64_t chunks = (entries + kScanChunk - 1) / kScanChunk;
  char* p = (char*)ws;
  RadixWs w;
  w.counts = (uint32_t*)p;
  p += al(4ull * entries);
  w.sums = (uint32_t*)p;
  p += al(4ull * chunks);
  w.sums2 = (uint32_t*)p;
  p += al(4ull * ((chunks + kScanChunk - 1) / kScanChunk));
  w.k = (uint32_t*)p;
  p += al(4ull * n);
  w.v = (uint32_t*)p;
  return w;
}

// A pass's key source: the caller's keys on pass 0 (u32, u16 zero-extended, or
// f32 scores through score_key; optionally inverted for descending order),
// the staged u32 keys after it.
struct KeySrc {
  const uint32_t* k32;
  const uint16_t* k16;
  const float* f32;
  const uint32_t* vals;  // pass-0 values (nullptr: the key's index)
  bool invert;
};

// the source kind is a template parameter: a runtime choice per load would
// put a branch (and a wait for the load) between the 32 loads of a lane
enum { SRC_U32 = 0, SRC_U16 = 1, SRC_F32 = 2 };
template <int SRC>
__device__ __forceinline__ uint32_t load_key(const KeySrc& s, uint64_t i) {
  uint32_t key = SRC == SRC_U32 ? s.k32[i] : (SRC == SRC_U16 ? (uint32_t)s.k16[i] : score_key(s.f32[i]));
  return s.invert ? ~key : key;
}

// the lanes of this wave whose (digit < D) equals mine; lanes without a key
// (digit == D, past the end) match nobody
__device__ __forceinline__ uint64_t match_digit(uint32_t dig, bool ok, uint32_t bits) {
  uint64_t m = __ballot(ok);
  for (uint32_t b = 0; b < bits; ++b) {  // wave-uniform trip count
    const bool set = (dig >> b) & 1u;
    const uint64_t bb = __ballot(set);
    m &= set ? bb : ~bb;
  }
  return ok ? m : 0ull;
}

// Per-tile digit counts (order-independent): one LDS atomic per group of
// lanes sharing a digit (a skewed key distribution would otherwise serialise
// up to 64 same-address atomics per instruction).
template <int SRC, uint32_t MAXD>
__global__ __launch_bounds__(kBlock) void radix_count_kernel(KeySrc src, uint64_t n, uint32_t shift, uint32_t bits,
                                                             uint32_t D, uint64_t tiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[MAXD];
  const uint32_t mask = (1u << bits) - 1u;
  for (uint32_t d = threadIdx.x; d < D; d += kBlock) h[d] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  const uint64_t below = (1ull << lane_id()) - 1ull;
  uint32_t dig[kTile / kBlock];
#pragma unroll
  for (uint32_t i = 0; i < kTile / kBlock; ++i) {  // all loads first
    const uint64_t e = t0 + (uint64_t)i * kBlock + threadIdx.x;
    const uint32_t d = min((load_key<SRC>(src, e < n ? e : n - 1) >> shift) & mask, D - 1);  // unconditional load
    dig[i] = e < n ? d : D;
  }
  if (MAXD > kMaxDigits) {
    // the whole key as digit: spread over many bins, plain LDS atomics beat
    // an 11-ballot match per key
#pragma unroll
    for (uint32_t i = 0; i < kTile / kBlock; ++i)
      if (dig[i] < D) atomicAdd(&h[dig[i]], 1u);
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kTile / kBlock; ++i) {
      const bool ok = dig[i] < D;
      const uint64_t peers = match_digit(dig[i], ok, bits);
      if (ok && (peers & below) == 0ull) atomicAdd(&h[dig[i]], (uint32_t)__popcll(peers));
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < D; d += kBlock) counts[(uint64_t)d * tiles + blockIdx.x] = h[d];
}

// In-place exclusive scan of chunks of kScanChunk entries (one workgroup per
// chunk); the chunk totals go to sums (when non-null).
__global__ __launch_bounds__(kScanBlock) void scan_chunk_kernel(uint32_t* __restrict__ x, uint64_t m,
                                                                uint32_t* __restrict__ sums) {
  __shared__ uint32_t wsum[kScanBlock / 64];
  const uint32_t t = threadIdx.x, lane = lane_id(), wid = t >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)t * kScanPer;
  uint32_t v[kScanPer], s = 0;
  if (base + kScanPer <= m && (m & 3u) == 0u) {  // whole 16-byte vectors (the usual case)
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j += 4) {
      const uint4 y = *(const uint4*)(x + base + j);
      v[j] = y.x;
      v[j + 1] = y.y;
      v[j + 2] = y.z;
      v[j + 3] = y.w;
    }
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
      const uint32_t y = x[base + j < m ? base + j : m - 1];  // unconditional load
      v[j] = base + j < m ? y : 0u;
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) s += v[j];
  uint32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t off = incl - s, tot = 0;
  for (uint32_t w = 0; w < kScanBlock / 64; ++w) {
    off += w < wid ? wsum[w] : 0u;
    tot += wsum[w];
  }
  if (base + kScanPer <= m && (m & 3u) == 0u) {
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j += 4) {
      uint4 y;
      y.x = off;
      y.y = y.x + v[j];
      y.z = y.y + v[j + 1];
      y.w = y.z + v[j + 2];
      off = y.w + v[j + 3];
      *(uint4*)(x + base + j) = y;
    }
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
      if (base + j < m) x[base + j] = off;
      off += v[j];
    }
  }
  if (sums && t == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_add_kernel(uint32_t* __restrict__ x, uint64_t m,
                                                          const uint32_t* __restrict__ sums) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < m) x[i] += sums[i / kScanChunk];
}

// Scatter one tile stably by digit.  Thread layout: wave w owns keys
// [t0 + w * 1024, t0 + (w + 1) * 1024), round r lane l is key w * 1024 + r * 64 + l.
template <int SRC, int VAL, uint32_t MAXD>  // VAL: 0 = the key's index, 1 = src.vals, 2 = vin
__global__ __launch_bounds__(kBlock) void radix_scatter_kernel(KeySrc src, const uint32_t* __restrict__ vin, uint64_t n,
                                                               uint32_t shift, uint32_t bits, uint32_t D, uint64_t tiles,
                                                               const uint32_t* __restrict__ base,
                                                               const uint32_t* __restrict__ csums, uint32_t nchunks,
                                                               uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint32_t cnt[kBlock / 64][MAXD];  // per wave: running digit counts, then output bases
  const uint32_t mask = (1u << bits) - 1u;
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  for (uint32_t d = lane; d < D; d += 64) cnt[wid][d] = 0;
  const uint64_t w0 = (uint64_t)blockIdx.x * kTile + (uint64_t)wid * kWaveKeys;
  uint32_t key[kRounds], val[kRounds];
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) {  // every load in flight before the ranking
    const uint64_t e = w0 + r * 64u + lane;
    const uint64_t ec = e < n ? e : n - 1;  // unconditional loads (a guarded load waits before the next)
    key[r] = load_key<SRC>(src, ec);
    val[r] = VAL == 2 ? vin[ec] : (VAL == 1 ? src.vals[ec] : (uint32_t)e);
  }
  // exclusive prefix of the scan-chunk totals (nchunks <= kScanFold):
  // one wave's scan into LDS, read per digit below
  __shared__ uint32_t cpre[kScanFold];
  if (csums && wid == 0) fold_chunk_sums(csums, nchunks, cpre, lane);
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t pos[kRounds];
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) {
    const bool ok = w0 + r * 64u + lane < n;
    const uint32_t dig = ok ? min((key[r] >> shift) & mask, D - 1) : D;
    const uint64_t peers = match_digit(dig, ok, bits);
    const uint32_t rk = (uint32_t)__popcll(peers & below);
    // every lane of a group reads the counter, then the group's first lane bumps
    // it: a wave's LDS operations retire in order
    const uint32_t c = ok ? cnt[wid][dig] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (ok && rk == 0u) cnt[wid][dig] = c + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    pos[r] = ok ? c + rk : 0xFFFFFFFFu;
  }
  __syncthreads();
  // Stage the tile in LDS in digit order, then write it out in that order:
  // consecutive lanes store consecutive addresses of a digit's output run
  // (scattering straight from the ranking spreads one store instruction
  // over up to 64 runs).
  __shared__ uint32_t sk[kTile], sv[kTile];
  __shared__ uint32_t gofs[MAXD], wsum[kBlock / 64];
  constexpr uint32_t P = MAXD / kBlock;  // digits per thread: [t P, t P + P)
  const uint32_t t = threadIdx.x;
  uint32_t tcs[P], tsum = 0;  // keys of each digit in the tile; cnt[w][d] becomes the waves-before offset
#pragma unroll
  for (uint32_t j = 0; j < P; ++j) {
    const uint32_t d = t * P + j;
    uint32_t tc = 0;
    if (d < D) {
#pragma unroll
      for (uint32_t w = 0; w < kBlock / 64; ++w) {
        const uint32_t c = cnt[w][d];
        cnt[w][d] = tc;
        tc += c;
      }
    }
    tcs[j] = tc;
    tsum += tc;
  }
  uint32_t incl = tsum;  // block exclusive scan over the threads' digit ranges -> local digit starts
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t ls = incl - tsum;
  for (uint32_t w = 0; w < wid; ++w) ls += wsum[w];
#pragma unroll
  for (uint32_t j = 0; j < P; ++j) {
    const uint32_t d = t * P + j;
    if (d < D) {
#pragma unroll
      for (uint32_t w = 0; w < kBlock / 64; ++w) cnt[w][d] += ls;  // local start of (wave w, digit d)
      // base: exclusive scan WITHIN its scan chunk; cpre: the prefix of the
      // chunk totals (scan_chunks)
      const uint64_t e = (uint64_t)d * tiles + blockIdx.x;
      const uint32_t pre = csums ? cpre[e / kScanChunk] : 0u;
      gofs[d] = base[e] + pre - ls;  // output index = gofs[d] + local index
    }
    ls += tcs[j];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kRounds; ++r) {
    if (pos[r] != 0xFFFFFFFFu) {
      const uint32_t lp = cnt[wid][min((key[r] >> shift) & mask, D - 1)] + pos[r];
      sk[lp] = key[r];
      sv[lp] = val[r];
    }
  }
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  const uint32_t nt = (uint32_t)(n - t0 < kTile ? n - t0 : kTile);
  for (uint32_t i = t; i < nt; i += kBlock) {
    const uint32_t k = sk[i];
    const uint32_t o = gofs[min((k >> shift) & mask, D - 1)] + i;
    if (kout) kout[o] = k;
    vout[o] = sv[i];
  }
}

// Single-pass scatter of u16 keys (digit = the whole key, D <= 2048; the
// value is the key's index): the rank order of an integer objective.  The
// same stable ranking as radix_scatter_kernel with 16 waves per tile instead
// of 4 (256 keys each, 4 rounds): one workgroup per CU at the headline, so the
// 4-wave version left each SIMD a single wave to hide the ranking's LDS
// round trips and the ballots behind.  Per-wave digit counters are u16 (a
// tile has 4096 keys) in dynamic LDS sized by D, the tile is staged as u16
// keys and u16 tile-local indices.
constexpr uint32_t kWideWaves = 16;
constexpr uint32_t kWideThreads = kWideWaves * 64;
constexpr uint32_t kWideRounds = kTile / kWideThreads;  // 4 rounds of 64 keys per wave
static_assert(kWideDigits % kWideThreads == 0, "digits per thread");

inline uint32_t wide_scatter_lds(uint32_t D) {
  const uint32_t Dp = (D + 1u) & ~1u;  // u16 rows keep 4-byte alignment
  return kWideWaves * Dp * 2u + kTile * 2u * 2u + Dp * 4u;
}

__global__ __launch_bounds__(kWideThreads) void radix_scatter_wide_kernel(
    const uint16_t* __restrict__ keys, uint64_t n, uint32_t bits, uint32_t D, uint64_t tiles,
    const uint32_t* __restrict__ base, const uint32_t* __restrict__ csums, uint32_t nchunks,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  const uint32_t Dp = (D + 1u) & ~1u;
  uint16_t* cnt = (uint16_t*)pga_sort_dyn_lds;  // [kWideWaves][Dp]: running counts, then local starts
  uint16_t* sk = cnt + kWideWaves * Dp;         // the tile in digit order: keys ...
  uint16_t* sv = sk + kTile;                    // ... and their tile-local indices
  uint32_t* gofs = (uint32_t*)(sv + kTile);     // [Dp]: output index = gofs[d] + staged position
  __shared__ uint32_t wsum[kWideWaves];
  __shared__ uint32_t cpre[kScanFold];
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6, t = threadIdx.x;
  uint16_t* mine = cnt + wid * Dp;
  for (uint32_t d = lane; d < D; d += 64) mine[d] = 0;  // this wave's row (its LDS ops retire in order)
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  const uint32_t l0 = wid * (kTile / kWideWaves);  // this wave's first tile-local key
  uint32_t key[kWideRounds];
#pragma unroll
  for (uint32_t r = 0; r < kWideRounds; ++r) {  // every load in flight before the ranking
    const uint64_t e = t0 + l0 + r * 64u + lane;
    key[r] = keys[e < n ? e : n - 1];  // unconditional load
  }
  if (csums && wid == 0) fold_chunk_sums(csums, nchunks, cpre, lane);  // (nchunks <= kScanFold)
  // this thread's digits' scanned counts, loaded now: their latency hides
  // behind the ranking instead of following it
  constexpr uint32_t P = kWideDigits / kWideThreads;  // digits per thread: [t P, t P + P)
  uint32_t bval[P];
#pragma unroll
  for (uint32_t j = 0; j < P; ++j) {
    const uint32_t d = t * P + j;
    bval[j] = base[(uint64_t)(d < D ? d : D - 1) * tiles + blockIdx.x];  // unconditional load
  }
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t pos[kWideRounds];
#pragma unroll
  for (uint32_t r = 0; r < kWideRounds; ++r) {
    const bool ok = t0 + l0 + r * 64u + lane < n;
    const uint32_t dig = ok ? min(key[r], D - 1) : D;
    key[r] = dig;
    const uint64_t peers = match_digit(dig, ok, bits);
    const uint32_t rk = (uint32_t)__popcll(peers & below);
    const uint32_t c = ok ? mine[dig] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (ok && rk == 0u) mine[dig] = (uint16_t)(c + (uint32_t)__popcll(peers));
    __builtin_amdgcn_wave_barrier();
    pos[r] = ok ? c + rk : 0xFFFFFFFFu;
  }
  __syncthreads();
  // per digit: the waves' counts become waves-before offsets, then local starts
  uint32_t tcs[P], tsum = 0;
#pragma unroll
  for (uint32_t j = 0; j < P; ++j) {
    const uint32_t d = t * P + j;
    uint32_t tc = 0;
    if (d < D) {
#pragma unroll
      for (uint32_t w = 0; w < kWideWaves; ++w) {
        const uint32_t c = cnt[w * Dp + d];
        cnt[w * Dp + d] = (uint16_t)tc;
        tc += c;
      }
    }
    tcs[j] = tc;
    tsum += tc;
  }
  uint32_t incl = tsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t ls = incl - tsum;
  for (uint32_t w = 0; w < wid; ++w) ls += wsum[w];
#pragma unroll
  for (uint32_t j = 0; j < P; ++j) {
    const uint32_t d = t * P + j;
    if (d < D) {
#pragma unroll
      for (uint32_t w = 0; w < kWideWaves; ++w) cnt[w * Dp + d] = (uint16_t)(cnt[w * Dp + d] + ls);
      const uint64_t e = (uint64_t)d * tiles + blockIdx.x;
      const uint32_t pre = csums ? cpre[e / kScanChunk] : 0u;
      gofs[d] = bval[j] + pre - ls;
    }
    ls += tcs[j];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kWideRounds; ++r) {
    if (pos[r] != 0xFFFFFFFFu) {
      const uint32_t lp = mine[key[r]] + pos[r];
      sk[lp] = (uint16_t)key[r];
      sv[lp] = (uint16_t)(l0 + r * 64u + lane);
    }
  }
  __syncthreads();
  const uint32_t nt = (uint32_t)(n - t0 < kTile ? n - t0 : kTile);
  for (uint32_t i = t; i < nt; i += kWideThreads) {
    const uint32_t k = sk[i];
    const uint32_t o = gofs[k] + i;
    if (kout) kout[o] = k;
    vout[o] = (uint32_t)t0 + sv[i];
  }
}

// The scatter's bases with at most kScanFold scan chunks: ONE launch scans
// each chunk in place and stores the chunk totals; the scatter adds the
// prefix of the totals itself (one wave scan into LDS) instead of two
// more launches (scan of the totals, add back: ~4.8 + 5.0 us for the rank
// order of 1M u16 keys, profiles/rank_kernel_stats_r03.csv).  Returns the
// chunk count (0: x is fully scanned, nothing to fold).
uint32_t scan_chunks(uint32_t* x, uint64_t m, const RadixWs& w, hipStream_t s);

// exclusive scan of m entries in place (m <= kScanChunk^3)
void scan_exclusive(uint32_t* x, uint64_t m, const RadixWs& w, hipStream_t s) {
  const uint64_t chunks = (m + kScanChunk - 1) / kScanChunk;
  if (chunks <= 1) {
    hipLaunchKernelGGL(scan_chunk_kernel, 1, kScanBlock, 0, s, x, m, (uint32_t*)nullptr);
    return;
  }
  hipLaunchKernelGGL(scan_chunk_kernel, (uint32_t)chunks, kScanBlock, 0, s, x, m, w.sums);
  const uint64_t chunks2 = (chunks + kScanChunk - 1) / kScanChunk;
  if (chunks2 > kScanChunk) throw std::invalid_argument("radix sort: too many keys");
  if (chunks2 <= 1) {
    hipLaunchKernelGGL(scan_chunk_kernel, 1, kScanBlock, 0, s, w.sums, chunks, (uint32_t*)nullptr);
  } else {
    hipLaunchKernelGGL(scan_chunk_kernel, (uint32_t)chunks2, kScanBlock, 0, s, w.sums, chunks, w.sums2);
    hipLaunchKernelGGL(scan_chunk_kernel, 1, kScanBlock, 0, s, w.sums2, chunks2, (uint32_t*)nullptr);
    hipLaunchKernelGGL(scan_add_kernel, (uint32_t)((chunks + kBlock - 1) / kBlock), kBlock, 0, s, w.sums, chunks,
                       w.sums2);
  }
  hipLaunchKernelGGL(scan_add_kernel, (uint32_t)((m + kBlock - 1) / kBlock), kBlock, 0, s, x, m, w.sums);
}

uint32_t scan_chunks(uint32_t* x, uint64_t m, const RadixWs& w, hipStream_t s) {
  const uint64_t chunks = (m + kScanChunk - 1) / kScanChunk;
  if (chunks <= 1 || chunks > kScanFold) {
    scan_exclusive(x, m, w, s);
    return 0;
  }
  hipLaunchKernelGGL(scan_chunk_kernel, (uint32_t)chunks, kScanBlock, 0, s, x, m, w.sums);
  return (uint32_t)chunks;
}

// one sort: per pass count -> scan -> scatter.  The passes ping-pong between
// the workspace staging (W) and the output (O); pass i writes O when an even
// number of passes follows it, so the last one lands in O.
// Single-pass mode: the keys are below a known range of at most 2^11 values
// and the digit is the whole key
bool wide_mode(uint32_t bits, uint32_t key_range) {
  return key_range >= 2 && key_range <= kWideDigits && bits > kMaxDigitBits && bits <= kWideBits &&
         (1u << bits) >= key_range;
}

// counts_ready (single-pass mode only): w.counts already holds the pass's
// tile counts (a fused producer wrote them), the count launch is skipped.
// want_keys = false: the last pass stores only the values (kout is still the
// ping-pong buffer of the passes before it).
void radix_run(const KeySrc& src0, uint64_t n, uint32_t bits, uint32_t* kout, uint32_t* vout, void* ws, hipStream_t s,
               uint32_t key_range = 0, bool counts_ready = false, bool want_keys = true) {
  if (n == 0) return;
  if (n > 0xFFFFFFFFull) throw std::invalid_argument("radix sort: more than 2^32 - 1 keys");
  bits = bits < 1 ? 1 : (bits > 32 ? 32 : bits);
  const bool wide = wide_mode(bits, key_range);  // ONE pass whose digit is the key
  const uint32_t passes = wide ? 1u : (bits + kMaxDigitBits - 1) / kMaxDigitBits;
  RadixWs w = radix_ws(ws, n);
  const uint64_t tiles = tiles_of(n);
  if (tiles > 0x7FFFFFFFull) throw std::invalid_argument("radix sort: too many tiles");
  uint32_t shift = 0;
  const uint32_t *ck = nullptr, *cv = nullptr;
  for (uint32_t p = 0; p < passes; ++p) {
    // split the bits evenly: the first (bits % passes) passes take one more
    const uint32_t pb = bits / passes + (p < bits % passes ? 1u : 0u);
    const bool to_out = (passes - 1 - p) % 2 == 0;
    uint32_t* dk = to_out ? kout : w.k;
    if (p + 1 == passes && !want_keys) dk = nullptr;
    uint32_t* dv = to_out ? vout : w.v;
    KeySrc src = p == 0 ? src0 : KeySrc{ck, nullptr, nullptr, nullptr, false};
    const int kind = p > 0 ? SRC_U32 : (src.k32 ? SRC_U32 : (src.k16 ? SRC_U16 : SRC_F32));
    const int vk = p > 0 ? 2 : (src.vals ? 1 : 0);
    const uint32_t D = wide ? key_range : (1u << pb);
    const dim3 g((uint32_t)tiles);
#define PGA_COUNT(K, MD) hipLaunchKernelGGL((radix_count_kernel<K, MD>), g, kBlock, 0, s, src, n, shift, pb, D, tiles, w.counts)
#define PGA_SCATTER(K, V, MD) hipLaunchKernelGGL((radix_scatter_kernel<K, V, MD>), g, kBlock, 0, s, src, cv, n, shift, pb, D, tiles, w.counts, nch ? w.sums : nullptr, nch, dk, dv)
    if (wide) {  // one pass over u16 keys (rank order of an integer objective)
      if (kind != SRC_U16 || vk != 0) throw std::logic_error("radix sort: single-pass mode is for u16 keys");
      if (!counts_ready) PGA_COUNT(SRC_U16, kWideDigits);
      const uint32_t nch = scan_chunks(w.counts, (uint64_t)D * tiles, w, s);
      const uint32_t lds = wide_scatter_lds(D);
      if (lds > 64u * 1024u) (void)allow_dynamic_lds((const void*)radix_scatter_wide_kernel);
      hipLaunchKernelGGL(radix_scatter_wide_kernel, g, kWideThreads, lds, s, src.k16, n, pb, D, tiles, w.counts,
                         nch ? w.sums : nullptr, nch, dk, dv);
    } else {
      if (kind == SRC_U32) PGA_COUNT(SRC_U32, kMaxDigits);
      if (kind == SRC_U16) PGA_COUNT(SRC_U16, kMaxDigits);
      if (kind == SRC_F32) PGA_COUNT(SRC_F32, kMaxDigits);
      const uint32_t nch = scan_chunks(w.counts, (uint64_t)D * tiles, w, s);
      if (vk == 2) PGA_SCATTER(SRC_U32, 2, kMaxDigits);
      else if (kind == SRC_U32) { if (vk) PGA_SCATTER(SRC_U32, 1, kMaxDigits); else PGA_SCATTER(SRC_U32, 0, kMaxDigits); }
      else if (kind == SRC_U16) { if (vk) PGA_SCATTER(SRC_U16, 1, kMaxDigits); else PGA_SCATTER(SRC_U16, 0, kMaxDigits); }
      else { if (vk) PGA_SCATTER(SRC_F32, 1, kMaxDigits); else PGA_SCATTER(SRC_F32, 0, kMaxDigits); }
    }
#undef PGA_COUNT
#undef PGA_SCATTER
    ck = dk;
    cv = dv;
    shift += pb;
  }
  PGA_HIP_CHECK(hipGetLastError());
}

}  // namespace

size_t radix_sort_workspace_bytes(uint64_t n) {
  const uint64_t entries = (uint64_t)kWideDigits * tiles_of(n);
  const uint64_t chunks = (entries + kScanChunk - 1) / kScanChunk;
  return al(4ull * entries) + al(4ull * chunks) + al(4ull * ((chunks + kScanChunk - 1) / kScanChunk)) + 2 * al(4ull * n);
}

void radix_sort_pairs(const uint32_t* keys, const uint32_t* vals, uint64_t n, uint32_t bits, bool descending,
                      uint32_t* keys_out, uint32_t* vals_out, void* ws, hipStream_t s) {
  radix_run(KeySrc{keys, nullptr, nullptr, vals, descending}, n, descending ? 32 : bits, keys_out, vals_out, ws, s);
}

// ---------------- rank order (linear ranking selection) ----------------
// order = individuals by ascending (score_key, index): one stable radix sort
// of (score_key, index) pairs.  The sorted keys land in the workspace's tail.
size_t rank_order_workspace_bytes(uint64_t S) { return radix_sort_workspace_bytes(S) + al(4ull * S); }

void rank_order_launch(const float* scores, uint64_t S, uint32_t* order, void* ws, hipStream_t s) {
  uint32_t* keys_out = (uint32_t*)((char*)ws + radix_sort_workspace_bytes(S));
  radix_run(KeySrc{nullptr, nullptr, scores, nullptr, false}, S, 32, keys_out, order, ws, s, 0, false, false);
}

// integer objectives: the u16 tournament keys order exactly like the scores;
// only the bits of the largest possible key (key_range - 1) are sorted
namespace {
uint32_t key_bits(uint32_t key_range) {
  uint32_t bits = 1;
  while (bits < 16 && (1u << bits) < key_range) ++bits;
  return bits;
}
}  // namespace

void rank_order16_launch(const uint16_t* keys16, uint64_t S, uint32_t key_range, uint32_t* order, void* ws,
                         hipStream_t s, bool counts_ready) {
  const uint32_t bits = key_bits(key_range);
  if (counts_ready && !wide_mode(bits, key_range)) throw std::logic_error("rank order: fused counts need the single pass");
  uint32_t* keys_out = (uint32_t*)((char*)ws + radix_sort_workspace_bytes(S));
  radix_run(KeySrc{nullptr, keys16, nullptr, nullptr, false}, S, bits, keys_out, order, ws, s, key_range, counts_ready,
            false);
}

uint32_t* rank_order16_counts(void* ws, uint64_t S, uint32_t key_range) {
  if (!ws || S == 0 || !wide_mode(key_bits(key_range), key_range)) return nullptr;
  return radix_ws(ws, S).counts;
}

}  // namespace pga
