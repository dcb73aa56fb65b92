// sort.hip — stable LSD radix sort of (key, value) pairs on gfx950, written
// for the engine's two sorts: the rank order of linear-ranking selection
// (every generation, S keys) and the sorted top-k (k keys).  No library sort:
// 4-bit digits, one "onesweep" launch per digit (Merrill & Garland's
// decoupled look-back single-pass scan, applied per digit).
//
// Per pass a workgroup takes the next TILE = 256 x 8 keys (tile ids handed
// out by an atomic ticket, so every lower tile is already owned by a resident
// workgroup and the look-back below always terminates), ranks them stably in
// LDS (a [16 digits][256 threads] counter table, scanned digit-major), then
// lanes 0..15 of wave 0 publish the tile's per-digit counts and look back over
// the earlier tiles' status words for the exclusive prefix of each digit.  A
// status word carries its own payload ({flag, count} in 32 bits, one store),
// so neither side needs a fence: the consumer polls it with L1-bypassing
// atomic loads.  Keys land at digit_base[d] + prefix[d] + local rank.
// digit_base comes from one up-front histogram launch that counts every
// pass's digits at once (digit counts do not depend on the key order).
//
// Reference: the reference has no selection but binary tournament
// (src/pga.cu:278-292); linear ranking is the "placeholder" selection enum
// (include/pga.h:36-42) made real.
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"

namespace pga {
namespace {

using namespace dev;

constexpr uint32_t kRadixBits = 4;
constexpr uint32_t kRadix = 1u << kRadixBits;  // 16 digits
constexpr uint32_t kItems = 8;                   // keys per thread
constexpr uint32_t kTile = kBlock * kItems;      // 2048 keys per workgroup
constexpr uint32_t kMaxPasses = 8;               // 32-bit keys
constexpr uint32_t kFlagAgg = 1u << 30, kFlagIncl = 2u << 30, kCountMask = (1u << 30) - 1u;

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// workspace: [hist kMaxPasses x 16 | tickets kMaxPasses | pad] [status passes x tiles x 16] [keys A] [vals A]
struct RadixWs {
  uint32_t* hist;
  uint32_t* ticket;
  uint32_t* status;
  uint32_t* k;
  uint32_t* v;
  size_t head_bytes;  // hist + tickets + status: zeroed before every sort
};

RadixWs radix_ws(void* ws, uint64_t n) {
  const uint64_t tiles = (n + kTile - 1) / kTile;
  char* p = (char*)ws;
  RadixWs w;
  w.hist = (uint32_t*)p;
  w.ticket = w.hist + kMaxPasses * kRadix;
  p += al(4ull * (kMaxPasses * kRadix + kMaxPasses));
  w.status = (uint32_t*)p;
  p += al(4ull * kMaxPasses * tiles * kRadix);
  w.head_bytes = (size_t)(p - (char*)ws);
  w.k = (uint32_t*)p;
  p += al(4ull * n);
  w.v = (uint32_t*)p;
  return w;
}

// keys (and iota values when vals == nullptr) -> staging; every pass's digit
// histogram.  Key sources: u32 keys, u16 keys (zero-extended), or f32 scores
// (score_key: ascending score order), selected by which pointer is set.
__global__ __launch_bounds__(kBlock) void radix_hist_kernel(const uint32_t* k32, const uint16_t* k16, const float* f32,
                                                            bool invert, const uint32_t* vals, uint64_t n,
                                                            uint32_t passes, uint32_t* keys_out, uint32_t* vals_out,
                                                            uint32_t* hist) {
  __shared__ uint32_t h[kMaxPasses][kRadix];
  for (uint32_t i = threadIdx.x; i < kMaxPasses * kRadix; i += kBlock) (&h[0][0])[i] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    uint32_t key = k32 ? k32[i] : (k16 ? (uint32_t)k16[i] : score_key(f32[i]));
    if (invert) key = ~key;
    keys_out[i] = key;
    vals_out[i] = vals ? vals[i] : (uint32_t)i;
    for (uint32_t p = 0; p < passes; ++p) atomicAdd(&h[p][(key >> (kRadixBits * p)) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < passes * kRadix; i += kBlock) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], c);
  }
}

__device__ __forceinline__ uint32_t ld_status(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One digit pass: keys/vals in -> out, stable, by digit (key >> shift) & 15.
__global__ __launch_bounds__(kBlock) void radix_pass_kernel(const uint32_t* __restrict__ kin,
                                                            const uint32_t* __restrict__ vin,
                                                            uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                            uint64_t n, uint32_t pass, const uint32_t* hist,
                                                            uint32_t* ticket, uint32_t* status) {
  __shared__ uint32_t cnt[kRadix][kBlock];   // [digit][thread], then its digit-major exclusive scan
  __shared__ uint32_t lds_tile, lds_base[kRadix], lds_wsum[kBlock / 64];
  const uint32_t t = threadIdx.x, lane = lane_id(), wid = t >> 6;
  const uint32_t shift = kRadixBits * pass;
  if (t == 0) lds_tile = atomicAdd(&ticket[pass], 1u);
  for (uint32_t d = 0; d < kRadix; ++d) cnt[d][t] = 0;
  __syncthreads();
  const uint32_t tile = lds_tile;
  const uint64_t base = (uint64_t)tile * kTile + (uint64_t)t * kItems;  // blocked: thread t owns 8 consecutive keys

  uint32_t key[kItems], val[kItems], dig[kItems], rnk[kItems];
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i) {
    const bool ok = base + i < n;
    key[i] = ok ? kin[base + i] : 0xFFFFFFFFu;
    val[i] = ok ? vin[base + i] : 0u;
    dig[i] = ok ? (key[i] >> shift) & (kRadix - 1) : kRadix;  // past the end: no digit
  }
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i) {  // rank within the thread (column t is private)
    if (dig[i] < kRadix) {
      rnk[i] = cnt[dig[i]][t];
      cnt[dig[i]][t] = rnk[i] + 1;
    }
  }
  __syncthreads();
  // exclusive scan of cnt in digit-major order: thread t owns the 16
  // consecutive entries [16 t, 16 t + 16) of the flattened table
  uint32_t* flat = &cnt[0][0];
  uint32_t loc[kRadix], s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kRadix; ++j) {
    loc[j] = s;
    s += flat[kRadix * t + j];
  }
  uint32_t incl = s;  // wave inclusive scan of the thread sums
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) lds_wsum[wid] = incl;
  __syncthreads();
  uint32_t off = incl - s;
  for (uint32_t w = 0; w < wid; ++w) off += lds_wsum[w];
#pragma unroll
  for (uint32_t j = 0; j < kRadix; ++j) flat[kRadix * t + j] = off + loc[j];
  __syncthreads();
  // cnt[d][u] = keys of the tile with digit < d, plus digit d in threads < u
  if (wid == 0 && lane < kRadix) {
    const uint32_t d = lane;
    const uint32_t start = cnt[d][0];
    const uint32_t total = (d + 1 < kRadix ? cnt[d + 1][0] : (uint32_t)min((uint64_t)kTile, n - (uint64_t)tile * kTile)) - start;
    uint32_t* st = status + ((uint64_t)pass * ((n + kTile - 1) / kTile) + tile) * kRadix;
    st_status(st + d, (tile == 0 ? kFlagIncl : kFlagAgg) | total);
    uint32_t prefix = 0;
    if (tile > 0) {
      // look back: add aggregates until an inclusive prefix is found
      for (int64_t j = (int64_t)tile - 1; j >= 0; --j) {
        const uint32_t* sp = st - (uint64_t)(tile - j) * kRadix + d;
        uint32_t w = ld_status(sp);
        for (uint32_t spin = 0; (w >> 30) == 0u && spin < (1u << 24); ++spin) {  // bounded: predecessors are resident
          __builtin_amdgcn_s_sleep(1);
          w = ld_status(sp);
        }
        prefix += w & kCountMask;
        if ((w >> 30) == 2u) break;
      }
      st_status(st + d, kFlagIncl | (prefix + total));
    }
    // digit base over all keys: the histogram's exclusive prefix
    uint32_t db = 0;
    for (uint32_t e = 0; e < d; ++e) db += hist[pass * kRadix + e];
    lds_base[d] = db + prefix - start;  // + cnt[d][u] + rank = output position
  }
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < kItems; ++i) {
    if (dig[i] < kRadix) {
      const uint32_t pos = lds_base[dig[i]] + cnt[dig[i]][t] + rnk[i];
      kout[pos] = key[i];
      vout[pos] = val[i];
    }
  }
}

uint32_t passes_for(uint32_t bits) { return (bits + kRadixBits - 1) / kRadixBits; }

// one sort: zero the counters, stage + histogram, the digit passes.  The
// passes ping-pong between the workspace staging (A) and the output (B); the
// keys are staged where an even number of flips ends in B.
void radix_run(const uint32_t* k32, const uint16_t* k16, const float* f32, bool invert, const uint32_t* vals,
               uint64_t n, uint32_t bits, uint32_t* kout, uint32_t* vout, void* ws, hipStream_t s) {
  if (n == 0) return;
  if (n > (uint64_t)kCountMask) throw std::invalid_argument("radix sort: more than 2^30 keys");
  const uint32_t passes = passes_for(bits < 1 ? 1 : (bits > 32 ? 32 : bits));
  RadixWs w = radix_ws(ws, n);
  PGA_HIP_CHECK(hipMemsetAsync(ws, 0, w.head_bytes, s));
  uint32_t* ck = passes % 2 ? w.k : kout;
  uint32_t* cv = passes % 2 ? w.v : vout;
  const uint32_t grid = launch_grid(n, kBlock * 8);
  hipLaunchKernelGGL(radix_hist_kernel, grid, kBlock, 0, s, k32, k16, f32, invert, vals, n, passes, ck, cv, w.hist);
  const uint32_t tiles = (uint32_t)((n + kTile - 1) / kTile);
  for (uint32_t p = 0; p < passes; ++p) {
    uint32_t* dk = ck == w.k ? kout : w.k;
    uint32_t* dv = cv == w.v ? vout : w.v;
    hipLaunchKernelGGL(radix_pass_kernel, tiles, kBlock, 0, s, ck, cv, dk, dv, n, p, w.hist, w.ticket, w.status);
    ck = dk;
    cv = dv;
  }
  PGA_HIP_CHECK(hipGetLastError());
}

}  // namespace

size_t radix_sort_workspace_bytes(uint64_t n) {
  const uint64_t tiles = (n + kTile - 1) / kTile;
  return al(4ull * (kMaxPasses * kRadix + kMaxPasses)) + al(4ull * kMaxPasses * tiles * kRadix) + 2 * al(4ull * n);
}

void radix_sort_pairs(const uint32_t* keys, const uint32_t* vals, uint64_t n, uint32_t bits, bool descending,
                      uint32_t* keys_out, uint32_t* vals_out, void* ws, hipStream_t s) {
  radix_run(keys, nullptr, nullptr, descending, vals, n, descending ? 32 : bits, keys_out, vals_out, ws, s);
}

// ---------------- rank order (linear ranking selection) ----------------
// order = individuals by ascending (score_key, index): one stable radix sort
// of (score_key, index) pairs.  The sorted keys land in the workspace's tail.
size_t rank_order_workspace_bytes(uint64_t S) { return radix_sort_workspace_bytes(S) + al(4ull * S); }

void rank_order_launch(const float* scores, uint64_t S, uint32_t* order, void* ws, hipStream_t s) {
  uint32_t* keys_out = (uint32_t*)((char*)ws + radix_sort_workspace_bytes(S));
  radix_run(nullptr, nullptr, scores, false, nullptr, S, 32, keys_out, order, ws, s);
}

// integer objectives: the u16 tournament keys order exactly like the scores;
// only the bits of the largest possible key (key_range - 1) are sorted
void rank_order16_launch(const uint16_t* keys16, uint64_t S, uint32_t key_range, uint32_t* order, void* ws,
                         hipStream_t s) {
  uint32_t bits = 1;
  while (bits < 16 && (1u << bits) < key_range) ++bits;
  uint32_t* keys_out = (uint32_t*)((char*)ws + radix_sort_workspace_bytes(S));
  radix_run(nullptr, keys16, nullptr, false, nullptr, S, bits, keys_out, order, ws, s);
}

}  // namespace pga
