// util.hip — population-wide reductions, roulette prefix sums, radix-select
// top-k, and row gather/scatter (elitism, migration, best queries).
//
// Replaces the reference's host-side argmax over a D2H copy of every score
// (pga_get_best, src/pga.cu:218-236) and implements its stubbed top-N /
// migration entry points (src/pga.cu:238-248, :368-374) on the device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <unordered_map>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/tp.hpp"

namespace pga {

int device_cu_count() {
  static int counts[64] = {0};
  int dev = 0;
  PGA_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (counts[dev] == 0) {
    int n = 0;
    PGA_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    counts[dev] = n > 0 ? n : 256;
  }
  return counts[dev];
}

uint32_t launch_grid(uint64_t S, uint32_t per_block) {
  uint64_t need = (S + per_block - 1) / per_block;
  uint64_t cap = (uint64_t)device_cu_count() * 8;
  if (cap > kMaxGrid) cap = kMaxGrid;
  uint64_t g = need < cap ? need : cap;
  return (uint32_t)(g == 0 ? 1 : g);
}

uint32_t occupancy_blocks(const void* kernel, int block, size_t dyn_lds) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, int, size_t>, int> cache;
  int dev = 0;
  PGA_HIP_CHECK(hipGetDevice(&dev));
  const auto key = std::make_tuple(kernel, dev, block, dyn_lds);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return (uint32_t)it->second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, block, dyn_lds) != hipSuccess || n <= 0) n = 1;
  cache[key] = n;
  return (uint32_t)n;
}

bool force_generic_kernels() {
  static const bool v = [] {
    const char* e = getenv("PGA_FORCE_GENERIC");
    return e && e[0] == '1';
  }();
  return v;
}

size_t allow_dynamic_lds(const void* kernel) {
  // once per (kernel, device): the attribute is per device, so a process that
  // drives a second GPU raises it there too
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> raised;
  int dev = 0;
  PGA_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = raised.find({kernel, dev});
  if (it != raised.end()) return it->second;
  hipFuncAttributes at;
  PGA_HIP_CHECK(hipFuncGetAttributes(&at, kernel));
  const size_t avail = 160 * 1024 - at.sharedSizeBytes;
  PGA_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)avail));
  raised[{kernel, dev}] = avail;
  return avail;
}

TpGeom tp_geometry(uint64_t S, uint32_t islands, const void* kernel, uint32_t ng, uint32_t pseg) {
  (void)allow_dynamic_lds(kernel);  // the 16-wave launch's dynamic LDS is above the default limit
  return tp_geometry_occ(S, islands, occupancy_blocks(kernel, 256, dev::tp_dyn_lds(4, pseg)), ng, pseg);
}

uint32_t tp_dyn_lds_bytes(uint32_t nw, uint32_t pseg) { return dev::tp_dyn_lds(nw, pseg); }
uint32_t tp_jit_stage_bytes(uint32_t nw) { return dev::tp_jit_stage_lds(nw); }

uint32_t tp_skew_units(const TpGeom& t, uint64_t S) {
  // PGA_TP_SKEW = units each odd block of a pair hands to its even
  // neighbour (one 16-wave block per CU only: there block b runs on XCD b % 8;
  // at most a quarter of a block's units)
  static const uint32_t d = [] {
    // default 2 of the 64 units of the headline's blocks: interleaved A/B
    // (round 4) 0 / 2 / 4 / 6 -> 90.7 / 90.2 / 92.7 / 95.4 us per generation
    const char* e = std::getenv("PGA_TP_SKEW");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 2u;
  }();
  if (d == 0 || t.block != dev::kTpMaxWaves * 64 || t.grid < 2) return 0;
  const uint64_t per = (S + t.grid - 1) / t.grid, units = (per + t.unit - 1) / t.unit;
  return d * 4 < units ? d : 0u;
}

uint32_t tp_pool_units(const TpGeom& t, uint64_t S) {
  // PGA_TP_POOL = d: 1/d of each block's units in the pair pool (default 0: none)
  static const uint32_t d = [] {
    const char* e = std::getenv("PGA_TP_POOL");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;  // off by default (tp.hpp)
  }();
  if (d == 0 || t.block != dev::kTpMaxWaves * 64 || t.grid < 2) return 0;
  const uint64_t per = (S + t.grid - 1) / t.grid, units = (per + t.unit - 1) / t.unit;
  return (uint32_t)(units / d);
}

TpGeom tp_geometry_occ(uint64_t S, uint32_t islands, uint32_t occ4, uint32_t ng, uint32_t pseg) {
  if (islands == 0) islands = 1;
  if (ng == 0 || ng > 64) ng = 64;
  const uint32_t cus = (uint32_t)device_cu_count();
  const uint32_t share = cus / islands > 0 ? cus / islands : 1;
  // one 16-wave block per CU when every wave breeds at least one 64-child unit
  if ((S + 63) / 64 >= (uint64_t)dev::kTpMaxWaves * share)
    return {share, dev::kTpMaxWaves * 64, dev::tp_dyn_lds(dev::kTpMaxWaves, pseg), 64};
  // else 4-wave blocks on the occupancy grid, with units small enough that
  // every resident wave gets one (each unit costs U / ng dependent steps)
  uint64_t cap = (uint64_t)cus * (occ4 > 0 ? occ4 : 1) / islands;
  if (cap < 1) cap = 1;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint64_t per_wave = (S + 4 * cap - 1) / (4 * cap);
  uint32_t u = ng * dev::tp_prefetch_depth(64 / ng);  // a unit holds >= PD steps
  static const uint32_t umax = [] {  // PGA_TP_UMAX: largest unit of this grid (sweeps)
    const char* e = std::getenv("PGA_TP_UMAX");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 64u;
  }();
  while (u < 64 && u < per_wave && 2 * u <= umax) u *= 2;
  const uint64_t need = (S + 4ull * u - 1) / (4ull * u);
  const uint64_t g = need < cap ? need : cap;
  return {(uint32_t)(g == 0 ? 1 : g), 256u, dev::tp_dyn_lds(4, pseg), u};
}

uint32_t launch_grid_occ(uint64_t S, uint32_t per_block, const void* kernel) {
  uint64_t need = (S + per_block - 1) / per_block;
  uint64_t cap = (uint64_t)device_cu_count() * occupancy_blocks(kernel, dev::kBlock);
  if (cap > kMaxGrid) cap = kMaxGrid;
  uint64_t g = need < cap ? need : cap;
  return (uint32_t)(g == 0 ? 1 : g);
}

void build_mut_table(float p, uint32_t L, uint32_t* out, float* inv_log2_1mp) {
  const double q = 1.0 - (double)p;
  double t = 1.0;
  for (uint32_t m = 1; m <= L; ++m) {
    t *= q;
    double v = std::floor(t * 4294967296.0);
    out[m - 1] = v >= 4294967295.0 ? 0xFFFFFFFFu : (v <= 0.0 ? 0u : (uint32_t)v);
  }
  if (p <= 0.f) *inv_log2_1mp = 0.f;
  else if (p >= 1.f) *inv_log2_1mp = 0.f;
  else *inv_log2_1mp = (float)(1.0 / std::log2(q));
}

void build_binom_table(float p, uint32_t L, uint32_t* out) {
  // out[k] = floor(P(K <= k) * 2^32), K ~ Binomial(L, p); 0xFFFFFFFF once the
  // remaining tail is below 2^-32 (ends the table, see binom_count)
  const long double pp = p, qq = 1.0L - pp;
  long double pmf = expl((long double)L * log1pl(-pp)), cdf = 0.0L;
  for (uint32_t k = 0; k < kMutCap; ++k) {
    cdf += pmf;
    const long double v = floorl(cdf * 4294967296.0L);
    out[k] = v >= 4294967295.0L ? 0xFFFFFFFFu : (uint32_t)v;
    pmf = k < L ? pmf * (long double)(L - k) / (long double)(k + 1) * pp / qq : 0.0L;
  }
  out[kMutCap - 1] = 0xFFFFFFFFu;
}

namespace {
using namespace dev;

__global__ __launch_bounds__(kBlock) void reduce_best_kernel(const unsigned long long* parts, uint32_t n,
                                                             unsigned long long* out) {
  __shared__ unsigned long long lds[kBlock / 64];
  unsigned long long b = block_reduce_parts(parts, n, lds);
  if (threadIdx.x == 0) out[0] = b;
}

// per-block best partials of a score array; with `keys` also refreshes the
// u16 tournament keys in the same pass (integer objectives)
__global__ __launch_bounds__(kBlock) void best_of_scores_kernel(const float* scores, uint64_t S,
                                                                unsigned long long* parts, uint16_t* keys) {
  __shared__ unsigned long long lds[kBlock / 64];
  unsigned long long b = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < S; i += (uint64_t)gridDim.x * kBlock) {
    const float v = scores[i];
    unsigned long long p = pack_best(v, i);
    b = p > b ? p : b;
    if (keys) keys[i] = (uint16_t)(!(v > 0.f) ? 0.f : (v >= 65535.f ? 65535.f : v));
  }
  b = block_max_u64(b, lds);
  if (threadIdx.x == 0) parts[blockIdx.x] = b;
}

template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* lds, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane_id() == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  T r = lds[0];
#pragma unroll
  for (int i = 1; i < kBlock / 64; ++i) r = op(r, lds[i]);
  return r;
}

struct FMin { __device__ float operator()(float a, float b) const { return fminf(a, b); } };
struct FMax { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
struct FAdd { __device__ float operator()(float a, float b) const { return a + b; } };

// stage 1: per-block {min, max, sum}
__global__ __launch_bounds__(kBlock) void stats_part_kernel(const float* s, uint64_t S, float* parts) {
  __shared__ float lds[kBlock / 64];
  float mn = INFINITY, mx = -INFINITY, sm = 0.f;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < S; i += (uint64_t)gridDim.x * kBlock) {
    float v = s[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    sm += v;
  }
  mn = block_reduce(mn, lds, FMin());
  mx = block_reduce(mx, lds, FMax());
  sm = block_reduce(sm, lds, FAdd());
  if (threadIdx.x == 0) {
    parts[3 * blockIdx.x + 0] = mn;
    parts[3 * blockIdx.x + 1] = mx;
    parts[3 * blockIdx.x + 2] = sm;
  }
}

__global__ __launch_bounds__(kBlock) void stats_final_kernel(const float* parts, uint32_t n, uint64_t S,
                                                             float* out) {
  __shared__ float lds[kBlock / 64];
  float mn = INFINITY, mx = -INFINITY, sm = 0.f;
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
    mn = fminf(mn, parts[3 * i]);
    mx = fmaxf(mx, parts[3 * i + 1]);
    sm += parts[3 * i + 2];
  }
  mn = block_reduce(mn, lds, FMin());
  mx = block_reduce(mx, lds, FMax());
  sm = block_reduce(sm, lds, FAdd());
  if (threadIdx.x == 0) {
    out[0] = mn;
    out[1] = mx;
    out[2] = sm;
    out[3] = (float)S;
  }
}

// roulette: contiguous range per block, weights = max(s - min, 0)
__device__ __forceinline__ float block_excl_scan(float v, float* lds, float& total) {
  // inclusive wave scan
  const uint32_t lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float t = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += t;
  }
  __syncthreads();
  if (lane == 63) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  float off = 0.f;
  total = 0.f;
  for (int i = 0; i < kBlock / 64; ++i) {
    if (i < (int)(threadIdx.x >> 6)) off += lds[i];
    total += lds[i];
  }
  return off + v;  // inclusive
}

// Roulette in three launches: PART (per-block weight sums), FINAL (each block
// reduces the sums before it for its carry, scans its range into cumfit; the
// last block publishes the guide scale), GUIDE (bucket -> first individual).
// The score minimum comes from the generation kernel's fused {min, sum}
// partials when it stored them (PART reduces them in every block and block 0
// publishes it), else from score_stats_launch beforehand.
__device__ __forceinline__ float parts_min(const float* parts, uint32_t n, float* lds) {
  float mn = INFINITY;
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) mn = fminf(mn, parts[2 * i]);
  return block_reduce(mn, lds, FMin());
}

__global__ __launch_bounds__(kBlock) void prefix_part_kernel(const float* s, uint64_t S, uint64_t per_block,
                                                             const float* parts, uint32_t nparts, float* stats,
                                                             float* block_sums) {
  __shared__ float lds[kBlock / 64];
  float mn;
  if (parts) {
    mn = parts_min(parts, nparts, lds);
    if (blockIdx.x == 0 && threadIdx.x == 0) stats[0] = mn;
  } else {
    mn = stats[0];
  }
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  float sm = 0.f;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += kBlock) sm += fmaxf(s[i] - mn, 0.f);
  sm = block_reduce(sm, lds, FAdd());
  if (threadIdx.x == 0) block_sums[blockIdx.x] = sm;
}

__global__ __launch_bounds__(kBlock) void prefix_final_kernel(const float* s, uint64_t S, uint64_t per_block,
                                                              const float* stats, const float* block_sums,
                                                              float* cumfit, float* meta) {
  __shared__ float lds[kBlock / 64];
  const float mn = stats[0];
  // carry = the sums of the blocks before this one, in a fixed order
  float pre = 0.f;
  for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kBlock) pre += block_sums[j];
  float carry = block_reduce(pre, lds, FAdd());
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  for (uint64_t t0 = b0; t0 < b1; t0 += kBlock) {
    uint64_t i = t0 + threadIdx.x;
    float v = i < b1 ? fmaxf(s[i] - mn, 0.f) : 0.f;
    float total;
    float inc = block_excl_scan(v, lds, total);
    if (i < b1) cumfit[i] = carry + inc;
    if (i == S - 1) meta[0] = carry + inc > 0.f ? (float)S / (carry + inc) : 0.f;  // guide scale (roulette_bucket)
    carry += total;
    __syncthreads();
  }
}

// Integer objectives: the same two passes with u64 weight sums, so cumfit[i]
// is the exact prefix rounded once to f32 — what roulette_fused_kernel and the
// CPU backend's f64 prefix give, at any population size.
template <int BLK>
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane_id() == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long t = 0;
  for (uint32_t w = 0; w < BLK / 64; ++w) t += lds[w];
  return t;
}

__global__ __launch_bounds__(kBlock) void prefix_part_int_kernel(const float* s, uint64_t S, uint64_t per_block,
                                                                 const float* parts, uint32_t nparts, float* stats,
                                                                 unsigned long long* block_sums) {
  __shared__ float lds[kBlock / 64];
  __shared__ unsigned long long lds64[kBlock / 64];
  float mn;
  if (parts) {
    mn = parts_min(parts, nparts, lds);
    if (blockIdx.x == 0 && threadIdx.x == 0) stats[0] = mn;
  } else {
    mn = stats[0];
  }
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  unsigned long long sm = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += kBlock) sm += (unsigned long long)fmaxf(s[i] - mn, 0.f);
  sm = block_sum_u64<kBlock>(sm, lds64);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = sm;
}

__global__ __launch_bounds__(kBlock) void prefix_final_int_kernel(const float* s, uint64_t S, uint64_t per_block,
                                                                  const float* stats,
                                                                  const unsigned long long* block_sums, float* cumfit,
                                                                  float* meta) {
  __shared__ unsigned long long lds64[kBlock / 64];
  const float mn = stats[0];
  unsigned long long pre = 0;
  for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kBlock) pre += block_sums[j];
  unsigned long long carry = block_sum_u64<kBlock>(pre, lds64);
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  for (uint64_t t0 = b0; t0 < b1; t0 += kBlock) {
    const uint64_t i = t0 + threadIdx.x;
    const unsigned long long v = i < b1 ? (unsigned long long)fmaxf(s[i] - mn, 0.f) : 0ull;
    unsigned long long inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    __syncthreads();
    if (lane == 63) lds64[wid] = inc;
    __syncthreads();
    unsigned long long off = 0, total = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w) {
      off += w < wid ? lds64[w] : 0ull;
      total += lds64[w];
    }
    const float c = __ull2float_rn(carry + off + inc);
    if (i < b1) cumfit[i] = c;
    if (i == S - 1) meta[0] = c > 0.f ? (float)S / c : 0.f;  // guide scale (roulette_bucket)
    carry += total;
  }
}

// guide[b] = i for every bucket b in (bucket(cumfit[i-1]), bucket(cumfit[i])].
// Spans of 32 buckets or more (one individual holding >= 32/S of the total
// weight) are queued in LDS and filled by the whole block, so no thread loops
// over a heavy individual's buckets.
// cov: kGuideCovered, or 0 (no covered flags: S >= 2^31, or PGA_ROUL_COVER=0)
// gsh 1: the packed table (GenArgs::roul_packed): guide[b] at word 2 b, cumfit[i] at word 2 i + 1
__global__ __launch_bounds__(kBlock) void roulette_guide_kernel(const float* c, uint64_t S, const float* meta,
                                                                 uint32_t* guide, uint32_t cov, uint32_t gsh) {
  __shared__ uint4 spans[kBlock];
  __shared__ uint32_t nsp;
  const float scale = meta[0];
  const uint32_t B = (uint32_t)S;
  for (uint64_t t0 = (uint64_t)blockIdx.x * kBlock; t0 < S; t0 += (uint64_t)gridDim.x * kBlock) {  // block-uniform
    if (threadIdx.x == 0) nsp = 0;
    __syncthreads();
    const uint64_t i = t0 + threadIdx.x;
    if (i < S) {
      const float ci = c[i];
      if (gsh) guide[2 * i + 1] = __builtin_bit_cast(uint32_t, ci);
      const uint32_t hi = roulette_bucket(ci, scale, B);
      const uint32_t lo = i ? roulette_bucket(c[i - 1], scale, B) + 1u : 0u;
      if (hi >= lo) {
        if (hi - lo < 32u) {
          for (uint32_t b = lo; b <= hi; ++b) guide[b << gsh] = (uint32_t)i | (b < hi ? cov : 0u);
        } else {
          spans[atomicAdd(&nsp, 1u)] = make_uint4(lo, hi, (uint32_t)i, 0u);
        }
      }
    }
    __syncthreads();
    const uint32_t n = nsp;
    for (uint32_t k = 0; k < n; ++k) {
      const uint4 sp = spans[k];
      for (uint32_t b = sp.x + threadIdx.x; b <= sp.y; b += kBlock) guide[b << gsh] = sp.z | (b < sp.y ? cov : 0u);
    }
    __syncthreads();
  }
}

// Roulette in ONE launch for an integer objective (roulette_fused_launch):
// block j of this grid takes the children block j of the generation kernel
// wrote (tp_share over the same grid), whose {min, sum} partials are exact
// integers in f32.  Every block reduces all partials itself: the minimum, the
// weight total sum_i - n_i * min of every partial, the total and the sum of
// the partials before it (its carry), in u64 — so the three-launch chain
// (partials pass, carry + scan, guide) becomes one, and the prefix sums are
// exact (cumfit[i] = the integer prefix rounded once; the guide scale is
// S / cumfit[S - 1] as in prefix_final_kernel).  The block then scans its
// range (kRoulPer consecutive individuals per thread, loaded and stored
// coalesced through LDS) and fills the guide
// buckets of its individuals as roulette_guide_kernel does.
constexpr uint32_t kRoulThreads = 1024, kRoulPer = 8, kRoulSpans = 1024;

__global__ __launch_bounds__(kRoulThreads) void roulette_fused_kernel(const float* __restrict__ s, uint64_t S,
                                                                      const float* __restrict__ parts, uint32_t unit,
                                                                      uint32_t skew, float* __restrict__ cumfit,
                                                                      uint32_t* __restrict__ guide, float* meta,
                                                                      uint32_t cov, uint32_t gsh) {
  __shared__ unsigned long long red[kRoulThreads / 64];
  __shared__ float fred[kRoulThreads / 64];
  __shared__ uint32_t wsum[kRoulThreads / 64];
  __shared__ uint4 spans[kRoulSpans];
  __shared__ uint32_t nsp;
  __shared__ __align__(16) uint32_t xch[kRoulThreads * kRoulPer];  // a chunk's weights, then its cumfit values
  const uint32_t t = threadIdx.x, lane = lane_id(), wid = t >> 6, np = gridDim.x;
  const uint32_t Su = (uint32_t)S;
  uint32_t bb, be;
  tp_share(Su, unit, blockIdx.x, bb, be, skew);
  // the first chunk's scores, loaded before the partials are reduced (the two
  // global round trips overlap; a share of up to kRoulThreads * kRoulPer, the
  // usual case, is this one chunk)
  float sv0[kRoulPer];
#pragma unroll
  for (uint32_t k = 0; k < kRoulPer; ++k) {
    const uint32_t i = bb + k * kRoulThreads + t;
    sv0[k] = s[i < be ? i : (be > 0u ? be - 1u : 0u)];  // unconditional load
  }
  float mn = __builtin_inff();
  for (uint32_t i = t; i < np; i += kRoulThreads) mn = fminf(mn, parts[2 * i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
  if (lane == 0) fred[wid] = mn;
  __syncthreads();
  mn = fred[0];
  for (uint32_t w = 1; w < kRoulThreads / 64; ++w) mn = fminf(mn, fred[w]);
  const unsigned long long mnu = (unsigned long long)mn;  // an integer objective's scores are >= 0
  unsigned long long below = 0, tot = 0;
  for (uint32_t i = t; i < np; i += kRoulThreads) {
    uint32_t b0, b1;
    tp_share(Su, unit, i, b0, b1, skew);
    const unsigned long long w = b1 > b0 ? (unsigned long long)parts[2 * i + 1] - (unsigned long long)(b1 - b0) * mnu : 0ull;
    tot += w;
    below += i < blockIdx.x ? w : 0ull;
  }
  tot = block_sum_u64<kRoulThreads>(tot, red);
  below = block_sum_u64<kRoulThreads>(below, red);
  const float total = __ull2float_rn(tot);
  const float scale = tot > 0ull ? (float)S / total : 0.f;
  if (blockIdx.x == 0 && t == 0) meta[0] = scale;
  unsigned long long carry = below;
  for (uint32_t c0 = bb; c0 < be; c0 += kRoulThreads * kRoulPer) {  // block-uniform
    // coalesced loads, transposed through LDS: thread t scans the kRoulPer
    // consecutive weights [t P, t P + P) of the chunk
#pragma unroll
    for (uint32_t k = 0; k < kRoulPer; ++k) {
      const uint32_t i = c0 + k * kRoulThreads + t;
      const float v = i < be ? (c0 == bb ? sv0[k] : s[i]) : mn;
      xch[k * kRoulThreads + t] = (uint32_t)fmaxf(v - mn, 0.f);
    }
    if (t == 0) nsp = 0;
    __syncthreads();
    uint32_t w[kRoulPer], ts = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRoulPer; j += 4) {
      const uint4 q = *(const uint4*)&xch[t * kRoulPer + j];
      w[j] = q.x;
      w[j + 1] = q.y;
      w[j + 2] = q.z;
      w[j + 3] = q.w;
    }
#pragma unroll
    for (uint32_t j = 0; j < kRoulPer; ++j) ts += w[j];
    uint32_t incl = ts;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();  // (every thread has read its weights: xch is reused for the prefix sums)
    uint32_t off = incl - ts, ctot = 0;
    for (uint32_t q = 0; q < kRoulThreads / 64; ++q) {
      off += q < wid ? wsum[q] : 0u;
      ctot += wsum[q];
    }
    unsigned long long run = carry + off;  // the exact prefix before the thread's first individual
    float c[kRoulPer];
#pragma unroll
    for (uint32_t j = 0; j < kRoulPer; ++j) {
      run += w[j];
      c[j] = __ull2float_rn(run);
    }
#pragma unroll
    for (uint32_t j = 0; j < kRoulPer; j += 4)
      *(float4*)&xch[t * kRoulPer + j] = make_float4(c[j], c[j + 1], c[j + 2], c[j + 3]);
    __syncthreads();
    // coalesced stores; the guide buckets of individual i, as roulette_guide_kernel
    const float prev0 = __ull2float_rn(carry);  // = cumfit[c0 - 1]
#pragma unroll
    for (uint32_t k = 0; k < kRoulPer; ++k) {
      const uint32_t e = k * kRoulThreads + t, i = c0 + e;
      if (i < be) {
        const float ci = __builtin_bit_cast(float, xch[e]);
        const float prev = e ? __builtin_bit_cast(float, xch[e - 1]) : prev0;
        cumfit[i] = ci;
        if (gsh) guide[2 * i + 1] = __builtin_bit_cast(uint32_t, ci);
        const uint32_t hi = roulette_bucket(ci, scale, Su);
        const uint32_t lo = i ? roulette_bucket(prev, scale, Su) + 1u : 0u;
        if (hi >= lo) {
          const uint32_t q = hi - lo < 32u ? kRoulSpans : atomicAdd(&nsp, 1u);
          if (q < kRoulSpans) spans[q] = make_uint4(lo, hi, i, 0u);
          else
            for (uint32_t b = lo; b <= hi; ++b) guide[b << gsh] = i | (b < hi ? cov : 0u);  // short span (or a full queue)
        }
      }
    }
    __syncthreads();
    const uint32_t n = nsp < kRoulSpans ? nsp : kRoulSpans;
    for (uint32_t q = 0; q < n; ++q) {
      const uint4 sp = spans[q];
      for (uint32_t b = sp.x + t; b <= sp.y; b += kRoulThreads) guide[b << gsh] = sp.z | (b < sp.y ? cov : 0u);
    }
    __syncthreads();  // (nsp, wsum and xch are reused by the next chunk)
    carry += ctot;
  }
}

// ---------------- radix-select top-k ----------------
struct TopkState {
  uint32_t prefix, mask, remaining, pad;
  uint32_t hist[256];
};

__device__ __forceinline__ uint32_t topk_key(float s, bool largest) {
  uint32_t k = score_key(s);
  return largest ? k : ~k;
}

// Keys of the selection: 32-bit orderable f32 keys, or (integer objectives)
// the population's u16 tournament keys — two radix passes instead of four.
// u16 keys are clamped to vmax (= R - 1 of a value-histogram selection) in
// every pass, exactly as the histogram bins them: a key above the objective's
// range (a checkpoint's or an unvalidated migrant's score) can then neither
// make the passes disagree nor write past k indices.
template <int BITS>
struct TopkKeys {
  const float* s;
  const uint16_t* k16;
  bool largest;
  uint32_t vmax = 0xFFFFu;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    if (BITS == 16) {
      const uint32_t v = min((uint32_t)k16[i], vmax);
      return largest ? v : 0xFFFFu - v;
    }
    return topk_key(s[i], largest);
  }
};

__global__ __launch_bounds__(kBlock) void topk_init_kernel(TopkState* st, uint32_t k) {
  if (threadIdx.x == 0) {
    st->prefix = 0;
    st->mask = 0;
    st->remaining = k;
  }
  st->hist[threadIdx.x] = 0;
}

// 8-bit digit histogram of the keys that match the prefix found so far.
// Scores cluster (a converging population shares its high bytes), so lanes
// of a wave are aggregated per distinct bin before the LDS atomic: one atomic
// per (wave, bin) instead of one per lane on the same address.
template <int BITS>
__global__ __launch_bounds__(kBlock) void topk_hist_kernel(TopkKeys<BITS> keys, uint64_t S, uint32_t shift,
                                                           TopkState* st) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  const uint32_t lane = lane_id();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < S; base += stride) {  // wave-uniform trip count
    const uint64_t i = base + threadIdx.x;
    uint32_t bin = 0;
    bool act = false;
    if (i < S) {
      const uint32_t key = keys(i);
      act = (key & mask) == prefix;
      bin = (key >> shift) & 255u;
    }
    // a converging population shares its high digits: when the whole wave
    // agrees on one bin, one atomic; otherwise plain per-lane LDS atomics
    const unsigned long long active = __ballot(act);
    if (active) {
      const int leader = __ffsll((long long)active) - 1;
      const uint32_t b = (uint32_t)__shfl((int)bin, leader, 64);
      const unsigned long long same = __ballot(act && bin == b);
      if (same == active) {
        if ((int)lane == leader) atomicAdd(&h[b], (uint32_t)__popcll(same));
      } else if (act) {
        atomicAdd(&h[bin], 1u);
      }
    }
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&st->hist[threadIdx.x], h[threadIdx.x]);
}

// pick the digit: the largest d whose suffix count reaches `remaining`
// (block-parallel suffix sums over the 256 bins; one thread per bin)
__global__ __launch_bounds__(kBlock) void topk_digit_kernel(TopkState* st, uint32_t shift) {
  __shared__ uint32_t suf[kBlock];
  const uint32_t t = threadIdx.x;
  const uint32_t c = st->hist[255 - t];  // reversed: suf[t] = sum of bins >= 255 - t
  const uint32_t rem = st->remaining;
  suf[t] = c;
  __syncthreads();
  for (uint32_t o = 1; o < kBlock; o <<= 1) {
    const uint32_t v = t >= o ? suf[t - o] : 0u;
    __syncthreads();
    suf[t] += v;
    __syncthreads();
  }
  // first t (largest digit 255 - t) whose inclusive suffix reaches rem
  const bool hit = suf[t] >= rem && (t == 0 || suf[t - 1] < rem);
  const bool last = t == kBlock - 1 && suf[t] < rem;  // cannot happen for k <= S; keep digit 0
  if (hit || last) {
    const uint32_t d = 255 - t;
    st->remaining = rem - (t ? suf[t - 1] : 0u);
    st->prefix |= d << shift;
    st->mask |= 255u << shift;
  }
  __syncthreads();
  st->hist[t] = 0;
}

// ---- integer objectives: the u16 keys take at most R = L + 1 values, so one
// LDS histogram of R bins replaces the radix passes ----
// 16 consecutive u16 keys [c0, c0+16) clipped to `end`: two dwordx4 loads
// issued together when the chunk is whole and aligned (c0 % 8 == 0), else
// per-key loads; bit e of the result marks key e valid
__device__ __forceinline__ uint32_t load_keys16(const uint16_t* k16, uint64_t c0, uint64_t end, uint32_t (&kv)[16]) {
  if (c0 + 16 <= end && (c0 & 7) == 0) {
    const uint4 a = *(const uint4*)(k16 + c0), b = *(const uint4*)(k16 + c0 + 8);
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      kv[2 * e] = w[e] & 0xFFFFu;
      kv[2 * e + 1] = w[e] >> 16;
    }
    return 0xFFFFu;
  }
  uint32_t m = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool ok = c0 + e < end;
    kv[e] = ok ? k16[c0 + e] : 0u;
    m |= ok ? (1u << e) : 0u;
  }
  return m;
}

// selections per block listed in LDS for the cooperative row move (a
// migration's k / blocks is ~41 at the headline; more go row by row).  Small:
// with ~9 KB of LDS the selections fit beside a generation kernel's block
// (120 KB), so one on the transport stream runs concurrently with it.
constexpr uint32_t kTopkMoveSlots = 1024;

// What the fused selection does with the i-th selected individual at output
// position pos (besides idx_out[pos] = i when idx_out is set):
//   GATHER   out rows[pos] = population row i, out scores[pos] = score i (emigrants)
//   SCATTER  population row i = in rows[pos], score i and its u16 key =
//            in scores[pos] (immigrants replace the selected victims)
// so an island-migration epoch needs no separate gather / scatter kernels.
__device__ __forceinline__ void topk_emit(const TopkMove& mv, uint32_t* idx_out, uint32_t pos, uint64_t i) {
  if (idx_out) idx_out[pos] = (uint32_t)i;
  if (mv.mode == TopkMove::GATHER) {
    for (uint32_t c = 0; c < mv.rw16; ++c) mv.dst_rows[(uint64_t)pos * mv.rw16 + c] = mv.src_rows[i * mv.rw16 + c];
    mv.dst_scores[pos] = mv.src_scores[i];
  } else if (mv.mode == TopkMove::SCATTER) {
    for (uint32_t c = 0; c < mv.rw16; ++c) mv.dst_rows[i * mv.rw16 + c] = mv.src_rows[(uint64_t)pos * mv.rw16 + c];
    const float v = mv.src_scores[pos];
    mv.dst_scores[i] = v;
    if (mv.dst_keys) mv.dst_keys[i] = (uint16_t)(!(v > 0.f) ? 0.f : (v >= 65535.f ? 65535.f : v));
  }
}

__global__ __launch_bounds__(kBlock) void topk16_hist_kernel(const uint16_t* k16, uint64_t S, uint32_t R, bool largest,
                                                             uint32_t* G, uint64_t* status, uint32_t n_status) {
  uint32_t* hr = (uint32_t*)pga_dyn_lds;
  // aggregate words and ticket counters of the topk16_select_kernel that follows
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_status; i += gridDim.x * kBlock) status[i] = 0;
  if (status && blockIdx.x == 0 && threadIdx.x < 2) ((uint32_t*)(status + n_status))[threadIdx.x] = 0;
  for (uint32_t i = threadIdx.x; i < R; i += kBlock) hr[i] = 0;
  __syncthreads();
  // 16 keys per thread per pass (coalesced 32-byte chunks)
  for (uint64_t c0 = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 16; c0 < S;
       c0 += (uint64_t)gridDim.x * kBlock * 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys16(k16, c0, S, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t v = min(kv[e], R - 1);
      if ((m >> e) & 1u) atomicAdd(&hr[largest ? v : R - 1 - v], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < R; i += kBlock)
    if (hr[i]) atomicAdd(&G[i], hr[i]);
}

// every block derives the threshold from the global histogram, block 0
// publishes it, then each block counts its range (as topk_count_kernel)
__global__ __launch_bounds__(kBlock) void topk16_count_kernel(const uint16_t* k16, uint64_t S, uint64_t per_block,
                                                              uint32_t R, bool largest, uint32_t k, const uint32_t* G,
                                                              TopkState* st, uint32_t* cnt) {
  __shared__ uint32_t part[kBlock];
  __shared__ uint32_t sh_T, sh_need;
  __shared__ uint32_t lds[kBlock / 64];
  // bins from the top: thread t owns bins [R-1 - (t+1)*per + 1, R-1 - t*per]
  const uint32_t per = (R + kBlock - 1) / kBlock;
  uint32_t mine = 0;
  for (uint32_t j = 0; j < per; ++j) {
    const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
    if (b >= 0) mine += G[b];
  }
  part[threadIdx.x] = mine;
  __syncthreads();
  for (uint32_t o = 1; o < kBlock; o <<= 1) {
    const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t before = threadIdx.x ? part[threadIdx.x - 1] : 0u;
  if (before < k && part[threadIdx.x] >= k) {
    uint32_t acc = before;
    for (uint32_t j = 0; j < per; ++j) {
      const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
      if (b < 0) break;
      const uint32_t c = G[b];
      if (acc + c >= k) {
        sh_T = (uint32_t)b;
        sh_need = k - acc;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  // bin -> key in TopkKeys<16> space (largest: v; smallest: 0xFFFF - v)
  const uint32_t Tb = sh_T;
  const uint32_t T = largest ? Tb : Tb + 0x10000u - R;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->prefix = T;
    st->remaining = sh_need;
  }
  const TopkKeys<16> keys{nullptr, k16, largest, R - 1};
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  uint32_t gt = 0, eq = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += kBlock) {
    const uint32_t key = keys(i);
    gt += key > T;
    eq += key == T;
  }
  auto add = [](uint32_t a, uint32_t b) { return a + b; };
  gt = block_reduce(gt, lds, add);
  eq = block_reduce(eq, lds, add);
  if (threadIdx.x == 0) {
    cnt[2 * blockIdx.x] = gt;
    cnt[2 * blockIdx.x + 1] = eq;
  }
}

// ordered compaction: contiguous range per block
template <int BITS>
__global__ __launch_bounds__(kBlock) void topk_count_kernel(TopkKeys<BITS> keys, uint64_t S, uint64_t per_block,
                                                            const TopkState* st, uint32_t* cnt) {
  __shared__ uint32_t lds[kBlock / 64];
  const uint32_t T = st->prefix;
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  uint32_t gt = 0, eq = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += kBlock) {
    uint32_t key = keys(i);
    gt += key > T;
    eq += key == T;
  }
  auto add = [](uint32_t a, uint32_t b) { return a + b; };
  gt = block_reduce(gt, lds, add);
  eq = block_reduce(eq, lds, add);
  if (threadIdx.x == 0) {
    cnt[2 * blockIdx.x] = gt;
    cnt[2 * blockIdx.x + 1] = eq;
  }
}

__device__ __forceinline__ uint32_t block_excl_scan_u(uint32_t v, uint32_t* lds, uint32_t& total) {
  const uint32_t lane = lane_id();
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= (uint32_t)o) inc += t;
  }
  __syncthreads();
  if (lane == 63) lds[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t off = 0;
  total = 0;
  for (int i = 0; i < kBlock / 64; ++i) {
    if (i < (int)(threadIdx.x >> 6)) off += lds[i];
    total += lds[i];
  }
  return off + inc - v;
}

// exclusive scan of the per-block (gt, eq) counts, n <= 4 * kBlock, one block
__global__ __launch_bounds__(kBlock) void topk_offsets_kernel(uint32_t* cnt, uint32_t n, uint32_t* G, uint32_t R) {
  for (uint32_t i = threadIdx.x; i < R; i += kBlock) G[i] = 0;  // ready for the next selection
  __shared__ uint32_t lds[kBlock / 64];
  uint32_t g[4] = {0, 0, 0, 0}, e[4] = {0, 0, 0, 0};
  uint32_t sg = 0, se = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = 4 * threadIdx.x + j;
    if (i < n) {
      g[j] = cnt[2 * i];
      e[j] = cnt[2 * i + 1];
    }
    sg += g[j];
    se += e[j];
  }
  uint32_t tg, te;
  uint32_t og = block_excl_scan_u(sg, lds, tg);
  __syncthreads();
  uint32_t oe = block_excl_scan_u(se, lds, te);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = 4 * threadIdx.x + j;
    if (i < n) {
      cnt[2 * i] = og;
      cnt[2 * i + 1] = oe;
    }
    og += g[j];
    oe += e[j];
  }
  if (threadIdx.x == 0) cnt[2 * n] = tg;  // total strictly greater
}

// ---- integer objectives, one launch after the histogram: threshold, count,
// block offsets and the ordered write ----
// Each block takes a ticket (its position in dispatch order) and owns the
// ticket-th contiguous range; each thread owns a contiguous sub-range, so one
// block scan of the per-thread counts orders the block.  The block publishes
// its aggregate (flag | gt | eq) and then reads the aggregates of ALL its
// predecessors in parallel (one word per thread, no look-back chain): a
// predecessor by ticket is already dispatched and publishes without waiting
// on anyone, so every wait ends.  The words carry all the data, so relaxed
// agent-scope atomics suffice.  The last ticket (which has seen every other
// block's word, so every read of the histogram is done) re-zeroes the
// histogram; topk16_hist_kernel zeroes the words and the tickets before
// every selection.  Same result as count -> offsets -> write (population
// order: the strictly-beyond-threshold keys, then the first ties).
constexpr uint64_t kLbAgg = 1ull << 62, kLbMask31 = 0x7FFFFFFFull;

// G in bin space (bin = key for the largest, R - 1 - key for the smallest)
// unless grev: then G is a value-order histogram read only (the generation
// kernel's fused histogram, GenArgs::key_hist), bin b at G[R - 1 - b] for the
// smallest, and nothing re-zeroes it
// Two-pass selection, first pass (fused value-order histogram): the
// threshold exactly as topk16_select_kernel derives it, and the block's (gt,
// eq) counts over the same range -> counts[2 b], counts[2 b + 1]
__global__ __launch_bounds__(kBlock) void topk16_count2_kernel(const uint16_t* k16, uint64_t S, uint64_t per_block,
                                                               uint32_t R, bool largest, uint32_t k, const uint32_t* G,
                                                               uint32_t* counts) {
  __shared__ uint32_t sh_T;
  __shared__ uint32_t lds[kBlock / 64];
  const uint32_t per = (R + kBlock - 1) / kBlock;
  uint32_t mine = 0;
  for (uint32_t j = 0; j < per; ++j) {
    const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
    if (b >= 0) mine += G[!largest ? R - 1 - b : b];
  }
  uint32_t tot;
  const uint32_t before = block_excl_scan_u(mine, lds, tot);
  if (before < k && before + mine >= k) {
    uint32_t acc = before;
    for (uint32_t j = 0; j < per; ++j) {
      const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
      if (b < 0) break;
      const uint32_t c = G[!largest ? R - 1 - b : b];
      if (acc + c >= k) {
        sh_T = (uint32_t)b;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  const uint32_t T = largest ? sh_T : sh_T + 0x10000u - R;
  const uint32_t flip = largest ? 0u : 0xFFFFu;
  const uint64_t pt = ((per_block + kBlock - 1) / kBlock + 15) / 16 * 16;
  const uint64_t blo = (uint64_t)blockIdx.x * per_block;
  const uint64_t bhi = blo + per_block < S ? blo + per_block : S;
  const uint64_t t0 = blo + threadIdx.x * pt;
  const uint64_t t1 = t0 + pt < bhi ? t0 + pt : bhi;
  uint32_t gt = 0, eq = 0;
  for (uint64_t c0 = t0; c0 < t1; c0 += 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys16(k16, c0, t1, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t key = min(kv[e], R - 1) ^ flip;
      gt += ((m >> e) & 1u) && key > T;
      eq += ((m >> e) & 1u) && key == T;
    }
  }
  auto add = [](uint32_t x, uint32_t y) { return x + y; };
  gt = block_reduce(gt, lds, add);
  eq = block_reduce(eq, lds, add);
  if (threadIdx.x == 0) {
    counts[2 * blockIdx.x] = gt;
    counts[2 * blockIdx.x + 1] = eq;
  }
}

// counts (two-pass mode, fused histograms only): the per-block (gt, eq)
// counts of topk16_count2_kernel, complete before this launch — every block
// reads its predecessors' instead of publishing and polling status words
__global__ __launch_bounds__(kBlock) void topk16_select_kernel(const uint16_t* k16, uint64_t S, uint64_t per_block,
                                                               uint32_t R, bool largest, uint32_t k, uint32_t* G,
                                                               uint64_t* status, uint32_t* ctr, uint32_t nblocks,
                                                               uint32_t* idx_out, TopkMove mv, bool fused,
                                                               const uint32_t* counts = nullptr) {
  __shared__ uint32_t sel_pos[kTopkMoveSlots], sel_src[kTopkMoveSlots];  // row moves: output position, source
  __shared__ uint32_t sh_T, sh_need, sh_b;
  __shared__ uint32_t lds[kBlock / 64];
  if (threadIdx.x == 0) sh_b = counts ? blockIdx.x : atomicAdd(&ctr[0], 1u);
  // threshold bin: thread t owns bins [R-1 - (t+1)*per + 1, R-1 - t*per], counted from the top
  const uint32_t per = (R + kBlock - 1) / kBlock;
  uint32_t mine = 0;
  for (uint32_t j = 0; j < per; ++j) {
    const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
    if (b >= 0) mine += G[fused && !largest ? R - 1 - b : b];
  }
  uint32_t tot;
  const uint32_t before = block_excl_scan_u(mine, lds, tot);
  if (before < k && before + mine >= k) {  // the one thread holding the threshold re-reads its bins
    uint32_t acc = before;
    for (uint32_t j = 0; j < per; ++j) {
      const int64_t b = (int64_t)R - 1 - (int64_t)threadIdx.x * per - j;
      if (b < 0) break;
      const uint32_t c = G[fused && !largest ? R - 1 - b : b];
      if (acc + c >= k) {
        sh_T = (uint32_t)b;
        sh_need = k - acc;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  const uint32_t T = largest ? sh_T : sh_T + 0x10000u - R;
  const uint32_t need_eq = sh_need, gt_total = k - sh_need;
  const uint32_t b = sh_b;
  const uint64_t pt = ((per_block + kBlock - 1) / kBlock + 15) / 16 * 16;  // keys per thread, whole 16-key chunks
  const uint64_t blo = (uint64_t)b * per_block;
  const uint64_t bhi = blo + per_block < S ? blo + per_block : S;
  const uint64_t t0 = blo + threadIdx.x * pt;
  const uint64_t t1 = t0 + pt < bhi ? t0 + pt : bhi;
  const uint32_t flip = largest ? 0u : 0xFFFFu;  // keys(i) = v ^ flip = TopkKeys<16>
  uint32_t gt = 0, eq = 0;
  for (uint64_t c0 = t0; c0 < t1; c0 += 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys16(k16, c0, t1, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t key = min(kv[e], R - 1) ^ flip;  // as the histogram bins it
      gt += ((m >> e) & 1u) && key > T;
      eq += ((m >> e) & 1u) && key == T;
    }
  }
  uint32_t bg, be;
  uint32_t og = block_excl_scan_u(gt, lds, bg);
  __syncthreads();
  uint32_t oe = block_excl_scan_u(eq, lds, be);
  if (threadIdx.x == 0 && !counts)
    __hip_atomic_store(&status[b], kLbAgg | ((uint64_t)bg << 31) | (uint64_t)be, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // block prefix = sum of the predecessors' aggregates, read in parallel
  uint32_t pg = 0, pe = 0;
  for (uint32_t j = threadIdx.x; j < b; j += kBlock) {
    if (counts) {
      pg += counts[2 * j];
      pe += counts[2 * j + 1];
      continue;
    }
    uint64_t w = 0;
    for (uint32_t spins = 0; spins < (1u << 26); ++spins) {  // bound: never hang the device
      w = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w) break;
    }
    pg += (uint32_t)((w >> 31) & kLbMask31);
    pe += (uint32_t)(w & kLbMask31);
  }
  auto add = [](uint32_t x, uint32_t y) { return x + y; };
  pg = block_reduce(pg, lds, add);
  pe = block_reduce(pe, lds, add);
  // every other block published its aggregate, hence had read the histogram:
  // the last ticket zeroes it for the next selection
  if (b == nblocks - 1 && !fused && !counts)
    for (uint32_t i = threadIdx.x; i < R; i += kBlock) G[i] = 0;
  uint32_t gpos = pg + og, epos = pe + oe;
  // with a row move, the block's selections are listed in LDS first (slot:
  // gt ones in scan order, then the taken ties) and copied by the whole block
  // afterwards, 16 bytes per lane, rows contiguous: one thread per row was
  // 3x slower than the separate gather / scatter kernels
  const bool move = mv.mode != TopkMove::NONE;
  // SCATTER with best_parts: the best survivor (max key, lowest index: the
  // pack_best order, key == score) and the best immigrant placed here
  const bool bests = mv.mode == TopkMove::SCATTER && mv.best_parts != nullptr;
  unsigned long long keep_best = 0, imm_best = 0;
  uint32_t lg = og, le = bg + oe;
  for (uint64_t c0 = t0; c0 < t1; c0 += 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys16(k16, c0, t1, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (!((m >> e) & 1u)) continue;
      const uint32_t key = min(kv[e], R - 1) ^ flip;
      uint32_t pos = 0xFFFFFFFFu, slot = 0;
      if (key > T && gpos < gt_total) {
        pos = gpos++;
        slot = lg++;
      }
      if (key == T) {
        if (epos < need_eq) {
          pos = gt_total + epos;
          slot = le;
        }
        ++epos;
        ++le;
      }
      if (bests) {
        if (pos == 0xFFFFFFFFu) {
          const unsigned long long kb = ((unsigned long long)min(kv[e], R - 1) << 32) | (0xFFFFFFFFull - (uint32_t)(c0 + e));
          keep_best = kb > keep_best ? kb : keep_best;
        } else {
          const unsigned long long ib = pack_best(mv.src_scores[pos], c0 + e);
          imm_best = ib > imm_best ? ib : imm_best;
        }
      }
      if (pos == 0xFFFFFFFFu) continue;
      if (idx_out) idx_out[pos] = (uint32_t)(c0 + e);
      if (move && slot < kTopkMoveSlots) {
        sel_pos[slot] = pos;
        sel_src[slot] = (uint32_t)(c0 + e - blo);
      } else if (move) {
        topk_emit(mv, nullptr, pos, c0 + e);  // beyond the LDS list (huge blocks): per thread
      }
    }
  }
  if (bests) {  // block-uniform: the block's new packed best
    __shared__ unsigned long long red[kBlock / 64];
    const unsigned long long kb = block_max_u64(keep_best, red);
    const unsigned long long ib = block_max_u64(imm_best, red);
    if (threadIdx.x == 0) {
      unsigned long long pb = ib;
      if (kb) {  // the survivor's own score (key == score for the integer objectives)
        const uint64_t i = 0xFFFFFFFFull - (uint32_t)kb;
        const unsigned long long sb = pack_best(mv.dst_scores[i], i);
        pb = sb > pb ? sb : pb;
      }
      mv.best_parts[b] = pb;
    }
  }
  if (!move) return;
  // slots [0, bg) are gt selections (all taken up to gt_total), [bg, bg+be)
  // ties, of which only those with a global tie rank < need_eq were filled
  __syncthreads();
  const uint32_t taken_eq = pe >= need_eq ? 0u : min(be, need_eq - pe);
  const uint32_t n_gt = pg >= gt_total ? 0u : min(bg, gt_total - pg);
  const uint32_t nsel = min(bg + taken_eq, kTopkMoveSlots);
  const uint32_t rw16 = mv.rw16;
  for (uint32_t t = threadIdx.x; t < nsel * rw16; t += kBlock) {
    const uint32_t r = t / rw16, c = t % rw16;
    if (r >= n_gt && r < bg) continue;  // gt slots beyond gt_total were never filled
    const uint64_t i = blo + sel_src[r];
    const uint64_t pos = sel_pos[r];
    if (mv.mode == TopkMove::GATHER) {
      mv.dst_rows[pos * rw16 + c] = mv.src_rows[i * rw16 + c];
      if (c == 0) mv.dst_scores[pos] = mv.src_scores[i];
    } else {
      mv.dst_rows[i * rw16 + c] = mv.src_rows[pos * rw16 + c];
      if (c == 0) {
        const float v = mv.src_scores[pos];
        mv.dst_scores[i] = v;
        if (mv.dst_keys) mv.dst_keys[i] = (uint16_t)(!(v > 0.f) ? 0.f : (v >= 65535.f ? 65535.f : v));
      }
    }
  }
}

// ---- f32 scores: the exact top-k in selection order from three radix
// digits of the 32-bit orderable keys (11 / 11 / 10 bits) and one ticketed
// select: 4 launches per selection (the 8-bit radix path above takes 11, and
// the gather / scatter / best passes after it 3 more).  Each histogram
// kernel's blocks re-derive the previous digit's threshold from its global
// histogram themselves (block 0 also records it for the next launch), so no
// single-block digit kernels sit between the passes; the select kernel
// derives the last digit, counts, orders (status words, as
// topk16_select_kernel) and moves the rows.  Same result as topk_run: every
// key above the threshold by index, then the first ties by index. ----
constexpr uint32_t kT32R1 = 2048, kT32R2 = 2048, kT32R3 = 1024;  // digit bins: key >> 21, (key >> 10) & 2047, key & 1023
constexpr uint32_t kT32State = kT32R1 + kT32R2 + kT32R3;         // G word offset of {T1, k2, T2, k3}

// 16 keys of [c0, c0 + 16) clipped to end (float4 loads when whole and aligned)
__device__ __forceinline__ uint32_t load_keys32(const float* s, uint64_t c0, uint64_t end, bool largest,
                                                uint32_t (&kv)[16]) {
  if (c0 + 16 <= end && (c0 & 3) == 0) {
    float4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = *(const float4*)(s + c0 + 4 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kv[4 * j] = topk_key(v[j].x, largest);
      kv[4 * j + 1] = topk_key(v[j].y, largest);
      kv[4 * j + 2] = topk_key(v[j].z, largest);
      kv[4 * j + 3] = topk_key(v[j].w, largest);
    }
    return 0xFFFFu;
  }
  uint32_t m = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool ok = c0 + e < end;
    kv[e] = ok ? topk_key(s[c0 + e], largest) : 0u;
    m |= ok ? (1u << e) : 0u;
  }
  return m;
}

// the threshold bin of R (from the top: the bin where the count of keys in
// higher bins first reaches k) and the k left for it; block-wide, every
// thread returns the same.  G: R global counts.
__device__ __forceinline__ void t32_threshold(const uint32_t* G, uint32_t R, uint32_t k, uint32_t* lds,
                                              uint32_t* sh, uint32_t& T, uint32_t& rem) {
  const uint32_t per = R / kBlock;  // 8 or 4
  uint32_t c[8], mine = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    c[j] = j < per ? G[R - 1 - threadIdx.x * per - j] : 0u;
    mine += c[j];
  }
  uint32_t tot;
  const uint32_t before = block_excl_scan_u(mine, lds, tot);
  if (before < k && before + mine >= k) {
    uint32_t acc = before;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      if (j < per && acc < k && acc + c[j] >= k) {
        sh[0] = R - 1 - threadIdx.x * per - j;
        sh[1] = k - acc;
      }
      acc += c[j];
    }
  }
  if (threadIdx.x == 0 && tot < k) {  // k > S cannot happen (the launcher checks); keep bin 0
    sh[0] = 0;
    sh[1] = k;
  }
  __syncthreads();
  T = sh[0];
  rem = sh[1];
}

// histogram of digit `level` (1, 2, 3) over the keys whose higher digits
// match the thresholds found so far; level 1 also zeroes the select's status
// words and tickets
__global__ __launch_bounds__(kBlock) void topk32_hist_kernel(const float* scores, uint64_t S, uint64_t per_block,
                                                             bool largest, uint32_t k, uint32_t level, uint32_t* G,
                                                             uint64_t* status, uint32_t n_status) {
  __shared__ uint32_t h[kT32R1];
  __shared__ uint32_t lds[kBlock / 64], sh[2];
  const uint32_t R = level == 3 ? kT32R3 : kT32R1;
  for (uint32_t i = threadIdx.x; i < R; i += kBlock) h[i] = 0;
  uint32_t pfx = 0, pmask = 0, shift = 21, dmask = kT32R1 - 1;
  if (level == 1) {
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_status; i += gridDim.x * kBlock) status[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2) ((uint32_t*)(status + n_status))[threadIdx.x] = 0;
  } else {
    uint32_t* st = G + kT32State;
    uint32_t T1, k2;
    if (level == 2) {
      t32_threshold(G, kT32R1, k, lds, sh, T1, k2);
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st[0] = T1;
        st[1] = k2;
      }
      pfx = T1 << 21;
      pmask = 0xFFE00000u;
      shift = 10;
    } else {
      T1 = st[0];
      k2 = st[1];
      uint32_t T2, k3;
      t32_threshold(G + kT32R1, kT32R2, k2, lds, sh, T2, k3);
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st[2] = T2;
        st[3] = k3;
      }
      pfx = (T1 << 21) | (T2 << 10);
      pmask = 0xFFFFFC00u;
      shift = 0;
      dmask = kT32R3 - 1;
    }
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint64_t pt = ((per_block + kBlock - 1) / kBlock + 15) / 16 * 16;
  const uint64_t blo = (uint64_t)blockIdx.x * per_block;
  const uint64_t bhi = blo + per_block < S ? blo + per_block : S;
  const uint64_t t0 = blo + threadIdx.x * pt, t1 = t0 + pt < bhi ? t0 + pt : bhi;
  // trip count uniform across the wave (per-thread ranges of equal length)
  for (uint64_t c0 = blo + threadIdx.x * pt, n = 0; n < pt; c0 += 16, n += 16) {
    uint32_t kv[16];
    const uint32_t m = c0 < t1 ? load_keys32(scores, c0, t1, largest, kv) : 0u;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const bool act = ((m >> e) & 1u) && (kv[e] & pmask) == pfx;
      const uint32_t bin = (kv[e] >> shift) & dmask;
      // a converging population shares its high digits: one atomic when the
      // wave agrees on one bin, else per-lane LDS atomics
      const unsigned long long active = __ballot(act);
      if (active) {
        const int leader = __ffsll((long long)active) - 1;
        const uint32_t b = (uint32_t)__shfl((int)bin, leader, 64);
        const unsigned long long same = __ballot(act && bin == b);
        if (same == active) {
          if ((int)lane == leader) atomicAdd(&h[b], (uint32_t)__popcll(same));
        } else if (act) {
          atomicAdd(&h[bin], 1u);
        }
      }
    }
  }
  __syncthreads();
  uint32_t* Gl = G + (level == 1 ? 0u : (level == 2 ? kT32R1 : kT32R1 + kT32R2));
  for (uint32_t i = threadIdx.x; i < R; i += kBlock)
    if (h[i]) atomicAdd(&Gl[i], h[i]);
}

// the select: threshold key T from the three digits, per-thread (gt, eq)
// counts over a contiguous range, block order by status words (every
// predecessor by ticket publishes without waiting), then the ordered write
// with the row moves; SCATTER also writes the block's packed best (the best
// survivor, key -> score exactly, or the best immigrant placed here)
__global__ __launch_bounds__(kBlock) void topk32_select_kernel(const float* scores, uint64_t S, uint64_t per_block,
                                                               bool largest, uint32_t k, uint32_t* G,
                                                               uint64_t* status, uint32_t* ctr, uint32_t nblocks,
                                                               uint32_t* idx_out, TopkMove mv) {
  __shared__ uint32_t sel_pos[kTopkMoveSlots], sel_src[kTopkMoveSlots];
  __shared__ uint32_t lds[kBlock / 64], sh[2], sh_b;
  if (threadIdx.x == 0) sh_b = atomicAdd(&ctr[0], 1u);
  const uint32_t* st = G + kT32State;
  const uint32_t T1 = st[0], T2 = st[2], k3 = st[3];
  uint32_t T3, need_eq;
  t32_threshold(G + kT32R1 + kT32R2, kT32R3, k3, lds, sh, T3, need_eq);  // (its barrier publishes sh_b)
  const uint32_t T = (T1 << 21) | (T2 << 10) | T3;
  const uint32_t gt_total = k - need_eq;  // every key above T
  const uint32_t b = sh_b;
  // G1 / G2 are read by no block of this launch: zeroed here for the next
  // selection (a slice per block); G3 and the state by the last ticket
  for (uint32_t i = b * kBlock + threadIdx.x; i < kT32R1 + kT32R2; i += nblocks * kBlock) G[i] = 0;
  const uint64_t pt = ((per_block + kBlock - 1) / kBlock + 15) / 16 * 16;  // keys per thread, whole 16-key chunks
  const uint64_t blo = (uint64_t)b * per_block;
  const uint64_t bhi = blo + per_block < S ? blo + per_block : S;
  const uint64_t t0 = blo + threadIdx.x * pt;
  const uint64_t t1 = t0 + pt < bhi ? t0 + pt : bhi;
  uint32_t gt = 0, eq = 0;
  for (uint64_t c0 = t0; c0 < t1; c0 += 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys32(scores, c0, t1, largest, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      gt += ((m >> e) & 1u) && kv[e] > T;
      eq += ((m >> e) & 1u) && kv[e] == T;
    }
  }
  uint32_t bg, be;
  uint32_t og = block_excl_scan_u(gt, lds, bg);
  __syncthreads();
  uint32_t oe = block_excl_scan_u(eq, lds, be);
  if (threadIdx.x == 0)
    __hip_atomic_store(&status[b], kLbAgg | ((uint64_t)bg << 31) | (uint64_t)be, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // block prefix = sum of the predecessors' aggregates, read in parallel
  uint32_t pg = 0, pe = 0;
  for (uint32_t j = threadIdx.x; j < b; j += kBlock) {
    uint64_t w = 0;
    for (uint32_t spins = 0; spins < (1u << 26); ++spins) {  // bound: never hang the device
      w = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w) break;
    }
    pg += (uint32_t)((w >> 31) & kLbMask31);
    pe += (uint32_t)(w & kLbMask31);
  }
  auto add = [](uint32_t x, uint32_t y) { return x + y; };
  pg = block_reduce(pg, lds, add);
  pe = block_reduce(pe, lds, add);
  // every other block published, hence had read G3 and the state: the last
  // ticket zeroes them for the next selection
  if (b == nblocks - 1)
    for (uint32_t i = threadIdx.x; i < kT32R3 + 4; i += kBlock) G[kT32R1 + kT32R2 + i] = 0;
  uint32_t gpos = pg + og, epos = pe + oe;
  const bool move = mv.mode != TopkMove::NONE;
  const bool bests = mv.mode == TopkMove::SCATTER && mv.best_parts != nullptr;
  unsigned long long keep_best = 0, imm_best = 0;
  uint32_t lg = og, le = bg + oe;
  for (uint64_t c0 = t0; c0 < t1; c0 += 16) {
    uint32_t kv[16];
    const uint32_t m = load_keys32(scores, c0, t1, largest, kv);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (!((m >> e) & 1u)) continue;
      uint32_t pos = 0xFFFFFFFFu, slot = 0;
      if (kv[e] > T && gpos < gt_total) {
        pos = gpos++;
        slot = lg++;
      }
      if (kv[e] == T) {
        if (epos < need_eq) {
          pos = gt_total + epos;
          slot = le;
        }
        ++epos;
        ++le;
      }
      if (bests) {
        if (pos == 0xFFFFFFFFu) {  // a survivor: its own score, exactly, from the key
          const float v = key_score(largest ? kv[e] : ~kv[e]);
          const unsigned long long kb = pack_best(v, c0 + e);
          keep_best = kb > keep_best ? kb : keep_best;
        } else {
          const unsigned long long ib = pack_best(mv.src_scores[pos], c0 + e);
          imm_best = ib > imm_best ? ib : imm_best;
        }
      }
      if (pos == 0xFFFFFFFFu) continue;
      if (idx_out) idx_out[pos] = (uint32_t)(c0 + e);
      if (move && slot < kTopkMoveSlots) {
        sel_pos[slot] = pos;
        sel_src[slot] = (uint32_t)(c0 + e - blo);
      } else if (move) {
        topk_emit(mv, nullptr, pos, c0 + e);  // beyond the LDS list (huge blocks): per thread
      }
    }
  }
  if (bests) {  // block-uniform: the block's new packed best
    __shared__ unsigned long long red[kBlock / 64];
    const unsigned long long kb = block_max_u64(keep_best, red);
    const unsigned long long ib = block_max_u64(imm_best, red);
    if (threadIdx.x == 0) mv.best_parts[b] = kb > ib ? kb : ib;
  }
  if (!move) return;
  // slots [0, bg): keys above T (those with a global rank < gt_total were
  // taken), [bg, bg + be): ties, of which those with a tie rank < need_eq
  __syncthreads();
  const uint32_t taken_eq = pe >= need_eq ? 0u : min(be, need_eq - pe);
  const uint32_t n_gt = pg >= gt_total ? 0u : min(bg, gt_total - pg);
  const uint32_t nsel = min(bg + taken_eq, kTopkMoveSlots);
  const uint32_t rw16 = mv.rw16;
  for (uint32_t t = threadIdx.x; t < nsel * rw16; t += kBlock) {
    const uint32_t r = t / rw16, c = t % rw16;
    if (r >= n_gt && r < bg) continue;
    const uint64_t i = blo + sel_src[r];
    const uint64_t pos = sel_pos[r];
    if (mv.mode == TopkMove::GATHER) {
      mv.dst_rows[pos * rw16 + c] = mv.src_rows[i * rw16 + c];
      if (c == 0) mv.dst_scores[pos] = mv.src_scores[i];
    } else {
      mv.dst_rows[i * rw16 + c] = mv.src_rows[pos * rw16 + c];
      if (c == 0) mv.dst_scores[i] = mv.src_scores[pos];
    }
  }
}

template <int BITS>
__global__ __launch_bounds__(kBlock) void topk_write_kernel(TopkKeys<BITS> keys, uint64_t S, uint64_t per_block,
                                                            const TopkState* st, const uint32_t* cnt, uint32_t nblocks,
                                                            uint32_t* keys_out, uint32_t* idx_out) {
  __shared__ uint32_t lds[kBlock / 64];
  const uint32_t T = st->prefix;
  const uint32_t need_eq = st->remaining;
  const uint32_t gt_total = cnt[2 * nblocks];
  uint32_t gpos = cnt[2 * blockIdx.x], epos = cnt[2 * blockIdx.x + 1];
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block;
  const uint64_t b1 = b0 + per_block < S ? b0 + per_block : S;
  for (uint64_t t0 = b0; t0 < b1; t0 += kBlock) {
    uint64_t i = t0 + threadIdx.x;
    uint32_t key = i < b1 ? keys(i) : 0u;
    uint32_t isg = (i < b1 && key > T) ? 1u : 0u;
    uint32_t ise = (i < b1 && key == T) ? 1u : 0u;
    uint32_t tg, te;
    uint32_t rg = block_excl_scan_u(isg, lds, tg);
    __syncthreads();
    uint32_t re = block_excl_scan_u(ise, lds, te);
    if (isg && gpos + rg < gt_total) {
      if (keys_out) keys_out[gpos + rg] = key;
      idx_out[gpos + rg] = (uint32_t)i;
    }
    if (ise && epos + re < need_eq) {
      if (keys_out) keys_out[gt_total + epos + re] = key;
      idx_out[gt_total + epos + re] = (uint32_t)i;
    }
    gpos += tg;
    epos += te;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void gather_rows_kernel(const uint4* rows, const float* scores, uint32_t rw16,
                                                             const uint32_t* idx, uint32_t n, uint4* out,
                                                             float* out_scores) {
  const uint64_t total = (uint64_t)n * rw16;
  for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
    uint64_t r = t / rw16, c = t % rw16;
    uint64_t src = idx[r];
    out[t] = rows[src * rw16 + c];
    if (c == 0 && scores && out_scores) out_scores[r] = scores[src];
  }
}

__global__ __launch_bounds__(kBlock) void scatter_rows_kernel(uint4* rows, float* scores, uint32_t rw16,
                                                              const uint32_t* idx, uint32_t n, const uint4* in,
                                                              const float* in_scores) {
  const uint64_t total = (uint64_t)n * rw16;
  for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
    uint64_t r = t / rw16, c = t % rw16;
    uint64_t dst = idx[r];
    rows[dst * rw16 + c] = in[t];
    if (c == 0 && scores && in_scores) scores[dst] = in_scores[r];
  }
}

// ---- MIG_STRIPE migration: one wave per stripe (grid-stride over stripes) ----
__device__ __forceinline__ uint16_t score_to_key16(float v) {
  return (uint16_t)(!(v > 0.f) ? 0.f : (v >= 65535.f ? 65535.f : v));
}

// 16 lanes per stripe (4 stripes per wave): at 1% of 1M the k = 10486 stripes
// of ~100 individuals are 2622 waves, all resident at once, each lane loading
// its ~7 scores in one burst
constexpr uint32_t kStripeLanes = 16;
constexpr uint32_t kStripeCache = 8;  // scores per lane kept in registers (stripes <= 128)

__global__ __launch_bounds__(kBlock) void stripe_emigrate_kernel(const float* __restrict__ scores,
                                                                 const uint4* __restrict__ rows, uint32_t rw16,
                                                                 uint64_t S, uint32_t k, uint4* __restrict__ out,
                                                                 float* __restrict__ out_scores) {
  const uint32_t sl = threadIdx.x & (kStripeLanes - 1);
  const uint32_t ng = gridDim.x * (kBlock / kStripeLanes);
  for (uint32_t i = (blockIdx.x * kBlock + threadIdx.x) / kStripeLanes; i < k; i += ng) {  // group-uniform
    const uint64_t lo = (uint64_t)i * S / k, hi = (uint64_t)(i + 1) * S / k;
    unsigned long long b = 0;
    for (uint64_t j = lo + sl; j < hi; j += kStripeLanes) {
      const unsigned long long p = pack_best(scores[j], j);
      b = p > b ? p : b;
    }
#pragma unroll
    for (int o = kStripeLanes / 2; o > 0; o >>= 1) {
      const unsigned long long x = shfl_xor_u64(b, o);
      b = x > b ? x : b;
    }
    const uint64_t src = best_index(b);
    for (uint32_t c = sl; c < rw16; c += kStripeLanes) out[(uint64_t)i * rw16 + c] = rows[src * rw16 + c];
    if (sl == 0) out_scores[i] = best_score(b);
  }
}

__global__ __launch_bounds__(kBlock) void stripe_immigrate_kernel(float* __restrict__ scores, uint16_t* keys,
                                                                  uint4* __restrict__ rows, uint32_t rw16, uint64_t S,
                                                                  uint32_t k, const uint4* __restrict__ in,
                                                                  const float* __restrict__ in_scores,
                                                                  unsigned long long* best_parts, float* stats_parts) {
  __shared__ unsigned long long lds_red[kBlock / 64];
  const uint32_t sl = threadIdx.x & (kStripeLanes - 1);
  const uint32_t ng = gridDim.x * (kBlock / kStripeLanes);
  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint32_t i = (blockIdx.x * kBlock + threadIdx.x) / kStripeLanes; i < k; i += ng) {  // group-uniform
    const uint64_t lo = (uint64_t)i * S / k, hi = (uint64_t)(i + 1) * S / k;
    const bool cached = hi - lo <= (uint64_t)kStripeLanes * kStripeCache;  // group-uniform
    // the immigrant (independent of the victim: issued with the score loads)
    const float sin = in_scores[i];
    const uint4 r0 = sl < rw16 ? in[(uint64_t)i * rw16 + sl] : make_uint4(0, 0, 0, 0);
    float v[kStripeCache];
    unsigned long long w = ~0ull;  // min of (score key << 32 | index): the worst, lowest index
#pragma unroll
    for (uint32_t t = 0; t < kStripeCache; ++t) {
      const uint64_t j = lo + sl + (uint64_t)t * kStripeLanes;
      v[t] = (cached && j < hi) ? scores[j] : 0.f;
      const unsigned long long p = ((unsigned long long)score_key(v[t]) << 32) | j;
      w = (cached && j < hi && p < w) ? p : w;
    }
    if (!cached)
      for (uint64_t j = lo + sl; j < hi; j += kStripeLanes) {
        const unsigned long long p = ((unsigned long long)score_key(scores[j]) << 32) | j;
        w = p < w ? p : w;
      }
#pragma unroll
    for (int o = kStripeLanes / 2; o > 0; o >>= 1) {
      const unsigned long long x = shfl_xor_u64(w, o);
      w = x < w ? x : w;
    }
    const uint64_t dst = (uint32_t)w;
    if (sl < rw16) rows[dst * rw16 + sl] = r0;
    for (uint32_t c = sl + kStripeLanes; c < rw16; c += kStripeLanes) rows[dst * rw16 + c] = in[(uint64_t)i * rw16 + c];
    if (sl == 0) {
      scores[dst] = sin;
      if (keys) keys[dst] = score_to_key16(sin);
    }
    // the stripe after the replacement: best partial and statistics
    if (cached) {
#pragma unroll
      for (uint32_t t = 0; t < kStripeCache; ++t) {
        const uint64_t j = lo + sl + (uint64_t)t * kStripeLanes;
        if (j < hi) {
          const float x = j == dst ? sin : v[t];
          const unsigned long long p = pack_best(x, j);
          my_best = p > my_best ? p : my_best;
          st.add(x);
        }
      }
    } else {
      for (uint64_t j = lo + sl; j < hi; j += kStripeLanes) {
        const float x = j == dst ? sin : scores[j];
        const unsigned long long p = pack_best(x, j);
        my_best = p > my_best ? p : my_best;
        st.add(x);
      }
    }
  }
  const unsigned long long b = block_max_u64(my_best, lds_red);
  if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
  if (stats_parts) block_stats_store(st, stats_parts);
}

__global__ __launch_bounds__(kBlock) void scores_to_keys_kernel(const float* s, uint64_t S, uint16_t* k) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < S; i += (uint64_t)gridDim.x * kBlock) {
    const float v = s[i];
    k[i] = (uint16_t)(!(v > 0.f) ? 0.f : (v >= 65535.f ? 65535.f : v));
  }
}

__global__ __launch_bounds__(kBlock) void scores_to_qkeys_kernel(const float* s, uint64_t S, const float* mm,
                                                                  uint16_t* k) {
  float lo, scale;
  qkey_params(mm[0], mm[1], lo, scale);
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < S; i += (uint64_t)gridDim.x * kBlock)
    k[i] = (uint16_t)qkey(s[i], lo, scale);
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

__global__ void advance_counter_kernel(uint32_t* c, uint32_t d) {
  if (threadIdx.x == 0) *c += d;
}

}  // namespace

void advance_counter_launch(uint32_t* counter, uint32_t delta, hipStream_t s) {
  hipLaunchKernelGGL(advance_counter_kernel, 1, 64, 0, s, counter, delta);
  PGA_HIP_CHECK(hipGetLastError());
}

void reduce_best_launch(const unsigned long long* parts, uint32_t n, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_best_kernel, 1, kBlock, 0, s, parts, n, out);
  PGA_HIP_CHECK(hipGetLastError());
}

uint32_t best_of_scores_launch(const float* scores, uint64_t S, unsigned long long* parts, hipStream_t s,
                               uint16_t* keys) {
  uint32_t grid = launch_grid(S, kBlock * 4);
  hipLaunchKernelGGL(best_of_scores_kernel, grid, kBlock, 0, s, scores, S, parts, keys);
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

void scores_to_keys_launch(const float* scores, uint64_t S, uint16_t* keys, hipStream_t s) {
  uint32_t grid = launch_grid(S, kBlock * 4);
  hipLaunchKernelGGL(scores_to_keys_kernel, grid, kBlock, 0, s, scores, S, keys);
  PGA_HIP_CHECK(hipGetLastError());
}

void scores_to_qkeys_launch(const float* scores, uint64_t S, const float* mm, uint16_t* keys, hipStream_t s) {
  uint32_t grid = launch_grid(S, kBlock * 4);
  hipLaunchKernelGGL(scores_to_qkeys_kernel, grid, kBlock, 0, s, scores, S, mm, keys);
  PGA_HIP_CHECK(hipGetLastError());
}

// {min, max, sum, count} of a generation from the fused partials its kernel
// stored: {min, sum} pairs (GenArgs::stats_parts) and packed bests (the max)
__global__ __launch_bounds__(kBlock) void stats_from_parts_kernel(const float* parts, const unsigned long long* best,
                                                                 uint32_t n, uint64_t S, float* out) {
  __shared__ float lds[kBlock / 64];
  __shared__ unsigned long long lds_b[kBlock / 64];
  float mn = INFINITY, sm = 0.f;
  unsigned long long b = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
    mn = fminf(mn, parts[2 * i]);
    sm += parts[2 * i + 1];
    b = best[i] > b ? best[i] : b;
  }
  mn = block_reduce(mn, lds, FMin());
  sm = block_reduce(sm, lds, FAdd());
  b = block_max_u64(b, lds_b);
  if (threadIdx.x == 0) {
    out[0] = mn;
    out[1] = best_score(b);
    out[2] = sm;
    out[3] = (float)S;
  }
}

void stats_from_parts_launch(const float* parts, const unsigned long long* best, uint32_t n, uint64_t S, float* out,
                             hipStream_t s) {
  hipLaunchKernelGGL(stats_from_parts_kernel, 1, kBlock, 0, s, parts, best, n, S, out);
  PGA_HIP_CHECK(hipGetLastError());
}

void score_stats_launch(const float* scores, uint64_t S, float* stats, hipStream_t s) {
  // stats buffer layout: [0..4) result, [4..) 3*grid partials
  uint32_t grid = launch_grid(S, kBlock * 4);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(stats_part_kernel, grid, kBlock, 0, s, scores, S, stats + 4);
  hipLaunchKernelGGL(stats_final_kernel, 1, kBlock, 0, s, stats + 4, grid, S, stats);
  PGA_HIP_CHECK(hipGetLastError());
}

size_t roulette_workspace_floats(uint64_t S) {
  // stats | stats partials | block sums | scale, pad | u64 block sums (integer objectives)
  (void)S;
  return kRoulScale + 4 + 2 * 1024;
}

void roulette_prefix_launch(const float* scores, uint64_t S, const float* parts, uint32_t nparts, float* cumfit,
                            float* ws, hipStream_t s, bool integer) {
  // ws layout: [0..4) stats, [4 .. 4+3*1024) stats partials, then block sums, then [kRoulScale] the guide scale
  if (!parts) score_stats_launch(scores, S, ws, s);
  uint32_t grid = launch_grid(S, kBlock * 4);
  if (grid > 1024) grid = 1024;
  const uint64_t per_block = (S + grid - 1) / grid;
  float* block_sums = ws + 4 + 3 * 1024;
  if (integer) {
    unsigned long long* sums64 = (unsigned long long*)(ws + kRoulScale + 4);
    hipLaunchKernelGGL(prefix_part_int_kernel, grid, kBlock, 0, s, scores, S, per_block, parts, nparts, ws, sums64);
    hipLaunchKernelGGL(prefix_final_int_kernel, grid, kBlock, 0, s, scores, S, per_block, ws,
                       (const unsigned long long*)sums64, cumfit, ws + kRoulScale);
  } else {
    hipLaunchKernelGGL(prefix_part_kernel, grid, kBlock, 0, s, scores, S, per_block, parts, nparts, ws, block_sums);
    hipLaunchKernelGGL(prefix_final_kernel, grid, kBlock, 0, s, scores, S, per_block, ws, block_sums, cumfit,
                       ws + kRoulScale);
  }
  PGA_HIP_CHECK(hipGetLastError());
}

// the guide's covered flag (tp.hpp reads it only while S < 2^31);
// PGA_ROUL_COVER=0 leaves it out (A/B knob)
static uint32_t guide_cover_flag(uint64_t S) {
  static const bool off = [] {
    const char* e = std::getenv("PGA_ROUL_COVER");
    return e && e[0] == '0';
  }();
  return !off && S <= kGuideIndexMask ? kGuideCovered : 0u;
}

bool roulette_fused_launch(const float* scores, uint64_t S, const float* parts, const TpPartition& part,
                           uint32_t max_score, float* cumfit, uint32_t* guide, float* ws, hipStream_t s, bool packed) {
  if (!parts || part.grid == 0 || part.unit == 0 || S == 0 || S > 0xFFFFFFFFull) return false;
  // the largest share (tp_share: ceil(S / grid) in whole units, plus the skew)
  // times the largest score stays below 2^24, so every f32 partial sum is exact
  const uint64_t per = ((S + part.grid - 1) / part.grid + part.unit - 1) / part.unit * part.unit;
  const uint64_t share = per + (uint64_t)part.skew * part.unit;
  if (share * (uint64_t)max_score >= (1ull << 24)) return false;
  // a chunk's u32 weight sum: kRoulThreads * kRoulPer * max_score < 2^32
  if ((uint64_t)kRoulThreads * kRoulPer * max_score >= (1ull << 32)) return false;
  hipLaunchKernelGGL(roulette_fused_kernel, part.grid, kRoulThreads, 0, s, scores, S, parts, part.unit, part.skew, cumfit,
                     guide, ws + kRoulScale, guide_cover_flag(S), packed ? 1u : 0u);
  PGA_HIP_CHECK(hipGetLastError());
  return true;
}

void roulette_guide_launch(const float* cumfit, uint64_t S, uint32_t* guide, float* ws, hipStream_t s, bool packed) {
  const uint32_t grid = launch_grid(S, kBlock);
  hipLaunchKernelGGL(roulette_guide_kernel, grid, kBlock, 0, s, cumfit, S, (const float*)(ws + kRoulScale), guide,
                     guide_cover_flag(S), packed ? 1u : 0u);
  PGA_HIP_CHECK(hipGetLastError());
}

size_t topk_workspace_bytes(uint64_t S, uint32_t k) {
  (void)S;
  // layout: state | counts | 3 k-arrays | radix-sort workspace (sorted mode) | value histogram (kept zeroed)
  return align_up(sizeof(TopkState)) + align_up(sizeof(uint32_t) * (2 * 1024 + 4)) + 3 * align_up(4ull * k) +
         align_up(radix_sort_workspace_bytes(k)) + align_up(4ull * kTopkMaxRange);
}

namespace {
template <int BITS>
void topk_run(TopkKeys<BITS> keys, uint64_t S, uint32_t k, bool sorted, uint32_t* idx_out, void* ws, hipStream_t s) {
  char* p = (char*)ws;
  TopkState* st = (TopkState*)p;
  p += align_up(sizeof(TopkState));
  uint32_t* cnt = (uint32_t*)p;
  p += align_up(sizeof(uint32_t) * (2 * 1024 + 4));
  uint32_t* keys_buf = (uint32_t*)p;
  p += align_up(4ull * k);
  uint32_t* keys_sorted = (uint32_t*)p;
  p += align_up(4ull * k);
  uint32_t* idx = (uint32_t*)p;
  p += align_up(4ull * k);

  const uint32_t grid = launch_grid(S, kBlock * 4);
  hipLaunchKernelGGL(topk_init_kernel, 1, kBlock, 0, s, st, k);
  for (int d = 0; d < BITS / 8; ++d) {
    const uint32_t shift = BITS - 8 - 8 * d;
    hipLaunchKernelGGL(topk_hist_kernel<BITS>, grid, kBlock, 0, s, keys, S, shift, st);
    hipLaunchKernelGGL(topk_digit_kernel, 1, kBlock, 0, s, st, shift);
  }
  const uint32_t cgrid = grid > 1024 ? 1024 : grid;
  const uint64_t per_block = (S + cgrid - 1) / cgrid;
  hipLaunchKernelGGL(topk_count_kernel<BITS>, cgrid, kBlock, 0, s, keys, S, per_block, st, cnt);
  hipLaunchKernelGGL(topk_offsets_kernel, 1, kBlock, 0, s, cnt, cgrid, (uint32_t*)nullptr, 0u);
  if (!sorted) {
    // selection order: every key above the threshold by index, then the
    // threshold ties by index — what the CPU backend's unsorted mode returns
    hipLaunchKernelGGL(topk_write_kernel<BITS>, cgrid, kBlock, 0, s, keys, S, per_block, st, cnt, cgrid,
                       (uint32_t*)nullptr, idx_out);
    PGA_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(topk_write_kernel<BITS>, cgrid, kBlock, 0, s, keys, S, per_block, st, cnt, cgrid, keys_buf, idx);
  PGA_HIP_CHECK(hipGetLastError());
  // stable descending sort (sort.hip) keeps equal keys in ascending index order
  radix_sort_pairs(keys_buf, idx, k, BITS, true, keys_sorted, idx_out, p, s);
}
}  // namespace

bool topk_move_supported(const uint16_t* keys16, uint32_t key_range, uint64_t S) {
  // u16 keys: the value-histogram select; f32 scores: the 3-digit radix select
  return (!keys16 || (key_range >= 2 && key_range <= kTopkMaxRange)) && S < (1ull << 31);
}

// keys per thread of the selection-order kernels (their grid: S / (256 kpt)
// blocks, at most 1024); PGA_TOPK_KPT overrides (16, 32, 64 or 128)
static uint32_t topk_kpt() {
  static const uint32_t v = [] {
    const char* e = std::getenv("PGA_TOPK_KPT");
    const uint32_t x = e ? (uint32_t)std::strtoul(e, nullptr, 10) : 16u;
    return (x == 16 || x == 32 || x == 64 || x == 128) ? x : 16u;
  }();
  return v;
}

uint32_t topk_launch(const float* scores, const uint16_t* keys16, uint32_t key_range, uint64_t S, uint32_t k,
                     bool largest, bool sorted, uint32_t* idx_out, void* ws, hipStream_t s, const TopkMove* mv,
                     const TopkFused* fused) {
  if (k == 0) return 0;
  if (k > S) throw std::runtime_error("topk: k > S");
  if (mv && (sorted || !topk_move_supported(keys16, key_range, S)))
    throw std::invalid_argument("topk: fused row moves need the u16-key selection-order path");
  if (keys16 && !sorted && key_range >= 2 && key_range <= kTopkMaxRange) {
    // integer objective, selection order: histogram over the R key values
    char* p = (char*)ws;
    TopkState* st = (TopkState*)p;
    p += align_up(sizeof(TopkState));
    uint32_t* cnt = (uint32_t*)p;
    p += align_up(sizeof(uint32_t) * (2 * 1024 + 4));
    p += 3 * align_up(4ull * k);
    p += align_up(radix_sort_workspace_bytes(k));
    uint32_t* G = (uint32_t*)p;  // zero on allocation and after every use
    const uint32_t R = key_range;
    uint32_t grid = launch_grid(S, kBlock * topk_kpt());
    const uint32_t cgrid = grid > 1024 ? 1024 : grid;
    const uint64_t per_block = (S + cgrid - 1) / cgrid;
    uint64_t* status = (uint64_t*)cnt;  // cgrid aggregate words, then 2 ticket counters
    if (S < (1ull << 31)) {  // histogram + ticketed select; 4-kernel path beyond
      const uint64_t pb16 = (per_block + 15) / 16 * 16;  // aligned 16-key chunks for every thread
      if (fused && fused->hist && fused->status) {
        // the generation kernel's histogram of these keys, its status words
        // zeroed by that kernel: the select alone (one pass over the keys)
        uint64_t* fst = (uint64_t*)fused->status;
        // PGA_TOPK_2PASS=1 (A/B): a count launch, then the select reads the
        // complete counts instead of publishing and polling status words
        static const bool two = std::getenv("PGA_TOPK_2PASS") && std::getenv("PGA_TOPK_2PASS")[0] == '1';
        uint32_t* counts = two ? (uint32_t*)fused->status : nullptr;  // 2 words per block <= kTopkStatusWords
        if (two)
          hipLaunchKernelGGL(topk16_count2_kernel, cgrid, kBlock, 0, s, keys16, S, pb16, R, largest, k,
                             fused->hist, counts);
        hipLaunchKernelGGL(topk16_select_kernel, cgrid, kBlock, 0, s, keys16, S, pb16, R, largest, k,
                           const_cast<uint32_t*>(fused->hist), fst, (uint32_t*)(fst + cgrid), cgrid, idx_out,
                           mv ? *mv : TopkMove{}, true, (const uint32_t*)counts);
        PGA_HIP_CHECK(hipGetLastError());
        return mv && mv->mode == TopkMove::SCATTER && mv->best_parts ? cgrid : 0u;
      }
      hipLaunchKernelGGL(topk16_hist_kernel, grid, kBlock, 4 * R, s, keys16, S, R, largest, G, status, cgrid);
      hipLaunchKernelGGL(topk16_select_kernel, cgrid, kBlock, 0, s, keys16, S, pb16, R, largest, k, G, status,
                         (uint32_t*)(status + cgrid), cgrid, idx_out, mv ? *mv : TopkMove{}, false);
      PGA_HIP_CHECK(hipGetLastError());
      return mv && mv->mode == TopkMove::SCATTER && mv->best_parts ? cgrid : 0u;
    }
    hipLaunchKernelGGL(topk16_hist_kernel, grid, kBlock, 4 * R, s, keys16, S, R, largest, G, (uint64_t*)nullptr, 0u);
    hipLaunchKernelGGL(topk16_count_kernel, cgrid, kBlock, 0, s, keys16, S, per_block, R, largest, k, G, st, cnt);
    hipLaunchKernelGGL(topk_offsets_kernel, 1, kBlock, 0, s, cnt, cgrid, G, R);
    hipLaunchKernelGGL(topk_write_kernel<16>, cgrid, kBlock, 0, s, TopkKeys<16>{scores, keys16, largest, R - 1}, S,
                       per_block, st, cnt, cgrid, (uint32_t*)nullptr, idx_out);
    PGA_HIP_CHECK(hipGetLastError());
    return 0;
  }
  if (!keys16 && !sorted && S < (1ull << 31)) {
    // f32 scores, selection order: 3 radix digits + the ticketed select (topk32_*)
    char* p = (char*)ws;
    p += align_up(sizeof(TopkState));
    uint64_t* status = (uint64_t*)p;  // cgrid aggregate words, then 2 ticket counters
    p += align_up(sizeof(uint32_t) * (2 * 1024 + 4));
    p += 3 * align_up(4ull * k);
    p += align_up(radix_sort_workspace_bytes(k));
    uint32_t* G = (uint32_t*)p;  // digit histograms + state: zero on allocation and after every use
    static_assert(kT32State + 4 <= kTopkMaxRange, "f32 selection histograms fit the value-histogram region");
    const uint32_t grid = launch_grid(S, kBlock * topk_kpt());
    const uint32_t cgrid = grid > 1024 ? 1024 : grid;
    const uint64_t per_block = ((S + cgrid - 1) / cgrid + 15) / 16 * 16;  // whole 16-key chunks per thread
    for (uint32_t level = 1; level <= 3; ++level)
      hipLaunchKernelGGL(topk32_hist_kernel, cgrid, kBlock, 0, s, scores, S, per_block, largest, k, level, G, status,
                         cgrid);
    hipLaunchKernelGGL(topk32_select_kernel, cgrid, kBlock, 0, s, scores, S, per_block, largest, k, G, status,
                       (uint32_t*)(status + cgrid), cgrid, idx_out, mv ? *mv : TopkMove{});
    PGA_HIP_CHECK(hipGetLastError());
    return mv && mv->mode == TopkMove::SCATTER && mv->best_parts ? cgrid : 0u;
  }
  if (keys16)
    topk_run<16>(TopkKeys<16>{scores, keys16, largest}, S, k, sorted, idx_out, ws, s);
  else
    topk_run<32>(TopkKeys<32>{scores, keys16, largest}, S, k, sorted, idx_out, ws, s);
  return 0;
}

void gather_rows_launch(const void* rows, const float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                        void* out_rows, float* out_scores, hipStream_t s) {
  if (n == 0) return;
  const uint32_t rw16 = row_words / 4;
  uint32_t grid = launch_grid((uint64_t)n * rw16, kBlock);
  hipLaunchKernelGGL(gather_rows_kernel, grid, kBlock, 0, s, (const uint4*)rows, scores, rw16, idx, n,
                     (uint4*)out_rows, out_scores);
  PGA_HIP_CHECK(hipGetLastError());
}

void stripe_emigrate_launch(const float* scores, const void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                            void* out_rows, float* out_scores, hipStream_t s) {
  if (k == 0) return;
  if (k > S) throw std::invalid_argument("stripe migration: k exceeds the population");
  uint64_t grid = ((uint64_t)k + kBlock / kStripeLanes - 1) / (kBlock / kStripeLanes);
  if (grid > kMaxGrid) grid = kMaxGrid;
  hipLaunchKernelGGL(stripe_emigrate_kernel, (uint32_t)grid, kBlock, 0, s, scores, (const uint4*)rows, row_words / 4,
                     S, k, (uint4*)out_rows, out_scores);
  PGA_HIP_CHECK(hipGetLastError());
}

uint32_t stripe_immigrate_launch(float* scores, uint16_t* keys, void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                                 const void* in_rows, const float* in_scores, unsigned long long* best_parts,
                                 float* stats_parts, hipStream_t s) {
  if (k == 0 || k > S) throw std::invalid_argument("stripe migration: k must be in [1, S]");
  uint64_t grid = ((uint64_t)k + kBlock / kStripeLanes - 1) / (kBlock / kStripeLanes);
  if (grid > kMaxGrid) grid = kMaxGrid;
  hipLaunchKernelGGL(stripe_immigrate_kernel, (uint32_t)grid, kBlock, 0, s, scores, keys, (uint4*)rows, row_words / 4,
                     S, k, (const uint4*)in_rows, in_scores, best_parts, stats_parts);
  PGA_HIP_CHECK(hipGetLastError());
  return (uint32_t)grid;
}

void scatter_rows_launch(void* rows, float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                         const void* in_rows, const float* in_scores, hipStream_t s) {
  if (n == 0) return;
  const uint32_t rw16 = row_words / 4;
  uint32_t grid = launch_grid((uint64_t)n * rw16, kBlock);
  hipLaunchKernelGGL(scatter_rows_kernel, grid, kBlock, 0, s, (uint4*)rows, scores, rw16, idx, n,
                     (const uint4*)in_rows, in_scores);
  PGA_HIP_CHECK(hipGetLastError());
}

}  // namespace pga
