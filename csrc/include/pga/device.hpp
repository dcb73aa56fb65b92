// device.hpp — wave64 helpers shared by the encoding kernels (gfx950 only).
#pragma once
#include "pga/core.hpp"

// The dynamic LDS of every kernel: one extern __shared__ symbol with external
// linkage (declared inside a kernel of an anonymous namespace it would have
// internal linkage and no definition, -Wundefined-internal).
extern __shared__ __attribute__((aligned(16))) unsigned char pga_dyn_lds[];

namespace pga {
namespace dev {

constexpr int kBlock = 256;  // 4 waves; every kernel uses this block size

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// reduction over an aligned group of GS lanes (GS power of two <= 64)
template <int GS>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = GS / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int GS>
__device__ __forceinline__ uint32_t group_sum_u(uint32_t v) {
#pragma unroll
  for (int o = GS / 2; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}
template <int GS>
__device__ __forceinline__ uint32_t group_min_u(uint32_t v) {
#pragma unroll
  for (int o = GS / 2; o > 0; o >>= 1) {
    uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
  uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
  uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
  return ((unsigned long long)hi << 32) | lo;
}

// block-wide max of a packed best, result valid in every thread (BLK threads)
template <int BLK = kBlock>
__device__ __forceinline__ unsigned long long block_max_u64(unsigned long long v, unsigned long long* lds4) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = shfl_xor_u64(v, o);
    v = w > v ? w : v;
  }
  if (BLK == 64) return v;
  __syncthreads();
  if (lane_id() == 0) lds4[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long r = lds4[0];
#pragma unroll
  for (int i = 1; i < BLK / 64; ++i) r = lds4[i] > r ? lds4[i] : r;
  return r;
}

// reduce an array of packed bests with the whole block
template <int BLK = kBlock>
__device__ __forceinline__ unsigned long long block_reduce_parts(const unsigned long long* parts, uint32_t n,
                                                                 unsigned long long* lds4) {
  unsigned long long v = 0;
  for (uint32_t i = threadIdx.x; i < n; i += BLK) v = parts[i] > v ? parts[i] : v;
  return block_max_u64<BLK>(v, lds4);
}

// one wave's max over an array of packed bests (every lane gets it)
__device__ __forceinline__ unsigned long long wave_reduce_parts(const unsigned long long* parts, uint32_t n) {
  unsigned long long v = 0;
  for (uint32_t i = lane_id(); i < n; i += 64) v = parts[i] > v ? parts[i] : v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = shfl_xor_u64(v, o);
    v = w > v ? w : v;
  }
  return v;
}

// the same two for a block of `nw` waves chosen at launch (nw <= 16; lds:
// nw entries)
__device__ __forceinline__ unsigned long long block_max_u64_n(unsigned long long v, unsigned long long* lds,
                                                              uint32_t nw) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = shfl_xor_u64(v, o);
    v = w > v ? w : v;
  }
  __syncthreads();
  if (lane_id() == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long r = lds[0];
  for (uint32_t i = 1; i < nw; ++i) r = lds[i] > r ? lds[i] : r;
  return r;
}
__device__ __forceinline__ unsigned long long block_reduce_parts_n(const unsigned long long* parts, uint32_t n,
                                                                   unsigned long long* lds, uint32_t nw) {
  unsigned long long v = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) v = parts[i] > v ? parts[i] : v;
  return block_max_u64_n(v, lds, nw);
}

// Fused per-generation statistics: every evaluating kernel keeps a running
// {min, sum} of the scores its lanes produce and, when GenArgs::stats_parts is
// set, stores one {min, sum} pair per block next to its packed best (the max),
// so min / max / mean of a generation need no pass over the scores.
struct ScoreStats {
  float mn = __builtin_inff(), sm = 0.f;
  __device__ __forceinline__ void add(float v) {
    mn = fminf(mn, v);
    sm += v;
  }
  __device__ __forceinline__ void add_if(bool ok, float v) {
    mn = ok ? fminf(mn, v) : mn;
    sm += ok ? v : 0.f;
  }
};

// block reduction of the lanes' ScoreStats -> parts[2*blockIdx.x .. +1]; every
// thread of the block calls it (block-uniform control flow)
template <int BLK = kBlock>
__device__ __forceinline__ void block_stats_store(ScoreStats st, float* parts) {
  __shared__ float lds_st[2][BLK / 64];
  float mn = st.mn, sm = st.sm;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    sm += __shfl_xor(sm, o, 64);
  }
  if (BLK > 64) {
    __syncthreads();
    if (lane_id() == 0) {
      lds_st[0][threadIdx.x >> 6] = mn;
      lds_st[1][threadIdx.x >> 6] = sm;
    }
    __syncthreads();
    mn = lds_st[0][0];
    sm = lds_st[1][0];
#pragma unroll
    for (int i = 1; i < BLK / 64; ++i) {
      mn = fminf(mn, lds_st[0][i]);
      sm += lds_st[1][i];
    }
  }
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = mn;
    parts[2 * blockIdx.x + 1] = sm;
  }
}

// block_stats_store for a block of `nw` waves chosen at launch (nw <= 16)
__device__ __forceinline__ void block_stats_store_n(ScoreStats st, float* parts, uint32_t nw) {
  __shared__ float lds_stn[2][16];
  float mn = st.mn, sm = st.sm;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    sm += __shfl_xor(sm, o, 64);
  }
  __syncthreads();
  if (lane_id() == 0) {
    lds_stn[0][threadIdx.x >> 6] = mn;
    lds_stn[1][threadIdx.x >> 6] = sm;
  }
  __syncthreads();
  mn = lds_stn[0][0];
  sm = lds_stn[1][0];
  for (uint32_t i = 1; i < nw; ++i) {
    mn = fminf(mn, lds_stn[0][i]);
    sm += lds_stn[1][i];
  }
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = mn;
    parts[2 * blockIdx.x + 1] = sm;
  }
}

// Child word pool: lane q of a GS-lane group holds Philox block q of the
// child's ST_CHILD stream.  Child word t < 3*GS lives in register t%3 of lane
// t/3 and is fetched with one ds_bpermute (t must be group-uniform); later
// words are computed on demand.  Register .w of lane q's block is the first
// mutation draw of chunk q (see core.hpp).
template <int GS>
struct Pool {
  u32x4 w;
  uint32_t gbase;
  __device__ __forceinline__ uint32_t get(uint32_t t, const RngKey& key, uint64_t child) const {
    if (t < 3u * GS) {
      const uint32_t v = sel3(w, t % 3u);
      if (GS == 1) return v;
      return (uint32_t)__shfl((int)v, (int)(gbase + t / 3u), 64);
    }
    return child_word(key, child, t);
  }
};

// fitness-proportional pick: smallest i with cumfit[i] > target (cumfit inclusive)
__device__ __forceinline__ uint32_t roulette_pick(const float* cumfit, uint32_t S, uint32_t w) {
  float total = cumfit[S - 1];
  if (!(total > 0.f)) return word_to_index(w, S);  // all weights zero: uniform
  float target = word_to_unit(w) * total;
  uint32_t lo = 0, hi = S - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (cumfit[mid] < target) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Parents of `child` from the ST_SEL words (BINARY and REAL layouts,
// core.hpp); group-uniform (every lane of the group computes the same).
// Mirrors cpu_ops.cpp bin_select_parents.
__device__ __forceinline__ void st_select_parents(const GenArgs& a, uint64_t child, uint32_t& pa, uint32_t& pb) {
  const uint32_t S = (uint32_t)a.S;
  u32x4 blk = draw(a.key, ST_SEL, child, 0);
  if (a.selection == SEL_TOURNAMENT && a.tour_k == 2) {
    const uint32_t i0 = word_to_index(blk.x, S), i1 = word_to_index(blk.y, S);
    const uint32_t i2 = word_to_index(blk.z, S), i3 = word_to_index(blk.w, S);
    const float s0 = a.score_cur[i0], s1 = a.score_cur[i1], s2 = a.score_cur[i2], s3 = a.score_cur[i3];
    pa = (s0 < s1) ? i1 : i0;
    pb = (s2 < s3) ? i3 : i2;
  } else if (a.selection == SEL_TOURNAMENT) {
    const uint32_t k = a.tour_k;
    uint32_t cb = 0, best[2];
    for (uint32_t p = 0; p < 2; ++p) {
      uint32_t b = 0;
      float bs = 0.f;
      for (uint32_t j = 0; j < k; ++j) {
        const uint32_t t = p * k + j;
        if ((t >> 2) != cb) {
          cb = t >> 2;
          blk = draw(a.key, ST_SEL, child, cb);
        }
        const uint32_t c = word_to_index(sel4(blk, t & 3u), S);
        const float cs = a.score_cur[c];
        if (j == 0 || bs < cs) {
          bs = cs;
          b = c;
        }
      }
      best[p] = b;
    }
    pa = best[0];
    pb = best[1];
  } else if (a.selection == SEL_ROULETTE) {
    pa = roulette_pick(a.cumfit, S, blk.x);
    pb = roulette_pick(a.cumfit, S, blk.y);
  } else if (a.selection == SEL_RANK) {
    const u32x4 b1 = draw(a.key, ST_SEL, child, 1);
    pa = a.rank_order[rank_pick(blk.x, blk.y, blk.z, S, a.rank_thresh)];
    pb = a.rank_order[rank_pick(blk.w, b1.x, b1.y, S, a.rank_thresh)];
  } else {
    pa = word_to_index(blk.x, S);
    pb = word_to_index(blk.y, S);
  }
}

// LDS written by other lanes of this wave is read after it (LDS ops of one
// wave complete in order; this only stops the compiler moving them)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// graph replay: take the generation from the device counter (see GenArgs)
__device__ __forceinline__ void resolve_gen(GenArgs& a) {
  if (a.gen_dev) a.key.gen = *a.gen_dev + a.gen_off;
}

// Pick two parents.  All selection words are group-uniform.  P: the group's
// Pool, or any view with the same get() (perm.hip LanePool: one lane's child)
template <int GS, typename P = Pool<GS>>
__device__ __forceinline__ void select_parents(const GenArgs& a, const P& pool, uint64_t child,
                                               uint32_t& pa, uint32_t& pb) {
  const uint32_t S = (uint32_t)a.S;
  if (a.selection == SEL_TOURNAMENT) {
    const uint32_t k = a.tour_k;
    if (k == 2) {
      // issue all four score loads before any compare (memory-level parallelism)
      uint32_t i0 = word_to_index(pool.get(W_SEL + 0, a.key, child), S);
      uint32_t i1 = word_to_index(pool.get(W_SEL + 1, a.key, child), S);
      uint32_t i2 = word_to_index(pool.get(W_SEL + 2, a.key, child), S);
      uint32_t i3 = word_to_index(pool.get(W_SEL + 3, a.key, child), S);
      float s0 = a.score_cur[i0], s1 = a.score_cur[i1], s2 = a.score_cur[i2], s3 = a.score_cur[i3];
      pa = (s0 < s1) ? i1 : i0;
      pb = (s2 < s3) ? i3 : i2;
    } else {
      uint32_t best[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint32_t b = word_to_index(pool.get(W_SEL + p * k, a.key, child), S);
        float bs = a.score_cur[b];
        for (uint32_t j = 1; j < k; ++j) {
          uint32_t c = word_to_index(pool.get(W_SEL + p * k + j, a.key, child), S);
          float cs = a.score_cur[c];
          if (bs < cs) { bs = cs; b = c; }
        }
        best[p] = b;
      }
      pa = best[0];
      pb = best[1];
    }
  } else if (a.selection == SEL_ROULETTE) {
    pa = roulette_pick(a.cumfit, S, pool.get(W_SEL + 0, a.key, child));
    pb = roulette_pick(a.cumfit, S, pool.get(W_SEL + 1, a.key, child));
  } else if (a.selection == SEL_RANK) {
    const uint32_t ra = rank_pick(pool.get(W_SEL + 0, a.key, child), pool.get(W_SEL + 1, a.key, child),
                                  pool.get(W_SEL + 2, a.key, child), S, a.rank_thresh);
    const uint32_t rb = rank_pick(pool.get(W_SEL + 3, a.key, child), pool.get(W_SEL + 4, a.key, child),
                                  pool.get(W_SEL + 5, a.key, child), S, a.rank_thresh);
    pa = a.rank_order[ra];
    pb = a.rank_order[rb];
  } else {
    pa = word_to_index(pool.get(W_SEL + 0, a.key, child), S);
    pb = word_to_index(pool.get(W_SEL + 1, a.key, child), S);
  }
}

}  // namespace dev
}  // namespace pga
