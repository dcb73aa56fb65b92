// binary.hip — bit-packed BINARY encoding on gfx950.
//
// One individual = one row of `chunks` 16-byte chunks (128 genes each).  A
// group of GS = group_size(chunks) lanes owns one individual: lane q holds
// chunk q (q+GS, ... for genomes longer than 64 chunks), so every parent-row
// gather is a fully used 16 B/lane dwordx4 load (8 lanes = one 128-B line for
// the 1024-bit headline config) and the fitness reduction is a GS-lane
// butterfly.  ONE launch per generation fuses
//     tournament selection -> crossover -> bit-flip mutation -> fitness
//     -> child store + score store + per-block best
// replacing the reference's RNG-fill + 3 kernels x ceil(S/512) launches + 3
// device syncs per generation (src/pga.cu:376-391, :250-347).  No random
// buffer is materialised: every draw is an in-register Philox4x32-10.
//
// Grid: persistent grid-stride over individuals, grid = min(ceil(S/GPB),
// 8 * CUs); a block's children are contiguous so its stores are contiguous.
// Parents are random rows, so there is no inter-block reuse to make
// XCD-aware (guide §5.5 T1 transfers only to neighbour-tile reuse).
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"

namespace pga {
namespace {

using namespace dev;

// per-lane objective accumulator over the chunks a lane owns
template <int OBJ>
struct BinObj {
  uint32_t u = 0;        // ONEMAX / TRAP counts
  uint32_t first0 = 0xFFFFFFFFu;  // LEADING_ONES: first zero bit position
  float v = 0.f, w = 0.f;         // KNAPSACK

  __device__ __forceinline__ void add(const GenArgs& a, uint4 x, uint32_t c) {
    const uint32_t wd[4] = {x.x, x.y, x.z, x.w};
    if (OBJ == OBJ_ONEMAX) {
      u += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
    } else if (OBJ == OBJ_KNAPSACK) {
      const float* val = a.obj_data;
      const float* wt = a.obj_data + a.L;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t bits = wd[j];
        const uint32_t base = c * 128u + 32u * j;
        while (bits) {
          uint32_t b = __ffs(bits) - 1;
          bits &= bits - 1;
          v += val[base + b];
          w += wt[base + b];
        }
      }
    } else if (OBJ == OBJ_TRAP) {
      const uint32_t k = (uint32_t)a.obj_i;
      const uint32_t km = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t base = c * 128u + 32u * j;
        for (uint32_t i = 0; i < 32u; i += k) {
          if (base + i + k > a.L) break;
          uint32_t ones = __popc((wd[j] >> i) & km);
          u += ones == k ? k : (k - 1 - ones);
        }
      }
    } else if (OBJ == OBJ_LEADING_ONES) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t inv = ~wd[j];
        if (inv != 0u) {
          uint32_t p = c * 128u + 32u * j + (__ffs(inv) - 1);
          first0 = p < first0 ? p : first0;
          break;
        }
      }
    }
  }

  template <int GS>
  __device__ __forceinline__ float finish(const GenArgs& a) {
    if (OBJ == OBJ_ONEMAX || OBJ == OBJ_TRAP) return (float)group_sum_u<GS>(u);
    if (OBJ == OBJ_KNAPSACK) {
      float vv = group_sum<GS>(v), ww = group_sum<GS>(w);
      return ww <= a.obj_f0 ? vv : a.obj_f0 - ww;
    }
    if (OBJ == OBJ_LEADING_ONES) {
      uint32_t m = group_min_u<GS>(first0);
      return (float)(m < a.L ? m : a.L);
    }
    return 0.f;
  }
};

__device__ __forceinline__ uint4 and4(uint4 a, uint4 b) { return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w); }
__device__ __forceinline__ uint4 mix4(uint4 a, uint4 b, uint4 m) {  // a where m, else b
  return make_uint4((a.x & m.x) | (b.x & ~m.x), (a.y & m.y) | (b.y & ~m.y), (a.z & m.z) | (b.z & ~m.z),
                    (a.w & m.w) | (b.w & ~m.w));
}
__device__ __forceinline__ void flip_bit(uint4& v, uint32_t b) {
  const uint32_t bit = 1u << (b & 31u);
  switch (b >> 5) {
    case 0: v.x ^= bit; break;
    case 1: v.y ^= bit; break;
    case 2: v.z ^= bit; break;
    default: v.w ^= bit; break;
  }
}

template <int GS, int OBJ, int MODE>
__global__ __launch_bounds__(kBlock) void binary_kernel(GenArgs a, unsigned long long* best_parts) {
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  constexpr uint32_t GPB = kBlock / GS;
  const uint32_t g_in_block = threadIdx.x / GS;
  const uint64_t rs = a.row_words >> 2;  // row stride in uint4
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  const uint32_t nchunks = a.chunks;
  const uint32_t L = a.L;

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
    __syncthreads();
  }

  const bool bitflip = (MODE == MODE_GEN || MODE == MODE_MUTATE) && a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f;
  const bool reset_one = (MODE == MODE_GEN || MODE == MODE_MUTATE) && a.mutation == MUT_RESET_ONE;
  const uint32_t mut_base = W_SEL + sel_words(a);

  unsigned long long my_best = 0;
  const uint64_t stride = (uint64_t)gridDim.x * GPB;
  for (uint64_t child = (uint64_t)blockIdx.x * GPB + g_in_block; child < a.S; child += stride) {
    float score = 0.f;
    if (MODE == MODE_GEN && child < a.n_elite) {
      // elitism: copy elite rows unchanged into the front of the next generation
      const uint32_t src = a.elite_idx ? a.elite_idx[child] : lds_elite;
      for (uint32_t c = q; c < nchunks; c += GS) nxt[child * rs + c] = cur[(uint64_t)src * rs + c];
      score = a.score_cur[src];
    } else {
      Pool<GS> pool;
      pool.gbase = gbase;
      uint32_t pa = 0, pb = 0;
      bool xo = false;
      uint32_t blo = 0, bhi = 0;  // ONE/TWO_POINT: bits [blo, bhi) come from parent B
      if (MODE == MODE_GEN || MODE == MODE_CROSS || MODE == MODE_MUTATE) pool.w = draw(a.key, ST_CHILD, child, q);
      if (MODE == MODE_GEN || MODE == MODE_CROSS) {
        select_parents<GS>(a, pool, child, pa, pb);
        xo = a.crossover != XO_NONE && do_crossover(a, pool.get(W_XOPROB, a.key, child));
        if (a.crossover == XO_ONE_POINT) {
          blo = word_to_index(pool.get(W_CUT1, a.key, child), L);
          bhi = L;
        } else if (a.crossover == XO_TWO_POINT) {
          uint32_t c1 = word_to_index(pool.get(W_CUT1, a.key, child), L);
          uint32_t c2 = word_to_index(pool.get(W_CUT2, a.key, child), L);
          blo = c1 < c2 ? c1 : c2;
          bhi = c1 < c2 ? c2 : c1;
        }
      }
      // mutation state: position of the next flip, next pool word
      uint32_t mpos = 0xFFFFFFFFu, mt = mut_base;
      if (bitflip) mpos = geom_skip(pool.get(mt++, a.key, child), a.mut_thr, L, a.mut_inv_log2_1mp);
      if (reset_one && pool.get(W_MUTIND, a.key, child) < a.mut_ind_thresh)
        mpos = word_to_index(pool.get(mt, a.key, child), L);

      BinObj<OBJ> acc;
      for (uint32_t c0 = 0; c0 < nchunks; c0 += GS) {  // group-uniform segment loop
        const uint32_t c = c0 + q;
        const bool have = c < nchunks;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (MODE == MODE_INIT) {
          if (have) {
            u32x4 r = draw(a.key, ST_INIT, child, c);
            v = make_uint4(r.x, r.y, r.z, r.w);
          }
        } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
          if (have) v = cur[child * rs + c];
        } else if (have) {
          const uint4 A = cur[(uint64_t)pa * rs + c];
          if (xo) {
            const uint4 B = cur[(uint64_t)pb * rs + c];
            uint4 m;  // 1 = take A
            if (a.crossover == XO_UNIFORM) {
              u32x4 r = draw(a.key, ST_XO, child, c);
              m = make_uint4(r.x, r.y, r.z, r.w);
            } else {
              const uint32_t b0 = c * 128u;
              m = make_uint4(~range_mask32(b0, blo, bhi), ~range_mask32(b0 + 32, blo, bhi),
                             ~range_mask32(b0 + 64, blo, bhi), ~range_mask32(b0 + 96, blo, bhi));
            }
            v = mix4(A, B, m);
          } else {
            v = A;
          }
        }
        if (c == nchunks - 1) v = and4(v, make_uint4(a.last_mask.x, a.last_mask.y, a.last_mask.z, a.last_mask.w));
        if (bitflip) {
          const uint32_t seg_end = (c0 + GS) * 128u < L ? (c0 + GS) * 128u : L;
          while (mpos < seg_end) {  // group-uniform
            if ((mpos >> 7) == c) flip_bit(v, mpos & 127u);
            mpos += 1u + geom_skip(pool.get(mt++, a.key, child), a.mut_thr, L, a.mut_inv_log2_1mp);
          }
        } else if (reset_one && mpos != 0xFFFFFFFFu && (mpos >> 7) == c) {
          flip_bit(v, mpos & 127u);
        }
        if (MODE != MODE_EVAL && have) nxt[child * rs + c] = v;
        if (OBJ != OBJ_NONE && (MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL) && have) acc.add(a, v, c);
      }
      if (OBJ != OBJ_NONE) score = acc.template finish<GS>(a);
    }
    if (OBJ != OBJ_NONE && (MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL) && q == 0) {
      a.score_next[child] = score;
      const unsigned long long pb = pack_best(score, child);
      my_best = pb > my_best ? pb : my_best;
    }
  }
  if (OBJ != OBJ_NONE && (MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL) && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
  }
}

template <int GS, int OBJ>
void launch_mode(int mode, const GenArgs& a, unsigned long long* parts, uint32_t grid, hipStream_t s) {
  switch (mode) {
    case MODE_GEN: hipLaunchKernelGGL((binary_kernel<GS, OBJ, MODE_GEN>), grid, kBlock, 0, s, a, parts); break;
    case MODE_INIT: hipLaunchKernelGGL((binary_kernel<GS, OBJ, MODE_INIT>), grid, kBlock, 0, s, a, parts); break;
    case MODE_EVAL: hipLaunchKernelGGL((binary_kernel<GS, OBJ, MODE_EVAL>), grid, kBlock, 0, s, a, parts); break;
    case MODE_CROSS: hipLaunchKernelGGL((binary_kernel<GS, OBJ_NONE, MODE_CROSS>), grid, kBlock, 0, s, a, parts); break;
    case MODE_MUTATE: hipLaunchKernelGGL((binary_kernel<GS, OBJ_NONE, MODE_MUTATE>), grid, kBlock, 0, s, a, parts); break;
  }
}

template <int GS>
void launch_obj(int mode, const GenArgs& a, unsigned long long* parts, uint32_t grid, hipStream_t s) {
  switch (a.objective) {
    case OBJ_ONEMAX: launch_mode<GS, OBJ_ONEMAX>(mode, a, parts, grid, s); break;
    case OBJ_KNAPSACK: launch_mode<GS, OBJ_KNAPSACK>(mode, a, parts, grid, s); break;
    case OBJ_TRAP: launch_mode<GS, OBJ_TRAP>(mode, a, parts, grid, s); break;
    case OBJ_LEADING_ONES: launch_mode<GS, OBJ_LEADING_ONES>(mode, a, parts, grid, s); break;
    default: launch_mode<GS, OBJ_NONE>(mode, a, parts, grid, s); break;
  }
}

}  // namespace

uint32_t binary_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  const uint32_t gs = group_size(a.chunks);
  const uint32_t gpb = kBlock / gs;
  const uint32_t grid = launch_grid(a.S, gpb);
  switch (gs) {
    case 1: launch_obj<1>(mode, a, best_parts, grid, s); break;
    case 2: launch_obj<2>(mode, a, best_parts, grid, s); break;
    case 4: launch_obj<4>(mode, a, best_parts, grid, s); break;
    case 8: launch_obj<8>(mode, a, best_parts, grid, s); break;
    case 16: launch_obj<16>(mode, a, best_parts, grid, s); break;
    case 32: launch_obj<32>(mode, a, best_parts, grid, s); break;
    default: launch_obj<64>(mode, a, best_parts, grid, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace pga
