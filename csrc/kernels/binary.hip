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
// Grid: persistent grid-stride over individuals, sized from the kernel's
// measured occupancy (no partial second wave); a block's children are
// contiguous so its stores are contiguous.  Parents are random rows, so there
// is no inter-block reuse to make XCD-aware (guide §5.5 T1 transfers only to
// neighbour-tile reuse).
//
// Two kernels:
//   binary_kernel<GS,OBJ,MODE>   every mode / operator; one child at a time
//   binary_gen_pipe<GS,OBJ,XO>   the hot generation path, software-pipelined
//                                three children deep (see below)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "pga/device.hpp"
#include "pga/ops.hpp"

namespace pga {
namespace {

using namespace dev;

// PGA_PIPELINE=0 forces the generic GEN kernel (A/B testing)
bool getenv_pipeline() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PGA_PIPELINE");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// per-lane objective accumulator over the chunks a lane owns
template <int OBJ>
struct BinObj {
  uint32_t u = 0;                 // ONEMAX / TRAP counts
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

__device__ __forceinline__ uint4 u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ uint4 and4(uint4 a, uint4 b) { return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w); }
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 mix4(uint4 a, uint4 b, uint4 m) {  // a where m, else b
  return make_uint4((a.x & m.x) | (b.x & ~m.x), (a.y & m.y) | (b.y & ~m.y), (a.z & m.z) | (b.z & ~m.z),
                    (a.w & m.w) | (b.w & ~m.w));
}
__device__ __forceinline__ uint4 range_keep_a(uint32_t c, uint32_t lo, uint32_t hi) {  // 1 = bit from A
  const uint32_t b0 = c * 128u;
  return make_uint4(~range_mask32(b0, lo, hi), ~range_mask32(b0 + 32, lo, hi), ~range_mask32(b0 + 64, lo, hi),
                    ~range_mask32(b0 + 96, lo, hi));
}
__device__ __forceinline__ uint4 bit4(uint32_t b) {  // one bit of a 128-bit chunk
  const uint32_t m = 1u << (b & 31u), j = b >> 5;
  return make_uint4(j == 0 ? m : 0u, j == 1 ? m : 0u, j == 2 ? m : 0u, j == 3 ? m : 0u);
}
__device__ __forceinline__ uint32_t chunk_len(uint32_t L, uint32_t c) {
  const uint32_t b = c * 128u;
  return L - b >= 128u ? 128u : L - b;
}

// ---------------------------------------------------------------------------
// Generic kernel: every mode, every operator, any genome length.
// ---------------------------------------------------------------------------
template <int GS, int OBJ, int MODE>
__global__ __launch_bounds__(kBlock) void binary_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  __shared__ uint32_t lds_thr[kMutCap];

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
  constexpr bool MUTATES = MODE == MODE_GEN || MODE == MODE_MUTATE;
  constexpr bool EVALS = OBJ != OBJ_NONE && (MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL);
  const bool bitflip = MUTATES && a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (MUTATES && bitflip)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

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
      pool.w = u32x4{0, 0, 0, 0};
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
      uint32_t rpos = 0xFFFFFFFFu;  // RESET_ONE: the one flipped bit
      if (reset_one && pool.get(W_MUTIND, a.key, child) < a.mut_ind_thresh)
        rpos = word_to_index(pool.get(W_MUTPOS, a.key, child), L);

      BinObj<OBJ> acc;
      for (uint32_t c0 = 0; c0 < nchunks; c0 += GS) {  // group-uniform segment loop
        const uint32_t c = c0 + q;
        if (c >= nchunks) continue;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (MODE == MODE_INIT) {
          v = u4(draw(a.key, ST_INIT, child, c));
        } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
          v = cur[child * rs + c];
        } else {
          const uint4 A = cur[(uint64_t)pa * rs + c];
          if (xo) {
            const uint4 B = cur[(uint64_t)pb * rs + c];
            const uint4 m = a.crossover == XO_UNIFORM ? u4(draw(a.key, ST_XO, child, c)) : range_keep_a(c, blo, bhi);
            v = mix4(A, B, m);
          } else {
            v = A;
          }
        }
        if (c == nchunks - 1) v = and4(v, u4(a.last_mask));
        if (bitflip) {
          const uint32_t r0 = c == q ? pool.w.w : chunk_mut_word(a.key, child, c);
          v = xor4(v, u4(chunk_flip_mask(a, child, c, chunk_len(L, c), r0, lds_thr)));
        } else if (reset_one && (rpos >> 7) == c) {
          v = xor4(v, bit4(rpos & 127u));
        }
        if (MODE != MODE_EVAL) nxt[child * rs + c] = v;
        if (EVALS) acc.add(a, v, c);
      }
      if (EVALS) score = acc.template finish<GS>(a);
    }
    if (EVALS && q == 0) {
      a.score_next[child] = score;
      if (a.key_next) a.key_next[child] = (uint16_t)score;
      const unsigned long long pb = pack_best(score, child);
      my_best = pb > my_best ? pb : my_best;
    }
  }
  if (EVALS && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
  }
}

// ---------------------------------------------------------------------------
// Software-pipelined fused generation (the hot path).
//
// Every child is a chain of two DEPENDENT global round trips (tournament
// score reads -> parent-row gathers) followed by a few hundred VALU
// instructions.  Each group keeps three children in flight:
//   body:  S2(c+1)  tournament compare + issue the parent-row loads
//          S1(c+2)  Philox pool + issue 4 score loads
//          S3(c)    crossover mask + mutation + fitness + stores
// The body is unrolled x3 over statically rotated register sets (a register
// COPY of an in-flight load forces s_waitcnt vmcnt(0)), the mutation table
// lives in LDS (a global table lookup would wait on every older load: vmcnt
// retires in order) and mutation flips go to a separate mask so no loop ever
// touches an in-flight register.  Valid when every lane owns at most one
// chunk (L <= 8192 bits) and selection is tournament-2 or random.
// Bit-identical to binary_kernel.
// ---------------------------------------------------------------------------
constexpr int XOK_UNIFORM = 0, XOK_RANGE = 1;  // crossover kind template values

// Diagnostic ablation switches (bench/micro/ablate builds only, see
// bench/micro/README.md; the shipped build defines none of them).
// Waves per SIMD the pipelined kernel is register-limited to.  Measured: a
// fourth register set (rows of c+1 AND c+2 in flight) at 5 or 4 waves/SIMD
// ran 96.8 / 97.9 us/gen against 92.4 for three sets at 6 waves (headline).
#ifndef PGA_PIPE_WAVES
#define PGA_PIPE_WAVES 6
#endif
#ifndef PGA_ABL
#define PGA_ABL 0
#endif
constexpr int kAblXoRng = 1, kAblPoolRng = 2, kAblMut = 4, kAblGather = 8;
#ifndef PGA_CACHE
#define PGA_CACHE 0  // 1: non-temporal child stores, 2: non-temporal parent loads
#endif
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_row(uint4* p, uint4 v) {
  if (PGA_CACHE & 1) {
    v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (v4u*)p);
  } else {
    *p = v;
  }
}
__device__ __forceinline__ uint4 load_row(const uint4* p) {
  if (PGA_CACHE & 2) {
    v4u x = __builtin_nontemporal_load((const v4u*)p);
    return make_uint4(x[0], x[1], x[2], x[3]);
  }
  return *p;
}

// PGA_STAMP builds (bench/micro only): per-wave start/end wall-clock stamps of
// the pipelined kernel, dumped by pga_stamp_report() (ramp-up / tail study)
#ifndef PGA_STAMP
#define PGA_STAMP 0
#endif
#if PGA_STAMP
__device__ unsigned long long g_stamps[2 * 65536];
#endif

// RESET: the per-individual reset mutation is possible (otherwise only
// bit-flip / none, and the pool words are dead after stage 2: fewer VGPRs)
template <int GS, int OBJ, int XOK, bool KEY, bool RESET>
__global__ __launch_bounds__(kBlock, RESET ? PGA_PIPE_WAVES - 1 : PGA_PIPE_WAVES) void binary_gen_pipe(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  __shared__ uint32_t lds_thr[kMutCap];

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  constexpr uint32_t GPB = kBlock / GS;
  const uint64_t rs = a.row_words >> 2;
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  const uint32_t L = a.L;
  const uint32_t S = (uint32_t)a.S;
  const bool have = q < a.chunks;
  const bool last = q == a.chunks - 1;
  const uint32_t clen = have ? chunk_len(L, q) : 0u;
  const bool k2 = a.selection == SEL_TOURNAMENT;  // tour_k == 2 guaranteed by the launcher
  const bool xo_on = a.crossover != XO_NONE;
  const bool bitflip = a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f;
  const bool reset_one = RESET && a.mutation == MUT_RESET_ONE;
  const uint4 lmask = u4(a.last_mask);

  if (a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (bitflip)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

#if PGA_STAMP
  const uint32_t wid_ = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (lane == 0 && wid_ < 65536) g_stamps[2 * wid_] = wall_clock64();
#endif
  unsigned long long my_best = 0;
  const uint64_t stride = (uint64_t)gridDim.x * GPB;
  uint64_t c0 = (uint64_t)blockIdx.x * GPB + threadIdx.x / GS;

  // elites first (only the first few groups of the grid have any)
  while (c0 < a.n_elite && c0 < a.S) {
    const uint32_t src = a.elite_idx ? a.elite_idx[c0] : lds_elite;
    if (have) nxt[c0 * rs + q] = cur[(uint64_t)src * rs + q];
    const float sc = a.score_cur[src];
    if (q == 0) {
      a.score_next[c0] = sc;
      if (KEY) a.key_next[c0] = (uint16_t)sc;
      const unsigned long long pb = pack_best(sc, c0);
      my_best = pb > my_best ? pb : my_best;
    }
    c0 += stride;
  }

#define PGA_SET(P)                                                       \
  u32x4 P##w{0, 0, 0, 0};                                                \
  uint32_t P##i0 = 0, P##i1 = 0, P##i2 = 0, P##i3 = 0;                   \
  float P##t0 = 0.f, P##t1 = 0.f, P##t2 = 0.f, P##t3 = 0.f;              \
  uint4 P##A = make_uint4(0, 0, 0, 0), P##B = make_uint4(0, 0, 0, 0);    \
  uint32_t P##lo = 0, P##hi = 0;                                         \
  bool P##xo = false;
  PGA_SET(X)
  PGA_SET(Y)
  PGA_SET(Z)
#undef PGA_SET

  // Stages 1 and 2 issue their loads UNCONDITIONALLY (indices clamped for
  // tail children, lanes without a chunk re-read chunk 0, B re-reads A's line
  // when there is no crossover): hipcc's waitcnt pass must assume the minimum
  // number of vector-memory ops over all paths, so any conditionally issued
  // load between a load and its use degrades the wait to vmcnt(0).
  const uint32_t qq = have ? q : 0u;

  // stage 1: Philox pool + tournament contestant score loads
#define PGA_STAGE1(c, P)                                                   \
  {                                                                        \
    const uint64_t cc_ = (c) < a.S ? (c) : a.S - 1;                        \
    if (PGA_ABL & kAblPoolRng) {                                           \
      const uint32_t h_ = (uint32_t)cc_ * 0x9E3779B9u + q * 0x85EBCA6Bu;   \
      P##w = u32x4{h_, h_ * 0xC2B2AE35u, h_ ^ 0x27D4EB2Fu, h_ * 3u};        \
    } else {                                                               \
      P##w = draw(a.key, ST_CHILD, cc_, q);                                \
    }                                                                      \
    Pool<GS> pool_{P##w, gbase};                                           \
    P##i0 = word_to_index(pool_.get(W_SEL + 0, a.key, cc_), S);            \
    P##i1 = word_to_index(pool_.get(W_SEL + 1, a.key, cc_), S);            \
    P##i2 = word_to_index(pool_.get(W_SEL + 2, a.key, cc_), S);            \
    P##i3 = word_to_index(pool_.get(W_SEL + 3, a.key, cc_), S);            \
    if (KEY) { /* exact u16 keys: L2-resident, same comparisons */        \
      P##t0 = (float)a.key_cur[P##i0];                                     \
      P##t1 = (float)a.key_cur[P##i1];                                     \
      P##t2 = (float)a.key_cur[P##i2];                                     \
      P##t3 = (float)a.key_cur[P##i3];                                     \
    } else {                                                               \
      P##t0 = a.score_cur[P##i0];                                          \
      P##t1 = a.score_cur[P##i1];                                          \
      P##t2 = a.score_cur[P##i2];                                          \
      P##t3 = a.score_cur[P##i3];                                          \
    }                                                                      \
  }

  // stage 2: tournament winners (branch-free select), crossover plan, row loads
#define PGA_STAGE2(c, P)                                                                    \
  {                                                                                         \
    const uint64_t cc_ = (c) < a.S ? (c) : a.S - 1;                                         \
    uint32_t pa_, pb_;                                                                      \
    if (k2) {                                                                               \
      pa_ = P##i0 ^ ((P##i0 ^ P##i1) & (0u - (uint32_t)(P##t0 < P##t1)));                   \
      pb_ = P##i2 ^ ((P##i2 ^ P##i3) & (0u - (uint32_t)(P##t2 < P##t3)));                   \
    } else {                                                                                \
      pa_ = P##i0;                                                                          \
      pb_ = P##i1;                                                                          \
    }                                                                                       \
    Pool<GS> pool_{P##w, gbase};                                                            \
    P##xo = xo_on && do_crossover(a, pool_.get(W_XOPROB, a.key, cc_));                      \
    if (XOK == XOK_RANGE) {                                                                 \
      const uint32_t x1_ = word_to_index(pool_.get(W_CUT1, a.key, cc_), L);                 \
      if (a.crossover == XO_ONE_POINT) {                                                    \
        P##lo = x1_;                                                                        \
        P##hi = L;                                                                          \
      } else {                                                                              \
        const uint32_t x2_ = word_to_index(pool_.get(W_CUT2, a.key, cc_), L);               \
        P##lo = x1_ < x2_ ? x1_ : x2_;                                                      \
        P##hi = x1_ < x2_ ? x2_ : x1_;                                                      \
      }                                                                                     \
    }                                                                                       \
    pb_ = P##xo ? pb_ : pa_;                                                                \
    if (PGA_ABL & kAblGather) {                                                             \
      pa_ = (uint32_t)cc_;                                                                  \
      pb_ = (uint32_t)cc_;                                                                  \
    }                                                                                       \
    P##A = load_row(cur + (uint64_t)pa_ * rs + qq);                                         \
    P##B = load_row(cur + (uint64_t)pb_ * rs + qq);                                         \
  }

  // stage 3: crossover, mutation (own-register first draw, LDS thresholds),
  // fitness, stores
#define PGA_STAGE3(c, P)                                                                     \
  if ((c) < a.S) {                                                                           \
    /* branch-free: a phi between the loaded row and the mixed row would be a   */          \
    /* register copy of an in-flight load (= s_waitcnt vmcnt(0))                 */          \
    const uint4 mx_ = (PGA_ABL & kAblXoRng) ? make_uint4(P##w.x, P##w.y, ~P##w.x, ~P##w.y)               \
                      : (XOK == XOK_UNIFORM ? u4(draw(a.key, ST_XO, (c), q)) : range_keep_a(q, P##lo, P##hi)); \
    const uint32_t keep_ = P##xo ? 0u : 0xFFFFFFFFu;                                         \
    const uint4 m_ = make_uint4(mx_.x | keep_, mx_.y | keep_, mx_.z | keep_, mx_.w | keep_); \
    uint4 v_ = mix4(P##A, P##B, m_);                                                         \
    if (last) v_ = and4(v_, lmask);                                                          \
    if (bitflip && !(PGA_ABL & kAblMut)) {                                                   \
      v_ = xor4(v_, u4(chunk_flip_mask(a, (c), q, clen, P##w.w, lds_thr)));                  \
    } else if (reset_one) {                                                                  \
      Pool<GS> pool_{P##w, gbase};                                                           \
      if (pool_.get(W_MUTIND, a.key, (c)) < a.mut_ind_thresh) {                              \
        const uint32_t mpos_ = word_to_index(pool_.get(W_MUTPOS, a.key, (c)), L);            \
        if ((mpos_ >> 7) == q) v_ = xor4(v_, bit4(mpos_ & 127u));                            \
      }                                                                                      \
    }                                                                                        \
    BinObj<OBJ> acc_;                                                                        \
    if (have) {                                                                              \
      store_row(nxt + (c) * rs + q, v_);                                                     \
      acc_.add(a, v_, q);                                                                    \
    }                                                                                        \
    const float sc_ = acc_.template finish<GS>(a);                                           \
    if (q == 0) {                                                                            \
      a.score_next[(c)] = sc_;                                                               \
      if (KEY) a.key_next[(c)] = (uint16_t)sc_;                                              \
      const unsigned long long pb_ = pack_best(sc_, (c));                                    \
      my_best = pb_ > my_best ? pb_ : my_best;                                               \
    }                                                                                        \
  }

  // prologue: X = c0 (after stage 2), Y = c1 (after stage 1).  Each body
  // issues the score loads of c+2, then the row loads of c+1 (whose score
  // loads went out one body earlier), then finishes c (rows one body old).
  PGA_STAGE1(c0, X)
  PGA_STAGE2(c0, X)
  PGA_STAGE1(c0 + stride, Y)
  while (c0 < a.S) {  // group-uniform
    PGA_STAGE1(c0 + 2 * stride, Z)
    PGA_STAGE2(c0 + stride, Y)
    PGA_STAGE3(c0, X)
    c0 += stride;
    if (c0 >= a.S) break;
    PGA_STAGE1(c0 + 2 * stride, X)
    PGA_STAGE2(c0 + stride, Z)
    PGA_STAGE3(c0, Y)
    c0 += stride;
    if (c0 >= a.S) break;
    PGA_STAGE1(c0 + 2 * stride, Y)
    PGA_STAGE2(c0 + stride, X)
    PGA_STAGE3(c0, Z)
    c0 += stride;
  }
#undef PGA_STAGE1
#undef PGA_STAGE2
#undef PGA_STAGE3
#if PGA_STAMP
  if (lane == 0 && wid_ < 65536) g_stamps[2 * wid_ + 1] = wall_clock64();
#endif

  unsigned long long b = block_max_u64(my_best, lds_red);
  if (threadIdx.x == 0 && best_parts) best_parts[blockIdx.x] = b;
}

template <typename K>
uint32_t go(K kernel, const GenArgs& a, unsigned long long* parts, uint32_t gpb, hipStream_t s) {
  const uint32_t grid = launch_grid_occ(a.S, gpb, (const void*)kernel);
  hipLaunchKernelGGL(kernel, grid, kBlock, 0, s, a, parts);
  return grid;
}

template <int GS, int OBJ>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  constexpr uint32_t gpb = kBlock / GS;
  switch (mode) {
    case MODE_GEN: {
      const bool pipe = a.chunks <= (uint32_t)GS &&
                        ((a.selection == SEL_TOURNAMENT && a.tour_k == 2) || a.selection == SEL_RANDOM) &&
                        !(a.n_elite > 1 && a.elite_idx == nullptr) && getenv_pipeline();
      if (pipe) {
        constexpr bool INT_OBJ = OBJ == OBJ_ONEMAX || OBJ == OBJ_LEADING_ONES || OBJ == OBJ_TRAP;
        const bool key = INT_OBJ && a.key_cur != nullptr;
        const bool range = a.crossover == XO_ONE_POINT || a.crossover == XO_TWO_POINT;
        const bool reset = a.mutation == MUT_RESET_ONE;
#define PGA_PIPE(XK, KY)                                                        \
  return reset ? go(binary_gen_pipe<GS, OBJ, XK, KY, true>, a, parts, gpb, s)   \
               : go(binary_gen_pipe<GS, OBJ, XK, KY, false>, a, parts, gpb, s);
        if (key) {
          if (range) { PGA_PIPE(XOK_RANGE, INT_OBJ) }
          PGA_PIPE(XOK_UNIFORM, INT_OBJ)
        }
        if (range) { PGA_PIPE(XOK_RANGE, false) }
        PGA_PIPE(XOK_UNIFORM, false)
#undef PGA_PIPE
      }
      return go(binary_kernel<GS, OBJ, MODE_GEN>, a, parts, gpb, s);
    }
    case MODE_INIT: return go(binary_kernel<GS, OBJ, MODE_INIT>, a, parts, gpb, s);
    case MODE_EVAL: return go(binary_kernel<GS, OBJ, MODE_EVAL>, a, parts, gpb, s);
    case MODE_CROSS: return go(binary_kernel<GS, OBJ_NONE, MODE_CROSS>, a, parts, gpb, s);
    default: return go(binary_kernel<GS, OBJ_NONE, MODE_MUTATE>, a, parts, gpb, s);
  }
}

template <int GS>
uint32_t launch_obj(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (a.objective) {
    case OBJ_ONEMAX: return launch_mode<GS, OBJ_ONEMAX>(mode, a, parts, s);
    case OBJ_KNAPSACK: return launch_mode<GS, OBJ_KNAPSACK>(mode, a, parts, s);
    case OBJ_TRAP: return launch_mode<GS, OBJ_TRAP>(mode, a, parts, s);
    case OBJ_LEADING_ONES: return launch_mode<GS, OBJ_LEADING_ONES>(mode, a, parts, s);
    default: return launch_mode<GS, OBJ_NONE>(mode, a, parts, s);
  }
}

}  // namespace

#if PGA_STAMP
// wave start/end distribution of the last pipelined launch (100 MHz wall clock)
void pga_stamp_report(uint32_t nwaves) {
  std::vector<unsigned long long> h(2ull * nwaves);
  PGA_HIP_CHECK(hipDeviceSynchronize());
  PGA_HIP_CHECK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_stamps), 16ull * nwaves));
  unsigned long long t0 = ~0ull;
  for (uint32_t i = 0; i < nwaves; ++i) t0 = h[2 * i] < t0 ? h[2 * i] : t0;
  std::vector<double> st, en, du;
  for (uint32_t i = 0; i < nwaves; ++i) {
    st.push_back((h[2 * i] - t0) * 0.01);
    en.push_back((h[2 * i + 1] - t0) * 0.01);
    du.push_back((h[2 * i + 1] - h[2 * i]) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    std::printf("%s us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n", n, v[0], v[v.size() / 10], v[v.size() / 2],
                v[v.size() * 9 / 10], v.back());
  };
  pr("wave start", st);
  pr("wave end  ", en);
  pr("wave life ", du);
}
#endif

uint32_t binary_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  uint32_t grid = 0;
  switch (group_size(a.chunks)) {
    case 1: grid = launch_obj<1>(mode, a, best_parts, s); break;
    case 2: grid = launch_obj<2>(mode, a, best_parts, s); break;
    case 4: grid = launch_obj<4>(mode, a, best_parts, s); break;
    case 8: grid = launch_obj<8>(mode, a, best_parts, s); break;
    case 16: grid = launch_obj<16>(mode, a, best_parts, s); break;
    case 32: grid = launch_obj<32>(mode, a, best_parts, s); break;
    default: grid = launch_obj<64>(mode, a, best_parts, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace pga
