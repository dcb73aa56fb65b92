// binary_dev.hpp — the BINARY encoding's device code (bit-packed rows, see
// csrc/kernels/binary.hip for the design): objective accumulators, the
// knapsack matrix-core evaluation, the sparse bit-flip samplers, the generic
// kernel and the hot two-phase generation kernel binary_gen_tp.  Included by
// binary.hip (the built-in objectives and the launchers) and by jitgen.hip
// (binary_gen_tp with a hipRTC-compiled user objective linked in, OBJ_JIT).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/tp.hpp"

// The user objective of a fused JIT generation kernel (jitgen.hip): defined in
// the user's bitcode, LTO-linked with the kernel's bitcode and inlined
// (jit.cpp).  Never referenced by the built-in kernels.
// The row pointer is an LDS (address space 3) pointer: the child's row as the
// step just staged it next to its global store (see kJitStageSteps).
typedef __attribute__((address_space(3))) const unsigned int* pga_lds_words;
extern "C" __device__ float pga_user_objective(pga_lds_words words, unsigned int nbits, const float* data);

namespace pga {
// jitgen.hip instantiates the generation kernel with external linkage (a named
// namespace), so the kernel keeps a predictable symbol in the bitcode the JIT
// links against; everywhere else the device code stays TU-local
#ifdef PGA_JIT_GEN
namespace jitgen {
#else
namespace {
#endif

using namespace dev;


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
// 0/1 knapsack on the matrix cores (the hot kernel's evaluation when the
// instance is integer-exact, see build_knap_table).
//
// score needs V = bits . values and W = bits . weights per child.  A wave's
// step holds its NG children as 64 16-byte chunks (lane = g*GS + q), staged
// in its LDS scratch as 16 "virtual rows" of 512 bits: virtual row m = the
// chunks of lanes 4m..4m+3 = part r = m % R (R = GS/4) of child m / R.  One
// v_mfma_i32_16x16x64_i8 per 64-bit slice s (8 slices):
//   A[m][k] = bit k of virtual row m (expanded to int8 0/1),
//   B[k][c] = digit d of quantity qty (values | weights) of the gene bit k of
//             part r stands for, column c = (2r + qty) * D + d,
// with balanced base-256 digits in [-128, 127] (D <= 4), so C[m][c] is an
// exact partial dot product in i32 and only the columns of row m's own part
// are used:  V = sum_r sum_d C[gR + r][2rD + d] 256^d  (W: qty = 1).
// The element order inside a slice (element j of lane group h <-> bit 16h + j
// of the slice's 64) is the same for A and B, so the hardware's internal k
// permutation cannot matter; the integer result equals the CPU backend's
// float sum bit for bit (every partial sum is an integer below 2^24).
// Reference: test2/test.cu:28-36 (the knapsack objective); SURVEY.md C10.
// ---------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kObjKnapMfma = 1000;  // launcher-only objective id: OBJ_KNAPSACK via knap_mfma
constexpr uint32_t kKnapSlices = 8;  // 512-bit virtual row / 64-bit MFMA k-step
constexpr uint32_t kKnapMaxCols = 16;

__device__ __forceinline__ v4i expand16(uint32_t h) {  // 16 bits -> 16 int8 {0,1}
  v4i r;
  r[0] = (int)(__umul24(h & 0xFu, 0x00204081u) & 0x01010101u);
  r[1] = (int)(__umul24((h >> 4) & 0xFu, 0x00204081u) & 0x01010101u);
  r[2] = (int)(__umul24((h >> 8) & 0xFu, 0x00204081u) & 0x01010101u);
  r[3] = (int)(__umul24((h >> 12) & 0xFu, 0x00204081u) & 0x01010101u);
  return r;
}

// chunk slot of lane 4m + h in the wave scratch: virtual row m, lane group h,
// XOR-swizzled so that both the lane-order store and the (h, n) fragment
// read touch 8 distinct 16-byte bank groups per 8 lanes
__device__ __forceinline__ uint32_t knap_slot(uint32_t m, uint32_t h) { return 4u * m + (h ^ ((m >> 1) & 3u)); }
constexpr uint32_t kKnapCStride = 20;  // ints per C column in the scratch (padded against bank conflicts)
constexpr uint32_t kKnapScratch = 16 * kKnapCStride / 4;  // uint4 per wave (>= 64 chunk slots)

// every lane of the wave calls this with its chunk `v` (zero if it holds
// none); returns the score of the lane's child.  scr: the wave's scratch
// (kKnapScratch uint4); tab: the digit table in LDS, [s][h][16 columns] x
// 16 B, columns >= knap_cols zero.
template <int GS>
__device__ __forceinline__ float knap_mfma(const GenArgs& a, uint4 v, uint32_t lane, uint32_t q, uint4* scr,
                                           const uint4* tab) {
  constexpr uint32_t R = GS / 4;
  const uint32_t D = a.knap_dig, NC = a.knap_cols;
  scr[knap_slot(lane >> 2, lane & 3u)] = v;
  wave_lds_sync();
  const uint32_t h = lane >> 4, n = lane & 15u;
  const uint4 x = scr[knap_slot(n, h)];  // A: virtual row n, lane group h's 128 bits
  const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
  const uint4* tb = tab + h * kKnapMaxCols + n;
  v4i acc = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t s = 0; s < kKnapSlices; ++s) {
    const uint4 t = tb[s * 4u * kKnapMaxCols];
    const uint32_t bits = (s & 1u) ? (xs[s >> 1] >> 16) : (xs[s >> 1] & 0xFFFFu);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(expand16(bits), v4i{(int)t.x, (int)t.y, (int)t.z, (int)t.w}, acc,
                                                0, 0, 0);
  }
  wave_lds_sync();
  int* cl = (int*)scr;  // C, column-major: [column n][row 4h + i], stride kKnapCStride
  *(v4i*)(cl + n * kKnapCStride + 4u * h) = acc;
  wave_lds_sync();
  const uint32_t g = lane / GS;
  uint32_t V = 0, W = 0;  // mod 2^32: exact, the true sums are below 2^24
  for (uint32_t e = q; e < NC; e += GS) {
    const uint32_t r = e / (2u * D), d = e % D;
    const uint32_t c = (uint32_t)cl[e * kKnapCStride + g * R + r] << (8u * d);
    if ((e / D) & 1u) W += c;
    else V += c;
  }
  const float vv = (float)(int)group_sum_u<GS>(V), ww = (float)(int)group_sum_u<GS>(W);
  return ww <= a.obj_f0 ? vv : a.obj_f0 - ww;
}

// Sparse bit-flip sampler, group-cooperative form: continue the sequence of
// mutation words at j with n distinct positions already flipped in fm (this
// lane's chunk q), until K distinct positions are flipped.  A candidate is a
// repeat iff its owner lane already has the bit: one ballot per candidate.
template <int GS, bool NH = false>
__device__ __forceinline__ uint4 sparse_continue(const GenArgs& a, uint64_t child, uint32_t K, uint32_t n, uint32_t j,
                                              uint4 fm, uint32_t q, uint32_t gbase) {
  u32x4 blk = draw<NH>(a.key, ST_BMUT, child, j >> 2);
  while (n < K) {  // group-uniform
    if ((j & 3u) == 0u) blk = draw<NH>(a.key, ST_BMUT, child, j >> 2);
    const uint32_t p = word_to_index(sel4(blk, j & 3u), a.L);
    ++j;
    const uint32_t b = p & 127u;
    const bool own = (p >> 7) == q;
    const uint32_t wd = sel4(u32x4{fm.x, fm.y, fm.z, fm.w}, b >> 5);
    unsigned long long bal = __ballot(own && ((wd >> (b & 31u)) & 1u));
    if (GS < 64) bal = (bal >> gbase) & ((1ull << GS) - 1ull);
    if (bal == 0ull) {
      if (own) fm = xor4(fm, bit4(b));
      ++n;
    }
  }
  return fm;
}

// Sparse bit-flip sampler, sequential form (the definition, cpu_ops.cpp
// sparse_positions): the first kk distinct word_to_index(mutation word j, L),
// packed as 16-bit positions (0xFFFF = none; positions are < kSparseMaxL);
// jn = the next unused word.
template <bool NH>
__device__ __forceinline__ uint4 sparse_seq(const RngKey& key, uint64_t child, uint32_t kk, uint32_t L, uint32_t& jn) {
  uint32_t w0 = 0xFFFFFFFFu, w1 = 0xFFFFFFFFu, w2 = 0xFFFFFFFFu, w3 = 0xFFFFFFFFu;
  uint32_t n = 0, j = 0;
  u32x4 blk{0, 0, 0, 0};
  while (n < kk) {
    if ((j & 3u) == 0u) blk = draw<NH>(key, ST_BMUT, child, j >> 2);
    const uint32_t p = word_to_index(sel4(blk, j & 3u), L);
    ++j;
    const bool seen = (w0 & 0xFFFFu) == p || (w0 >> 16) == p || (w1 & 0xFFFFu) == p || (w1 >> 16) == p ||
                      (w2 & 0xFFFFu) == p || (w2 >> 16) == p || (w3 & 0xFFFFu) == p || (w3 >> 16) == p;
    if (!seen) {
      const uint32_t sh = (n & 1u) * 16u, keep = ~(0xFFFFu << sh), v = p << sh, wi = n >> 1;
      w0 = wi == 0u ? (w0 & keep) | v : w0;
      w1 = wi == 1u ? (w1 & keep) | v : w1;
      w2 = wi == 2u ? (w2 & keep) | v : w2;
      w3 = wi == 3u ? (w3 & keep) | v : w3;
      ++n;
    }
  }
  jn = j;
  return make_uint4(w0, w1, w2, w3);
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
  const bool sparse = bitflip && a.mut_sparse;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (bitflip)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  const uint64_t stride = (uint64_t)gridDim.x * GPB;
  for (uint64_t child = (uint64_t)blockIdx.x * GPB + g_in_block; child < a.S; child += stride) {
    float score = 0.f;
    {
      // elitism: child = copy of the elite row, re-evaluated like every child
      const bool elite = MODE == MODE_GEN && child < a.n_elite;
      uint32_t pa = 0, pb = 0;
      bool xo = false;
      uint32_t blo = 0, bhi = 0;  // ONE/TWO_POINT: bits [blo, bhi) come from parent B
      u32x4 misc{0, 0, 0, 0};
      if (MODE == MODE_GEN || MODE == MODE_CROSS || MODE == MODE_MUTATE) misc = bin_misc(a.key, child);
      if (elite) {
        pa = pb = a.elite_idx ? a.elite_idx[child] : lds_elite;
      } else if (MODE == MODE_GEN || MODE == MODE_CROSS) {
        st_select_parents(a, child, pa, pb);
        xo = a.crossover != XO_NONE && do_crossover(a, misc.x);
        if (a.crossover == XO_ONE_POINT) {
          blo = word_to_index(misc.y, L);
          bhi = L;
        } else if (a.crossover == XO_TWO_POINT) {
          uint32_t c1 = word_to_index(misc.y, L);
          uint32_t c2 = word_to_index(misc.z, L);
          blo = c1 < c2 ? c1 : c2;
          bhi = c1 < c2 ? c2 : c1;
        }
      }
      uint32_t rpos = 0xFFFFFFFFu;  // RESET_ONE: the one flipped bit
      if (reset_one && !elite && misc.w < a.mut_ind_thresh) rpos = word_to_index(bin_mut_word(a.key, child, 0), L);
      uint4 fm = make_uint4(0, 0, 0, 0);  // sparse bit-flip: flips of chunk q (L <= 8192: one chunk per lane)
      if (sparse && !elite) fm = sparse_continue<GS>(a, child, binom_count(misc.w, lds_thr), 0, 0, fm, q, gbase);

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
        if (bitflip && !sparse && !elite) {
          v = xor4(v, u4(chunk_flip_mask(a, child, c, chunk_len(L, c), bin_chunk_mut_word(a.key, child, c), lds_thr)));
        } else if (sparse) {
          v = xor4(v, fm);
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
      st.add(score);
    }
  }
  if (EVALS && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}

// ---------------------------------------------------------------------------
// The hot generation kernel: transposed tournaments.
//
// A wave breeds NG = 64/GS children per STEP (group g: child bs + i*NG + g).
// Steps come in BATCHES of GS steps = 64 children, and the per-child work
// that does not touch the genome runs transposed, one lane per child of a
// whole batch.  A block owns a contiguous share of the population
// (tp_block_range), in ROUNDS of at most tp_par_cap children, each in two
// phases:
//   TOURNAMENTS  SEGMENTS of up to kSegBatches batches pulled from an LDS
//                counter, one per wave at a time: one Philox block = the 4
//                contestants of a child, all 4 x kSegBatches key loads in
//                flight together, compare -> (parent A, parent B) of every
//                child of the segment in LDS, then the segment's ready flag
//                (linear ranking: two rank picks, two rank-order loads)
//   BREED        UNITS of U <= 64 children pulled from a second counter once
//                no segment is left (a unit waits for its segment's flag):
//                RESOLVE the misc block (crossover test, cut points,
//                mutation count K) and the sparse bit-flip positions (one
//                more block, first K distinct by a pairwise check) -> a
//                32-byte child RECORD in the wave's LDS ring (2 batches);
//                per step: XO mask Philox (one block per chunk), mix, flips,
//                popcount, group butterfly, stores.
// Why two phases: the EA (L2 -> fabric) traffic is the bound (PMC: ~530 MB
// per generation at 1M x 1024 bits, ~5.7 TB/s).  Tournament keys are a 2 MB
// array read at random; interleaved with the row gathers, ~1/4 of the key
// reads missed the XCD's 4 MB L2 (a 128-B line each, ~1/4 of all EA bytes).
// At kernel start every wave is in its tournament phase, so the L2 holds
// little but key lines and the key reads cost ~2 MB of fabric per XCD.
// A child costs 3/64 of a Philox per lane for its child-level words, and
// mutation is a short loop over the record's positions instead of a
// divergent geometric search in every chunk.
// Why a counter: equal static shares per wave left the CU's youngest waves
// breeding alone for the last ~20 us (oldest-first issue, tp.hpp); pulled
// batches end every wave of a CU within about one batch of each other.
// ---------------------------------------------------------------------------

#ifdef PGA_TP_TIMING
// experiment builds only (tools/variants.sh): per-wave clocks of the two
// phases, wall-clock start / end and the XCD the wave ran on
__device__ unsigned long long pga_tp_clk[kMaxGrid * 4][8];
#endif

// kTpMaxElite (elites the fast kernel routes through its records),
// kSegBatches and the work units: tp.hpp

#ifndef PGA_TP_NOKEYS
#define PGA_TP_NOKEYS 0
#endif
// Small tail units (experiment builds: -DPGA_TP_SMALL=1): the last NW
// units' worth of a 16-wave block's round as 16-child units, so the CU's
// waves end within one small unit of each other.  Measured slower (round 5,
// interleaved A/B: 93.4 / 93.5 / 92.7 vs 91.8 / 91.7 / 92.3 us/gen on the
// driver's early generations, 90.3 vs 89.8 converged): a small unit's
// RESOLVE (64 lanes of child records for 16 children) and the refill of the
// PD-deep row pipeline at every unit cost more than the tail they remove.
#ifndef PGA_TP_SMALL
#define PGA_TP_SMALL 0
#endif

__device__ __forceinline__ uint32_t pos16(uint4 r1, uint32_t k) {  // k-th packed 16-bit position
  const uint32_t w = sel4(u32x4{r1.x, r1.y, r1.z, r1.w}, k >> 1);
  return (k & 1u) ? (w >> 16) : (w & 0xFFFFu);
}

// the uniform-crossover mask of chunk q of child c (ST_XO block q); experiment
// builds can swap in a multiplicative hash to measure the Philox's share
#ifdef PGA_TP_XOHASH
#define PGA_TP_XOMASK(c, q) make_uint4(mut_skip_word((c) * 4u, (q)), mut_skip_word((c) * 4u + 1u, (q)), \
                                       mut_skip_word((c) * 4u + 2u, (q)), mut_skip_word((c) * 4u + 3u, (q)))
#else
#define PGA_TP_XOMASK(c, q) u4(draw<true>(a.key, ST_XO, (c), (q)))
#endif

typedef uint32_t u32v4 __attribute__((ext_vector_type(4)));

template <int GS, int OBJ, bool FULL, bool DENSE>
__device__ __forceinline__ void binary_gen_tp_body(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  const uint32_t NW = blockDim.x >> 6;  // 4 or 16 waves (tp_dyn_lds of the launch)
  constexpr uint32_t NG = 64 / GS;      // children per wave per step
  constexpr uint32_t PD = tp_prefetch_depth(GS);  // steps of parent rows in flight (tp.hpp)
  constexpr bool EVALS = OBJ != OBJ_NONE;
  // integer objectives tournament on their exact u16 keys (L2-resident)
  constexpr bool KEY = OBJ == OBJ_ONEMAX || OBJ == OBJ_LEADING_ONES || OBJ == OBJ_TRAP;
  // dynamic LDS: per wave 2 batches x 64 records x 32 B, then the round's
  // (parent A, parent B) of every child
  uint4(*lds_rec)[2][64][2] = (uint4(*)[2][64][2])pga_dyn_lds;
  uint2* lds_par = (uint2*)(pga_dyn_lds + NW * 4096u);
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ uint32_t lds_el[kTpMaxElite];  // elite sources
  __shared__ unsigned long long lds_red[kTpMaxWaves];
  __shared__ uint32_t lds_next;   // the round's next unbred unit
  __shared__ uint32_t lds_tnext;  // the round's next tournament segment
  __shared__ uint32_t lds_role;   // the round's producer tickets (tp_producers)
  __shared__ uint32_t lds_ready[kTpMaxSegs];  // per segment: its parents are in LDS
  constexpr bool KMF = OBJ == kObjKnapMfma;
  __shared__ uint4 lds_kscr[KMF ? kTpMaxWaves : 1][kKnapScratch];      // knapsack: per-wave chunk / C scratch
  __shared__ uint4 lds_ktab[KMF ? kKnapSlices * 4 * kKnapMaxCols : 1];  // knapsack: digit table
  // JIT (a linked user objective): each step also stages its children's rows
  // in the wave's LDS slice (64 lanes x 16 B), and every kJitStageSteps steps
  // one lane per staged child runs the objective on its LDS row.  Reading the
  // rows back from global memory instead (round 3/4: once per unit) has to
  // wait for every load issued before it -- the parent rows in flight PD steps
  // ahead -- since vector memory counters retire in order: a drained pipeline
  // per unit (110.8 vs 89.8 us/gen); LDS reads wait on their own counter.
  constexpr bool JIT = OBJ == kObjJit;
  // fused key histogram (GenArgs::key_hist): an LDS histogram of the keys the
  // block writes, after the round's parents in dynamic LDS (the launcher adds
  // hist_bins words), flushed with one global atomic per non-empty bin
  constexpr bool HISTK = KEY && !JIT;

  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint32_t q = lane & (GS - 1), gbase = lane & ~(uint32_t)(GS - 1), g = lane / GS;
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  const uint32_t L = a.L, S = (uint32_t)a.S;
  // FULL: chunks == GS, every lane owns a chunk
  const bool have = FULL || q < a.chunks, last = q == a.chunks - 1;
  const uint32_t qq = have ? q : 0u;
  const uint32_t clen = have ? chunk_len(L, q) : 0u;
  const bool tourn = a.selection == SEL_TOURNAMENT;  // tour_k == 2 guaranteed by the launcher
  const bool rank = a.selection == SEL_RANK;
  const bool roul = a.selection == SEL_ROULETTE;     // else random
  const bool xo_on = a.crossover != XO_NONE;
  const bool range = a.crossover != XO_UNIFORM;  // ONE/TWO_POINT, or NONE (empty range)
  // DENSE: per-chunk geometric bit-flips; otherwise the record carries the
  // flip positions (sparse bit-flip, RESET_ONE, or none)
  const bool bitflip = a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f;
  const bool sparse = !DENSE && bitflip;
  const bool reset_one = !DENSE && a.mutation == MUT_RESET_ONE;
  const uint4 lmask = u4(a.last_mask);
  // Every row / score byte offset fits 32 bits (the launcher checks (S + pad)
  // rows < 4 GiB): uniform base + 32-bit lane offset, one VGPR per address
  const uint32_t rb = a.row_words * 4u;
#define ELEM(T, base, i) (*(T*)((char*)(base) + (uint32_t)(i) * (uint32_t)sizeof(T)))
#define ROW(base, row, ch) (*(uint4*)((char*)(base) + ((uint32_t)(row) * rb + (uint32_t)(ch) * 16u)))

  // this block's children [bbegin, bend) (tp.hpp)
  const uint32_t U = tp_unit(a, NG);  // children per breed unit (tp.hpp)
  constexpr uint32_t USMALL = PD * NG > 16u ? PD * NG : 16u;  // the round's tail units (a power of two <= 64)
  uint32_t bbegin, bend;
  tp_block_range(S, U, bbegin, bend, a.tp_skew);
  const uint32_t pcap = tp_par_cap(NW);
  // JIT staging after the parents: kJitStageSteps KB per wave (jit.cpp adds it to the launch's LDS)
  uint4* lds_stage = (uint4*)(pga_dyn_lds + NW * 4096u + pcap * 8u) + wid * (kJitStageSteps * 64u);
  (void)lds_stage;
  uint32_t* lds_hist = (uint32_t*)(pga_dyn_lds + NW * 4096u + pcap * 8u);  // (never with the JIT staging)
  const bool hist = HISTK && (a.key_hist != nullptr || a.rank_counts != nullptr);  // block-uniform
  const uint32_t hmax = a.hist_bins - 1u;
  // the pair pool (tp.hpp): one round, tournament or random selection; the
  // block's own units end at own_end, the last P units are the pair's
  const uint32_t P = a.tp_pool_units;
  bool pool_on = a.tp_pool != nullptr && P > 0u && bend - bbegin <= pcap && (tourn || a.selection == SEL_RANDOM);
  if (pool_on && a.n_elite > 0) {  // elites stay in block 0's own units (their sources are in its LDS)
    uint32_t b0b, b0e;
    tp_share(S, U, 0, b0b, b0e, a.tp_skew);
    pool_on = tp_pool_start(b0b, b0e, U, P) >= a.n_elite;
  }
  const uint32_t own_end = pool_on ? tp_pool_start(bbegin, bend, U, P) : bend;
  const uint32_t pair = blockIdx.x & ~1u, npair = pair + 1u < gridDim.x ? 2u : 1u;

  // The elite sources of children [0, n_elite) (n_elite <= kTpMaxElite, for
  // the block that holds any of them) and the mutation table are loaded by
  // wave 0 AFTER the round's first barrier and published by a flag that only
  // RESOLVE waits on: the tournaments never need them, and the barrier no
  // longer waits for their global round trips (nor block 0 for the reduction
  // of every block's best partial)
  __shared__ uint32_t lds_pro;  // 1: lds_el / lds_thr are loaded
  bool pro_ok = false;          // wave-uniform: this wave has seen lds_pro set
  if (KMF)
    for (uint32_t i = threadIdx.x; i < kKnapSlices * 4 * kKnapMaxCols; i += blockDim.x)
      lds_ktab[i] = ((const uint4*)a.knap_tab)[i];
  if (threadIdx.x == 0) lds_next = lds_tnext = lds_role = lds_pro = 0;
  if (threadIdx.x < kTpMaxSegs) lds_ready[threadIdx.x] = 0;
  if (hist) {
    for (uint32_t i = threadIdx.x; i < a.hist_bins; i += blockDim.x) lds_hist[i] = 0;
    if (a.hist_zero)  // a later generation's histogram starts from zero
      for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.hist_zero_words; i += gridDim.x * blockDim.x)
        a.hist_zero[i] = 0;
  }
  const uint32_t nprod = tp_producers(NW);

  unsigned long long my_best = 0;
  ScoreStats st;
  uint4(*rec)[64][2] = lds_rec[wid];
  static_assert(sizeof(lds_rec[0]) >= kSegBatches * 64 * sizeof(uint4), "contestant staging");
#ifdef PGA_TP_TIMING
  const unsigned long long clk0 = clock64(), rt0 = wall_clock64();
  unsigned long long clk_t = 0, clk_b = 0, n_bred = 0, clk_spin = 0;
#endif
  for (uint32_t rbeg = bbegin; rbeg < bend; rbeg += pcap) {  // block-uniform rounds
    const uint32_t rend0 = rbeg + pcap < bend ? rbeg + pcap : bend;
    const uint32_t rend = rend0 < own_end ? rend0 : own_end;                // the round's own children
    // the round's units: U children each (PGA_TP_SMALL: the last NW units'
    // worth of a 16-wave block as small units of USMALL >= PD steps)
    const uint32_t nu = (rend - rbeg + U - 1) / U;
    const bool tail_small = PGA_TP_SMALL && USMALL < U && NW == kTpMaxWaves && !pool_on && nu >= 2u * NW;
    const uint32_t nbig = tail_small ? nu - NW : nu;
    const uint32_t nb = nbig + (tail_small ? (rend - rbeg - nbig * U + USMALL - 1) / USMALL : 0u);
    const uint32_t nseg = (rend - rbeg + kSegBatches * 64 - 1) / (kSegBatches * 64);  // its tournament segments
    __syncthreads();  // tables / counters visible; the previous round's records and parents released
#ifdef PGA_TP_TIMING
    const unsigned long long clkA = clock64();
#endif
    if (rbeg == bbegin && wid == 0) {  // wave-uniform: the prologue loads (lds_pro)
      if (a.n_elite > 0 && bbegin < a.n_elite) {
        if (a.elite_idx) {
          for (uint32_t i = lane; i < a.n_elite; i += 64) lds_el[i] = a.elite_idx[i];
        } else {
          const unsigned long long b = wave_reduce_parts(a.best_cur, a.n_best_cur);
          if (lane == 0) lds_el[0] = (uint32_t)best_index(b);
        }
      }
      if (bitflip)
        for (uint32_t i = lane; i < kMutCap; i += 64) lds_thr[i] = a.mut_thr[i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      tp_flag_set(&lds_pro);
    }

    // TOURNAMENTS of the round, one segment of <= kSegBatches batches at a
    // time per wave, segments pulled from a counter: all key loads of a
    // segment in flight at once; the contestants wait in the wave's record
    // ring (free until it breeds).  A wave breeds as soon as no segment is
    // left; a unit's RESOLVE waits for its segment's flag (no block barrier)
    const bool produce = nprod >= NW || tp_ticket(&lds_role, lane) < nprod;  // wave-uniform
    while (produce) {
      const uint32_t sg = tp_ticket(&lds_tnext, lane);
      if (sg >= nseg) break;
      const uint32_t begin = rbeg + sg * kSegBatches * 64u;
      const uint32_t end = begin + kSegBatches * 64u < rend ? begin + kSegBatches * 64u : rend;
      uint2* par = lds_par + sg * kSegBatches * 64u;
      // the contestants wait in the wave's record ring (4 x 64 x 16 B = its
      // 4 KiB, free until it breeds); every key load of the segment in flight
      // at once (tp.hpp, the one definition shared with real_gen_tp)
      tp_select_segment<KEY ? (PGA_TP_NOKEYS ? TP_NOKEY : TP_KEY16) : TP_F32>(a, begin, end, lane, &rec[0][0][0], par);
      // publish: the segment's parents (this wave's LDS stores, in order)
      // before its flag
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      tp_flag_set(&lds_ready[sg]);
    }
    // several blocks per CU (the 4-wave grid): a barrier parks the waiting
    // waves (a flag spin would take issue slots from the other blocks' waves:
    // REAL at S = 100K, 36 -> 55 us/gen); one block per CU: the flags alone
    if (NW < kTpMaxWaves) __syncthreads();
#ifdef PGA_TP_TIMING
    const unsigned long long clkB = clock64();
    clk_t += clkB - clkA;
#endif

#ifdef PGA_TP_TIMING
#define PGA_TP_SPIN0 const unsigned long long sp0_ = clock64();
#define PGA_TP_SPIN1 clk_spin += clock64() - sp0_;
#else
#define PGA_TP_SPIN0
#define PGA_TP_SPIN1
#endif
    // RESOLVE: parents, crossover plan and flip positions of the round's unit
    // BI -> the records of ring slot SL (lanes past the unit: unused copies)
#define PGA_TP_RESOLVE(US, UE, SL)                                                                              \
  {                                                                                                             \
    if (!pro_ok) { /* the prologue loads of wave 0 (once per wave) */                                          \
      while (__hip_atomic_load(&lds_pro, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)                 \
        __builtin_amdgcn_s_sleep(1);                                                                            \
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");                                                    \
      pro_ok = true;                                                                                            \
    }                                                                                                           \
    const uint32_t tc = (US) + lane;                                                                            \
    const uint32_t cc = tc < (UE) ? tc : (UE) - 1;                                                              \
    uint32_t pa, pb;                                                                                            \
    if ((US) - rbeg < rend - rbeg) { /* an own unit: parents from the round's tournaments */                    \
      /* its segment is done (wave-uniform spin, rare) */                                                       \
      const uint32_t sg_ = ((US) - rbeg) / (kSegBatches * 64u);                                                 \
      PGA_TP_SPIN0                                                                                              \
      while (__hip_atomic_load(&lds_ready[sg_], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)          \
        __builtin_amdgcn_s_sleep(1);                                                                            \
      PGA_TP_SPIN1                                                                                              \
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");                                                    \
      const uint2 pp = lds_par[cc - rbeg];                                                                      \
      pa = pp.x;                                                                                                \
      pb = pp.y;                                                                                                \
    } else { /* a pool unit: its tournaments here, one lane per child (same words) */                           \
      const u32x4 sb = draw<true>(a.key, ST_SEL, cc, 0);                                                        \
      const uint32_t i0 = word_to_index(sb.x, S), i1 = word_to_index(sb.y, S);                                  \
      const uint32_t i2 = word_to_index(sb.z, S), i3 = word_to_index(sb.w, S);                                  \
      pa = i0;                                                                                                  \
      pb = i1;                                                                                                  \
      if (tourn) {                                                                                              \
        if constexpr (KEY) {                                                                                    \
          const uint32_t q0 = ELEM(const uint16_t, a.key_cur, i0), q1 = ELEM(const uint16_t, a.key_cur, i1);    \
          const uint32_t q2 = ELEM(const uint16_t, a.key_cur, i2), q3 = ELEM(const uint16_t, a.key_cur, i3);    \
          pa = q0 < q1 ? i1 : i0;                                                                               \
          pb = q2 < q3 ? i3 : i2;                                                                               \
        } else {                                                                                                \
          const float f0 = ELEM(const float, a.score_cur, i0), f1 = ELEM(const float, a.score_cur, i1);         \
          const float f2 = ELEM(const float, a.score_cur, i2), f3 = ELEM(const float, a.score_cur, i3);         \
          pa = f0 < f1 ? i1 : i0;                                                                               \
          pb = f2 < f3 ? i3 : i2;                                                                               \
        }                                                                                                       \
      }                                                                                                         \
    }                                                                                                           \
    const u32x4 misc = bin_misc<true>(a.key, cc);                                                               \
    const bool elite = tc < a.n_elite;                                                                          \
    const bool xo = !elite && xo_on && do_crossover(a, misc.x);                                                 \
    if (elite) pa = lds_el[tc];                                                                                 \
    pb = xo ? pb : pa;                                                                                          \
    uint32_t lo = 0, hi = 0;                                                                                    \
    if (range && xo) {                                                                                          \
      const uint32_t x1 = word_to_index(misc.y, L);                                                             \
      if (a.crossover == XO_ONE_POINT) {                                                                        \
        lo = x1;                                                                                                \
        hi = L;                                                                                                 \
      } else {                                                                                                  \
        const uint32_t x2 = word_to_index(misc.z, L);                                                           \
        lo = x1 < x2 ? x1 : x2;                                                                                 \
        hi = x1 < x2 ? x2 : x1;                                                                                 \
      }                                                                                                         \
    }                                                                                                           \
    uint32_t K = 0, jn = 0;                                                                                     \
    uint4 P = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);                                   \
    if (reset_one && !elite && misc.w < a.mut_ind_thresh) {                                                     \
      K = 1;                                                                                                    \
      P.x = word_to_index(bin_mut_word<true>(a.key, cc, 0), L) | 0xFFFF0000u;                                   \
    }                                                                                                           \
    if (sparse && !elite) {                                                                                     \
      K = binom_count(misc.w, lds_thr);                                                                         \
      if (K > 0u) {                                                                                             \
        const uint32_t kk = K < kRecPos ? K : kRecPos;                                                          \
        const u32x4 m0 = draw<true>(a.key, ST_BMUT, cc, 0);                                                     \
        const uint32_t c0 = word_to_index(m0.x, L), c1 = word_to_index(m0.y, L);                                \
        const uint32_t c2 = word_to_index(m0.z, L), c3 = word_to_index(m0.w, L);                                \
        /* common case: the first kk <= 4 candidates are distinct, hence the positions */                      \
        const bool slow = kk > 4u || (kk > 1u && c0 == c1) || (kk > 2u && (c2 == c0 || c2 == c1)) ||            \
                          (kk > 3u && (c3 == c0 || c3 == c1 || c3 == c2));                                      \
        P = make_uint4(c0 | (c1 << 16), c2 | (c3 << 16), 0xFFFFFFFFu, 0xFFFFFFFFu);                             \
        jn = kk;                                                                                                \
        if (slow) P = sparse_seq<true>(a.key, cc, kk, L, jn);                                                   \
      }                                                                                                         \
    }                                                                                                           \
    const uint32_t meta = (K > 255u ? 255u : K) | ((jn > 0xFFFFu ? 0xFFFFu : jn) << 8) | (elite ? 1u << 31 : 0u); \
    uint4(*r)[2] = rec[(SL)];                                                                                   \
    r[lane][0] = make_uint4(pa, pb, lo | (hi << 16), meta);                                                     \
    r[lane][1] = P;                                                                                             \
  }

    // BREED: the round's units in ticket order from the block's counter, as
    // two cursors over the wave's sequence of steps: the LOAD cursor issues
    // the parent-row loads of the step PD steps ahead of the BREED cursor
    // (PD register sets in flight: the row gathers are latency-bound, so the
    // bytes in flight per wave set the throughput) and RESOLVEs a unit into
    // the other ring slot when it enters it (a full unit has U / NG >= PD
    // steps, so the breed cursor has left that slot by then).  Every vector
    // memory operation is unconditional (s_waitcnt vmcnt retires in order and
    // hipcc assumes the fewest outstanding loads over all paths, so a
    // conditionally issued load would make the next wait drain it): an
    // exhausted load cursor re-reads the breed cursor's rows.
    // NEXT unit [US, UE) of this wave (US = kNoUnit: none): the block's own
    // units from its LDS counter, then pool units from the pair's counter
    constexpr uint32_t kNoUnit = 0xFFFFFFFFu;
    bool steal = false;  // wave-uniform: own units exhausted, pulling pool units
#define PGA_TP_NEXT(US, UE, UN)                                                                             \
  {                                                                                                         \
    US = kNoUnit;                                                                                           \
    UN = U / NG;                                                                                            \
    if (!steal) {                                                                                           \
      const uint32_t tk_ = tp_ticket(&lds_next, lane);                                                      \
      if (tk_ < nbig) {                                                                                     \
        US = rbeg + tk_ * U;                                                                                \
        UE = US + U < rend ? US + U : rend;                                                                 \
      } else if (tk_ < nb) { /* a small tail unit */                                                        \
        US = rbeg + nbig * U + (tk_ - nbig) * USMALL;                                                       \
        UE = US + USMALL < rend ? US + USMALL : rend;                                                       \
        UN = USMALL / NG;                                                                                   \
      } else {                                                                                              \
        steal = pool_on;                                                                                    \
      }                                                                                                     \
    }                                                                                                       \
    while (steal && US == kNoUnit) { /* ticket t: block pair + t % npair, its pool unit t / npair */       \
      const uint32_t t_ = tp_pool_grab(a.tp_pool + (pair >> 1) * kTpPoolStride, a.tp_seq, lane);            \
      if (t_ / npair >= P) {                                                                                \
        steal = false;                                                                                      \
      } else {                                                                                              \
        uint32_t pb_, pe_;                                                                                  \
        tp_share(S, U, pair + t_ % npair, pb_, pe_, a.tp_skew);                                             \
        const uint32_t ps_ = tp_pool_start(pb_, pe_, U, P) + (t_ / npair) * U;                             \
        if (ps_ < pe_) {                                                                                    \
          US = ps_;                                                                                         \
          UE = ps_ + U < pe_ ? ps_ + U : pe_;                                                               \
        }                                                                                                   \
      }                                                                                                     \
    }                                                                                                       \
  }

    uint32_t ns, ne = 0, nn = 0;  // the wave's next unit and its steps (prefetched ticket)
    PGA_TP_NEXT(ns, ne, nn)
    if (ns != kNoUnit) {
      // breed cursor: ring slot, step, its unit [bs, be) and steps.  Every
      // unit takes its full size / NG steps, a partial one (only ever at S)
      // too: its children past S write the padding rows, and a unit never
      // holds fewer steps than the PD the load cursor runs ahead
      uint32_t nst = nn;
      uint32_t slot = 0, i = 0, bs = ns, be = ne;
      PGA_TP_NEXT(ns, ne, nn)
      PGA_TP_RESOLVE(bs, be, 0u)
      // load cursor; lpend: at the end of its unit with unit ns next;
      // lmore = false: past the wave's last step
      uint32_t lslot = 0, li = 0, lbs = bs, lbe = be, lnst = nst;
      bool lpend = false, lmore = true, done = false;

      // LOAD the parent rows of the load cursor's step into (YA, YB) and
      // advance it
#define PGA_TP_LOAD(YA, YB)                                                                                 \
  {                                                                                                         \
    if (lpend) { /* entering the next unit */                                                               \
      PGA_TP_RESOLVE(ns, ne, lslot ^ 1u)                                                                    \
      lslot ^= 1u;                                                                                          \
      li = 0;                                                                                               \
      lbs = ns;                                                                                             \
      lbe = ne;                                                                                             \
      lnst = nn;                                                                                            \
      lpend = false;                                                                                        \
      PGA_TP_NEXT(ns, ne, nn)                                                                               \
    }                                                                                                       \
    const uint4 r = rec[lmore ? lslot : slot][(lmore ? li : i) * NG + g][0];                                \
    YA = ROW(cur, r.x, qq);                                                                                 \
    YB = ROW(cur, r.y, qq);                                                                                 \
    if (lmore && ++li == lnst) {                                                                            \
      lpend = ns != kNoUnit;                                                                                \
      lmore = lpend;                                                                                        \
    }                                                                                                       \
  }

      // one STEP: load PD steps ahead into (YA, YB), breed the breed cursor's
      // step i from (XA, XB) (its children past S, at the population's end
      // only, write the padding rows), advance the breed cursor
#define PGA_TP_STEP(XA, XB, YA, YB)                                                                         \
  {                                                                                                         \
    PGA_TP_LOAD(YA, YB)                                                                                     \
    const uint32_t c = bs + i * NG + g;                                                                     \
    const uint4 r0 = rec[slot][i * NG + g][0];                                                              \
    const uint32_t meta = r0.w;                                                                             \
    const uint4 m = range ? range_keep_a(q, r0.z & 0xFFFFu, r0.z >> 16) : PGA_TP_XOMASK(c, q);               \
    uint4 v = mix4(XA, XB, m);                                                                              \
    if (last) v = and4(v, lmask);                                                                           \
    uint4 fm = make_uint4(0, 0, 0, 0);                                                                      \
    if (DENSE) {                                                                                            \
      if (bitflip && !(meta >> 31)) /* elites are not mutated */                                           \
        fm = u4(chunk_flip_mask(a, c, q, clen, bin_chunk_mut_word<true>(a.key, c, q), lds_thr));            \
    } else {                                                                                                \
      const uint32_t K = meta & 0xFFu;                                                                      \
      if (K > 0u) {                                                                                         \
        const uint4 r1 = rec[slot][i * NG + g][1];                                                          \
        const uint32_t kk = K < kRecPos ? K : kRecPos;                                                      \
        /* the first 4 unrolled (a loop here costs ~20 VGPRs of the whole kernel) */                       \
        _Pragma("unroll") for (uint32_t k = 0; k < 4; ++k) {                                               \
          const uint32_t p = pos16(r1, k);                                                                  \
          if (k < kk && (p >> 7) == q) fm = xor4(fm, bit4(p & 127u));                                       \
        }                                                                                                   \
        if (kk > 4u)                                                                                        \
          for (uint32_t k = 4; k < kk; ++k) {                                                               \
            const uint32_t p = pos16(r1, k);                                                                \
            if ((p >> 7) == q) fm = xor4(fm, bit4(p & 127u));                                              \
          }                                                                                                 \
        if (K > kRecPos) fm = sparse_continue<GS, true>(a, c, K, kRecPos, (meta >> 8) & 0xFFFFu, fm, q, gbase); \
      }                                                                                                     \
    }                                                                                                       \
    v = xor4(v, fm);                                                                                        \
    float sc;                                                                                               \
    if constexpr (KMF) {                                                                                    \
      sc = knap_mfma<GS>(a, have ? v : make_uint4(0, 0, 0, 0), lane, q, lds_kscr[wid], lds_ktab);            \
    } else if constexpr (JIT) {                                                                             \
      sc = 0.f; /* evaluated after the unit */                                                              \
    } else {                                                                                                \
      BinObj<OBJ> acc;                                                                                      \
      if (have) acc.add(a, v, q);                                                                           \
      sc = acc.template finish<GS>(a);                                                                      \
    }                                                                                                       \
    if (have) {                                                                                             \
      if (a.nt_store) /* block-uniform */                                                                   \
        __builtin_nontemporal_store(__builtin_bit_cast(u32v4, v), (u32v4*)&ROW(nxt, c, q));                 \
      else                                                                                                  \
        ROW(nxt, c, q) = v;                                                                                 \
    }                                                                                                       \
    if constexpr (JIT) {                                                                                    \
      lds_stage[(i % kJitStageSteps) * 64u + lane] = v;                                                     \
      if (i % kJitStageSteps == kJitStageSteps - 1u || i + 1u == nst) PGA_TP_JIT_EVAL                       \
    }                                                                                                       \
    if (EVALS && !JIT) { /* every lane of the group stores the same score */                                \
      ELEM(float, a.score_next, c) = sc;                                                                    \
      if (KEY) ELEM(uint16_t, a.key_next, c) = (uint16_t)sc;                                                \
      if (hist && q == 0u && c < S) {                                                                       \
        const uint32_t kb = (uint16_t)sc;                                                                   \
        __hip_atomic_fetch_add(&lds_hist[kb < hmax ? kb : hmax], 1u, __ATOMIC_RELAXED,                      \
                               __HIP_MEMORY_SCOPE_WORKGROUP);                                               \
      }                                                                                                     \
      const unsigned long long pk = c < S ? pack_best(sc, c) : 0ull;                                        \
      my_best = pk > my_best ? pk : my_best;                                                                \
      st.add_if(q == 0u && c < S, sc);                                                                      \
    }                                                                                                       \
    if (++i == nst) {                                                                                       \
      PGA_TP_COUNT                                                                                          \
      if (lbs == bs) { /* the load cursor never left this unit: it was the wave's last */                   \
        done = true;                                                                                        \
      } else {                                                                                              \
        slot ^= 1u;                                                                                         \
        i = 0;                                                                                              \
        bs = lbs;                                                                                           \
        be = lbe;                                                                                           \
        nst = lnst;                                                                                         \
      }                                                                                                     \
    }                                                                                                       \
  }

      // JIT: the staged steps s0..i of the unit, child j = lane (step s0 + j / NG,
      // group j % NG); the wavefront fences keep the compiler from moving LDS
      // accesses across (one wave's LDS operations execute in order)
#define PGA_TP_JIT_EVAL                                                                                     \
  {                                                                                                         \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");                                                  \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");                                                  \
    const uint32_t s0 = i - i % kJitStageSteps, ns = i - s0 + 1u;                                           \
    const uint32_t cj = bs + s0 * NG + lane;                                                                \
    if (lane < ns * NG && cj < be) {                                                                        \
      const uint32_t js = lane / NG, jg = lane % NG;                                                        \
      const float sj = pga_user_objective((pga_lds_words)(lds_stage + js * 64u + jg * GS), L, a.obj_data);  \
      ELEM(float, a.score_next, cj) = sj;                                                                   \
      my_best = pack_best(sj, cj) > my_best ? pack_best(sj, cj) : my_best;                                  \
      st.add(sj);                                                                                           \
    }                                                                                                       \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");                                                  \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");                                                  \
  }
#ifdef PGA_TP_TIMING
#define PGA_TP_COUNT n_bred += be - bs;
#else
#define PGA_TP_COUNT
#endif

      uint4 A0, B0, A1, B1, A2, B2, A3, B3;  // PD + 1 register sets, rotated statically
      (void)A2; (void)B2; (void)A3; (void)B3;
      if constexpr (PD == 1) {
        PGA_TP_LOAD(A0, B0)
        for (;;) {
          PGA_TP_STEP(A0, B0, A1, B1)
          if (done) break;
          PGA_TP_STEP(A1, B1, A0, B0)
          if (done) break;
        }
      } else if constexpr (PD == 2) {
        PGA_TP_LOAD(A0, B0)
        PGA_TP_LOAD(A1, B1)
        for (;;) {
          PGA_TP_STEP(A0, B0, A2, B2)
          if (done) break;
          PGA_TP_STEP(A1, B1, A0, B0)
          if (done) break;
          PGA_TP_STEP(A2, B2, A1, B1)
          if (done) break;
        }
      } else {
        PGA_TP_LOAD(A0, B0)
        PGA_TP_LOAD(A1, B1)
        PGA_TP_LOAD(A2, B2)
        for (;;) {
          PGA_TP_STEP(A0, B0, A3, B3)
          if (done) break;
          PGA_TP_STEP(A1, B1, A0, B0)
          if (done) break;
          PGA_TP_STEP(A2, B2, A1, B1)
          if (done) break;
          PGA_TP_STEP(A3, B3, A2, B2)
          if (done) break;
        }
      }
#undef PGA_TP_STEP
#undef PGA_TP_LOAD
#undef PGA_TP_NEXT
#undef PGA_TP_JIT_EVAL
#undef PGA_TP_COUNT
    }
#undef PGA_TP_RESOLVE
#undef PGA_TP_SPIN0
#undef PGA_TP_SPIN1
#ifdef PGA_TP_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this round's stores issued and done
    clk_b += clock64() - clkB;
#endif
    __syncthreads();  // every wave out of the round's counters before they are reset
    if (threadIdx.x == 0) lds_next = lds_tnext = lds_role = 0;
    if (threadIdx.x < kTpMaxSegs) lds_ready[threadIdx.x] = 0;
  }
#undef ROW
#undef ELEM
#ifdef PGA_TP_TIMING
  if (lane == 0 && blockIdx.x * NW + wid < kMaxGrid * 4) {
    const uint32_t wv = blockIdx.x * NW + wid;
    pga_tp_clk[wv][0] = clk_t;
    pga_tp_clk[wv][1] = clk_b;
    pga_tp_clk[wv][2] = clock64() - clk0;
    pga_tp_clk[wv][3] = n_bred;
    pga_tp_clk[wv][4] = rt0;
    pga_tp_clk[wv][5] = wall_clock64();
    pga_tp_clk[wv][6] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
    pga_tp_clk[wv][7] = clk_spin;  // cycles a breeding wave waited for a segment's flag
  }
#endif
  if (hist)  // every wave passed the last round's barrier: the block's counts are complete
    for (uint32_t i = threadIdx.x; i < a.hist_bins; i += blockDim.x) {
      const uint32_t v = lds_hist[i];
      if (a.key_hist && v) __hip_atomic_fetch_add(&a.key_hist[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.rank_counts) a.rank_counts[i * gridDim.x + blockIdx.x] = v;  // this block's sort tile
    }
  if (EVALS && best_parts) {  // block-uniform
    unsigned long long bb = block_max_u64_n(my_best, lds_red, NW);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = bb;
    if (a.stats_parts) block_stats_store_n(st, a.stats_parts, NW);
  }
}

// 16-wave blocks (one per CU) for the headline launch and 4-wave blocks for
// small populations; 128 VGPRs either way (the breed phase measured alike at
// 4 and 5 waves per SIMD: the fabric is the bound)
template <int GS, int OBJ, bool FULL, bool DENSE>
__global__ __launch_bounds__(kTpMaxWaves * 64) void binary_gen_tp(GenArgs a, unsigned long long* best_parts) {
  binary_gen_tp_body<GS, OBJ, FULL, DENSE>(a, best_parts);
}

// ---------------------------------------------------------------------------
// Persistent multi-generation launch (the headline geometry only: one
// 16-wave block per CU, every block resident at once): G generations of the
// same island in ONE launch, a device-wide barrier between them in place of
// the kernel boundary, so the next generation's blocks start together the
// moment the barrier drops instead of re-entering one by one through the
// dispatcher (the launch ramp: the last of 4096 waves started 3.4-4 us after
// the first, pmc_r05.md).  The barrier does what the kernel boundary did for
// memory: every block's stores leave its XCD's L2 (agent-scope release) before
// it arrives, and every block drops stale L2 lines (agent-scope acquire) once
// all have arrived; the next generation reads the population just written.
// Integer objectives with tournament / random selection, elitism <= 1, no
// fused histogram (the launcher checks).  Generation i writes parts[i & 1] and
// stats[i & 1], so the host's parity bookkeeping is that of G plain launches.
// ---------------------------------------------------------------------------
struct GenMulti {
  GenArgs a;                     // generation 0
  unsigned long long* parts[2];  // best partials written by even / odd generations
  float* stats[2];               // {min, sum} partials likewise (nullptr: none)
  uint32_t gens;
  uint32_t* bar;  // arrival counter, zero at launch; generation i's barrier waits for grid * (i + 1)
  uint32_t* hist[3];  // fused key histograms, rotated as Island::run_plain does (hist[0] nullptr: off)
  uint32_t hist_rot;
};

__device__ __forceinline__ void tp_grid_sync(uint32_t* bar, uint32_t target) {
  __syncthreads();  // every wave's stores of the generation are in the L2 (workgroup release)
  if (threadIdx.x < 64u) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // ... and out of this XCD's L2
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // bounded: a grid that is not co-resident (never expected: the launcher
      // takes one block per CU) would otherwise hang the device
      for (uint32_t spins = 0; spins < (1u << 24); ++spins) {
        if (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // no stale line of the new population survives
  }
  __syncthreads();
}

template <int GS, int OBJ, bool FULL, bool DENSE>
__global__ __launch_bounds__(kTpMaxWaves * 64) void binary_gen_tp_multi(GenMulti m) {
  GenArgs a = m.a;
  for (uint32_t i = 0;; ++i) {
    a.stats_parts = m.stats[i & 1u];
    if (m.hist[0]) {
      a.key_hist = m.hist[(m.hist_rot + i) % 3u];
      a.hist_zero = m.hist[(m.hist_rot + i + 1u) % 3u];
    }
    binary_gen_tp_body<GS, OBJ, FULL, DENSE>(a, m.parts[i & 1u]);
    if (i + 1u >= m.gens) break;
    tp_grid_sync(m.bar, gridDim.x * (i + 1u));
    // the population just written is the next generation's current one
    const void* c = a.cur;
    a.cur = a.next;
    a.next = const_cast<void*>(c);
    const float* sc = a.score_cur;
    a.score_cur = a.score_next;
    a.score_next = const_cast<float*>(sc);
    const uint16_t* kc = a.key_cur;
    a.key_cur = a.key_next;
    a.key_next = const_cast<uint16_t*>(kc);
    a.best_cur = m.parts[i & 1u];
    a.n_best_cur = gridDim.x;
    ++a.key.gen;
  }
}

// ---------------------------------------------------------------------------
// Batched islands: up to kMaxBatch same-shape islands of one device in ONE
// launch, island = blockIdx.y (its GenArgs and best partials from the kernel
// argument block), blockIdx.x / gridDim.x the island's own grid.  Many small
// islands on separate streams are launch-bound and share the process's 4
// hardware queues; one launch fills the device with all of them.  The
// reference's islands are at most MAX_POPULATIONS = 10 per solver
// (include/pga.h:44), run serially (src/pga.cu:272-276).
// ---------------------------------------------------------------------------
constexpr uint32_t kMaxBatch = 10;
struct GenBatch {
  GenArgs a[kMaxBatch];
  unsigned long long* parts[kMaxBatch];
};

template <int GS, int OBJ, bool FULL, bool DENSE>
__global__ __launch_bounds__(kTpMaxWaves * 64) void binary_gen_tp_batch(GenBatch b) {
  binary_gen_tp_body<GS, OBJ, FULL, DENSE>(b.a[blockIdx.y], b.parts[blockIdx.y]);
}

}  // namespace (jitgen / anonymous)
}  // namespace pga
