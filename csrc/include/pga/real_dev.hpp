// real_dev.hpp — the REAL encoding's two-phase generation kernel
// (real_gen_tp, the binary_gen_tp design) and its device helpers.  Included
// by real.hip (the built-in objectives and the launchers) and by
// jitgen_real.hip (real_gen_tp with a user objective linked in, OBJ_JIT).
#pragma once
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/real_ops.hpp"
#include "pga/tp.hpp"

// The user objective of a fused JIT generation kernel (jitgen_real.hip):
// defined in the user's bitcode, LTO-linked with the kernel's bitcode and
// inlined (jit.cpp).  The genes are the child's row as the step staged it in
// LDS next to its global store (binary_dev.hpp: the same staging, and why).
typedef __attribute__((address_space(3))) const float* pga_lds_floats;
extern "C" __device__ float pga_user_objective_f32(pga_lds_floats genes, unsigned int n, const float* data);

namespace pga {
// jitgen_real.hip instantiates the kernel with external linkage (a named
// namespace) so it keeps a predictable symbol in the bitcode; everywhere else
// the device code stays TU-local
#ifdef PGA_JIT_GEN
namespace jitgen {
#else
namespace {
#endif

using namespace dev;
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int GS>
__device__ __forceinline__ float group_prod(float v) {
#pragma unroll
  for (int o = GS / 2; o > 0; o >>= 1) v *= __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float gene4(const float v[4], uint32_t b) {
  return fsel(b == 0, v[0], fsel(b == 1, v[1], fsel(b == 2, v[2], v[3])));
}
__device__ __forceinline__ void set_gene4(float v[4], uint32_t b, float x) {
  v[0] = fsel(b == 0, x, v[0]);
  v[1] = fsel(b == 1, x, v[1]);
  v[2] = fsel(b == 2, x, v[2]);
  v[3] = fsel(b == 3, x, v[3]);
}

// Sparse per-gene mutation, group-cooperative form: continue the sequence of
// mutation words at j with n distinct genes already mutated (mm = this lane's
// mask of mutated genes of its chunk q), until K distinct genes are mutated.
// A candidate is a repeat iff its owner lane already mutated it: one ballot
// per candidate.  The owner applies the n-th value.  Same result as the
// sequential definition (cpu_real.cpp).
template <int GS, bool NH = false>
__device__ __forceinline__ void real_sparse_group(const GenArgs& a, uint64_t child, uint32_t K, uint32_t n, uint32_t j,
                                                  uint32_t& mm, uint32_t q, uint32_t gbase, float v[4]) {
  u32x4 blk{0u, 0u, 0u, 0u};
  if (j & 3u) blk = draw<NH>(a.key, ST_BMUT, child, j >> 2);
  while (n < K) {  // group-uniform
    if ((j & 3u) == 0u) blk = draw<NH>(a.key, ST_BMUT, child, j >> 2);
    const uint32_t p = word_to_index(sel4(blk, j & 3u), a.L);
    ++j;
    const bool own = (p >> 2) == q;
    const uint32_t b = p & 3u;
    unsigned long long bal = __ballot(own && ((mm >> b) & 1u));
    if (GS < 64) bal = (bal >> gbase) & ((1ull << GS) - 1ull);
    if (bal == 0ull) {
      if (own) {
        set_gene4(v, b, real_mut_apply(a, real_mut_draw<NH>(a, child, n), gene4(v, b)));
        mm |= 1u << b;
      }
      ++n;
    }
  }
}

// ---------------------------------------------------------------------------
// The hot generation kernel: transposed tournaments (the binary_gen_tp design,
// binary_dev.hpp).  A wave breeds NG = 64/GS children per STEP; a block owns
// a contiguous share of the population, in rounds (tp.hpp tp_block_range):
//   TOURNAMENTS  tp_select_segment (tp.hpp): one lane per child, every f32
//                score load of a 256-child segment in flight together
//   BREED        UNITS of U <= 64 children pulled from the block's LDS
//                counter once no segment is left (a unit waits for its
//                segment's ready flag); per unit, RESOLVE (one lane
//                per child): the misc block
//                (crossover test, cut points / arithmetic u, mutation count
//                K), the first min(K, 3) distinct mutation positions and
//                their values (gaussian z by gauss_z) -> a 32-byte child
//                RECORD in the wave's LDS ring (2 units); per step: parent
//                rows loaded PD steps ahead, crossover (BLX: one Philox block
//                per lane), the record's mutations (K > 3: the group
//                continues the sequence), objective, group butterfly, stores.
// So a child costs 2 Philox blocks of child-level words computed once (not
// one pool block per lane) plus BLX's per-gene uniforms, and the per-gene
// mutation test is a K-position loop instead of a per-lane geometric search.
// Every vector memory operation is unconditional (hipcc's s_waitcnt vmcnt
// accounting otherwise assumes the fewest outstanding loads over all paths).
//
// Record: [0] = {parent A, parent B, crossover plan word, meta}
//         [1] = {3 positions (u8), mutation draws 0..2 (f32 bits)}
// meta: K (8 bits) | next mutation word j (16 bits) << 8 | xo << 30 | elite << 31
//
// ROT (GS 4 or 8, L <= 32): rotated objective f(M (x - o)) on the matrix
// cores, wave-local: the wave's 64/GS children are transposed through a
// private 16 x 36 LDS tile and multiplied by M^T with v_mfma_f32_4x4x1_16b_f32
// (rot_tile4: 16 independent 4x4 blocks = 64/GS children x 4 GS dims, no
// wasted rows), the same k-ordered fma chain as the CPU reference.
// ---------------------------------------------------------------------------
constexpr uint32_t kRotTW = 36;  // tile row stride (floats): conflict-free column reads, 16-byte rows

__device__ __forceinline__ void rot_tile4_sync() { wave_lds_sync(); }

// z (4 genes of this lane's chunk, shifted) -> rotated z, in place.  One k
// per instruction: each output is the same sequential fma chain as the CPU
// reference.  A = X[child][k] and B = M[n][k] come from LDS as dwordx4 runs
// of 4 k (xw: this wave's tile, ms: the block's M tile, row stride kRotTW).
template <int GS>
__device__ __forceinline__ void rot_tile4(float* xw, const float* ms, float z[4]) {
  constexpr int DP = 4 * GS;
  const uint32_t lane = lane_id();
  const uint32_t row = lane / GS, q = lane % GS;
  const uint32_t b = lane >> 2, rg = b / GS, cg = b % GS;
  const uint32_t ca = 4 * rg + (lane & 3);   // A row (child) of this lane
  const uint32_t nb = 4 * cg + (lane & 3);   // B column (output dim) of this lane
  *(float4*)(xw + row * kRotTW + 4 * q) = make_float4(z[0], z[1], z[2], z[3]);
  rot_tile4_sync();
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k4 = 0; k4 < DP / 4; ++k4) {
    const float4 xa = *(const float4*)(xw + ca * kRotTW + 4 * k4);
    const float4 mb = *(const float4*)(ms + nb * kRotTW + 4 * k4);
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(xa.x, mb.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(xa.y, mb.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(xa.z, mb.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(xa.w, mb.w, acc, 0, 0, 0);
  }
  rot_tile4_sync();
#pragma unroll
  for (int i = 0; i < 4; ++i) xw[(4 * rg + i) * kRotTW + nb] = acc[i];
  rot_tile4_sync();
  const float4 r = *(const float4*)(xw + row * kRotTW + 4 * q);
  z[0] = r.x;
  z[1] = r.y;
  z[2] = r.z;
  z[3] = r.w;
  rot_tile4_sync();
}

// experiment builds only (tools/variants.sh "p0:-DPGA_RTP_PROBE=0" ...): the
// kernel returns after its prologue (0), after the first round's tournaments
// (1) or skips the epilogue (2), to split the fixed per-generation cost
#ifndef PGA_RTP_PROBE
#define PGA_RTP_PROBE 9
#endif

template <int GS, int OBJ, bool ROT>
__device__ __forceinline__ void real_gen_tp_body(GenArgs a, unsigned long long* best_parts) {
  static_assert(!ROT || GS == 4 || GS == 8, "wave-local rotation: 16 or 32 padded dims");
  resolve_gen(a);
  a.objective = OBJ;  // compile-time objective: the term switches fold away
  const uint32_t NW = blockDim.x >> 6;  // 4 or 16 waves (tp_geometry)
  constexpr uint32_t NG = 64 / GS;      // children per wave per step
  constexpr uint32_t PD = tp_prefetch_depth(GS);  // steps of parent rows in flight (tp.hpp)
  constexpr uint32_t PSEG = ROT ? 6 : 7;  // tp_par_cap segments: the rotation tiles take static LDS
  constexpr bool EVALS = OBJ != OBJ_NONE;
  // JIT (a linked user objective, jitgen_real.hip): the steps also stage
  // their children in the wave's LDS slice; every kJitStageSteps steps one
  // lane per staged child runs the objective on its LDS row (binary_dev.hpp);
  // tournaments read the f32 scores
  // UFN: the reference ABI's `float obj(gene*, unsigned)` device function
  // pointer (pga_set_objective_function, src/pga.cu:206-208, :250-262) on the
  // same LDS staging, as an indirect call: only this instantiation carries the
  // call's scratch stack and conservative register allocation
  constexpr bool UFN = OBJ == kObjUserFn;
  constexpr bool JIT = OBJ == kObjJit || UFN;
  constexpr bool BUILTIN = EVALS && !JIT;
  // dynamic LDS: per wave 2 units x 64 records x 32 B, then the round's parents
  uint4(*lds_rec)[2][64][2] = (uint4(*)[2][64][2])pga_dyn_lds;
  uint2* lds_par = (uint2*)(pga_dyn_lds + NW * 4096u);
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ uint32_t lds_el[kTpMaxElite];  // elite sources
  __shared__ unsigned long long lds_red[kTpMaxWaves];
  __shared__ uint32_t lds_next;   // the round's next unbred unit
  __shared__ uint32_t lds_tnext;  // the round's next tournament segment
  __shared__ uint32_t lds_ready[kTpMaxSegs];  // per segment: its parents are in LDS
  __shared__ __attribute__((aligned(16))) float lds_rot[ROT ? (kTpMaxWaves + 2) * 16 * kRotTW : 1];  // wave tiles + M

  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint32_t q = lane & (GS - 1), gbase = lane & ~(uint32_t)(GS - 1), g = lane / GS;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L, S = (uint32_t)a.S;
  const bool have = q < a.chunks;
  const uint32_t qq = have ? q : 0u;
  const uint32_t clen = have ? (L - 4 * q >= 4 ? 4u : L - 4 * q) : 0u;
  const bool xo_on = a.crossover != XO_NONE;
  const bool uniform_xo = a.crossover == XO_UNIFORM;
  const bool u_word0 = uniform_xo && L <= 32u;  // the record carries every chunk's mask bits
  const bool uwords = uniform_xo && !u_word0 && L <= 128u;  // the record can carry the child's crossover block
  const bool per_gene = real_per_gene_mutation(a);
  const bool dense = per_gene && !a.mut_sparse;
  const bool sparse = per_gene && a.mut_sparse;
  const bool reset_one = a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(OBJ);
  // loop-invariant per-lane problem data
  float sh[4], w0[4], w1[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t d = 4 * q + j;
    sh[j] = (shift && d < L) ? a.obj_data2[d] : 0.f;
    w0[j] = 1.f;
    w1[j] = 0.f;
    if (BUILTIN && d < L) real_obj_data(a, d, w0[j], w1[j]);
  }
  // quantization of the next generation's tournament keys
  float qlo = 0.f, qscale = 0.f;
  if (BUILTIN) qkey_params(a.qk[0], a.qk[1], qlo, qscale);
  // 32-bit offsets (the launcher checks (S + pad) rows < 4 GiB)
  const uint32_t rb = a.row_words * 4u;
#define RROW(base, row, ch) (*(float4*)((char*)(base) + ((uint32_t)(row) * rb + (uint32_t)(ch) * 16u)))
#define RELEM(T, base, i) (*(T*)((char*)(base) + (uint32_t)(i) * (uint32_t)sizeof(T)))

  const uint32_t U = tp_unit(a, NG);  // children per breed unit (tp.hpp)
  uint32_t bbegin, bend;              // this block's children
  tp_block_range(S, U, bbegin, bend, a.tp_skew);
  const uint32_t pcap = tp_par_cap(NW, PSEG);
  // JIT staging after the parents: kJitStageSteps KB per wave (jit.cpp adds it to the launch's LDS)
  float4* lds_stage = (float4*)(pga_dyn_lds + NW * 4096u + pcap * 8u) + wid * (kJitStageSteps * 64u);
  (void)lds_stage;

  float* xw = lds_rot + (ROT ? wid * 16 * kRotTW : 0);          // this wave's X/Z tile
  float* ms = lds_rot + (ROT ? kTpMaxWaves * 16 * kRotTW : 0);  // M[n][k], block-shared
  if (ROT)
    for (uint32_t i = threadIdx.x; i < 32 * kRotTW; i += blockDim.x) {
      const uint32_t n = i / kRotTW, k = i % kRotTW;
      ms[i] = (n < L && k < L) ? a.obj_data[n * L + k] : 0.f;
    }
  // elite sources of children [0, n_elite), for the block that holds any of them
  if (a.n_elite > 0 && bbegin < a.n_elite) {
    if (a.elite_idx) {
      for (uint32_t i = threadIdx.x; i < a.n_elite; i += blockDim.x) lds_el[i] = a.elite_idx[i];
    } else {
      unsigned long long b = block_reduce_parts_n(a.best_cur, a.n_best_cur, lds_red, NW);
      if (threadIdx.x == 0) lds_el[0] = (uint32_t)best_index(b);
    }
  }
  if (per_gene)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += blockDim.x) lds_thr[i] = a.mut_thr[i];
  if (threadIdx.x == 0) lds_next = lds_tnext = 0;
  if (threadIdx.x < kTpMaxSegs) lds_ready[threadIdx.x] = 0;

  unsigned long long my_best = 0;
  ScoreStats st;
  uint4(*rec)[64][2] = lds_rec[wid];
  static_assert(sizeof(lds_rec[0]) >= kSegBatches * 64 * sizeof(uint4), "contestant staging");
  if constexpr (PGA_RTP_PROBE == 0) return;
  for (uint32_t rbeg = bbegin; rbeg < bend; rbeg += pcap) {  // block-uniform rounds
    const uint32_t rend = rbeg + pcap < bend ? rbeg + pcap : bend;
    const uint32_t nb = (rend - rbeg + U - 1) / U;                                  // the round's units
    const uint32_t nseg = (rend - rbeg + kSegBatches * 64 - 1) / (kSegBatches * 64);  // its tournament segments
    __syncthreads();  // tables / elites / M / counter visible; the previous round's records and parents released

    // TOURNAMENTS of the round (contestants wait in the wave's record ring),
    // on the quantized u16 keys when the objective scores the children here
    // pulled from a counter, each segment published by a ready flag; a unit's
    // RESOLVE waits for its segment's flag (no block barrier, binary_dev.hpp)
    for (;;) {
      const uint32_t sg = tp_ticket(&lds_tnext, lane);
      if (sg >= nseg) break;
      const uint32_t begin = rbeg + sg * kSegBatches * 64u;
      const uint32_t end = begin + kSegBatches * 64u < rend ? begin + kSegBatches * 64u : rend;
      tp_select_segment<BUILTIN ? TP_QKEY16 : TP_F32>(a, begin, end, lane, &rec[0][0][0],
                                                    lds_par + sg * kSegBatches * 64u);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the parents before the flag
      tp_flag_set(&lds_ready[sg]);
    }
    // several blocks per CU (the 4-wave grid): a barrier parks the waiting
    // waves (a flag spin would take issue slots from the other blocks' waves:
    // REAL at S = 100K, 36 -> 55 us/gen); one block per CU: the flags alone
    if (NW < kTpMaxWaves) __syncthreads();
    if constexpr (PGA_RTP_PROBE == 1) return;

    // RESOLVE: parents, crossover plan, mutation positions and draws of the
    // round's unit BI -> the records of ring slot SL
#define PGA_RTP_RESOLVE(BI, SL)                                                                              \
  {                                                                                                          \
    {  /* the unit's tournament segment is done (wave-uniform spin, rare) */                                 \
      const uint32_t sg_ = (BI) * U / (kSegBatches * 64u);                                                   \
      while (__hip_atomic_load(&lds_ready[sg_], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)       \
        __builtin_amdgcn_s_sleep(1);                                                                         \
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");                                                 \
    }                                                                                                        \
    const uint32_t bs_ = rbeg + (BI) * U;                                                                    \
    const uint32_t be_ = bs_ + U < rend ? bs_ + U : rend;                                                    \
    const uint32_t tc = bs_ + lane;                                                                          \
    const uint32_t cc = tc < be_ ? tc : be_ - 1;                                                             \
    const uint2 pp = lds_par[cc - rbeg];                                                                     \
    uint32_t pa = pp.x;                                                                                      \
    const u32x4 misc = real_misc<true>(a.key, cc);                                                           \
    const bool elite = tc < a.n_elite;                                                                       \
    const bool xo = !elite && xo_on && do_crossover(a, misc.x);                                              \
    if (elite) pa = lds_el[tc];                                                                              \
    const uint32_t pb = xo ? pp.y : pa;                                                                      \
    uint32_t cut = real_cut_word(a, misc);                                                                   \
    if (u_word0 && xo) cut = real_uniform_word0<true>(a.key, cc);                                            \
    uint32_t K = 0;                                                                                          \
    if (!elite && sparse) K = binom_count(misc.w, lds_thr);                                                  \
    if (!elite && reset_one) K = misc.w < a.mut_ind_thresh ? 1u : 0u;                                        \
    uint32_t posw = 0, jn = 0, d0 = 0, d1 = 0, d2 = 0;                                                       \
    if (K > 0u) {                                                                                            \
      const uint32_t kk = K < 3u ? K : 3u;                                                                   \
      const u32x4 m0 = draw<true>(a.key, ST_BMUT, cc, 0);                                                    \
      const uint32_t c0 = word_to_index(m0.x, L), c1 = word_to_index(m0.y, L), c2 = word_to_index(m0.z, L);  \
      /* common case: the first kk candidates are distinct, hence the positions */                          \
      const bool slow = (kk > 1u && c0 == c1) || (kk > 2u && (c2 == c0 || c2 == c1));                        \
      posw = c0 | (c1 << 8) | (c2 << 16);                                                                    \
      jn = kk;                                                                                               \
      if (slow) {                                                                                            \
        posw = c0;                                                                                           \
        uint32_t n = 1, j = 1;                                                                               \
        u32x4 blk = m0;                                                                                      \
        while (n < kk) {                                                                                     \
          if ((j & 3u) == 0u) blk = draw<true>(a.key, ST_BMUT, cc, j >> 2);                                  \
          const uint32_t p = word_to_index(sel4(blk, j & 3u), L);                                            \
          ++j;                                                                                               \
          if (p == (posw & 0xFFu) || (n > 1u && p == ((posw >> 8) & 0xFFu))) continue;                       \
          posw |= p << (8u * n);                                                                             \
          ++n;                                                                                               \
        }                                                                                                    \
        jn = j;                                                                                              \
      }                                                                                                      \
      d0 = f2u(real_mut_draw<true>(a, cc, 0));                                                               \
      if (kk > 1u) d1 = f2u(real_mut_draw<true>(a, cc, 1));                                                  \
      if (kk > 2u) d2 = f2u(real_mut_draw<true>(a, cc, 2));                                                  \
    }                                                                                                        \
    /* UNIFORM crossover, 33..128 genes, no mutation (the usual child of the                                 \
       reference operators): the child's crossover block rides in the unused                                \
       second record word, one Philox per child here instead of one per lane                                 \
       per step (meta bit 29) */                                                                             \
    const bool xw = uwords && xo && K == 0u;                                                                 \
    if (xw) {                                                                                                \
      const u32x4 xb = draw<true>(a.key, ST_XO, cc, 0);                                                      \
      posw = xb.x;                                                                                           \
      d0 = xb.y;                                                                                             \
      d1 = xb.z;                                                                                             \
      d2 = xb.w;                                                                                             \
    }                                                                                                        \
    const uint32_t meta = (K > 255u ? 255u : K) | ((jn > 0xFFFFu ? 0xFFFFu : jn) << 8) | (xw ? 1u << 29 : 0u) | \
                          (xo ? 1u << 30 : 0u) | (elite ? 1u << 31 : 0u);                                    \
    uint4(*r)[2] = rec[(SL)];                                                                                \
    r[lane][0] = make_uint4(pa, pb, cut, meta);                                                              \
    r[lane][1] = make_uint4(posw, d0, d1, d2);                                                               \
  }

    // BREED: the round's units in ticket order from the block's counter, as
    // two cursors (binary_dev.hpp binary_gen_tp_body): the LOAD cursor
    // issues the parent rows PD steps ahead of the BREED cursor and RESOLVEs
    // a unit into the other ring slot when it enters it; every vector memory
    // operation is unconditional (an exhausted load cursor re-reads the breed
    // cursor's rows; the children past S, at the end only, write the padding)
    const uint32_t b0 = tp_ticket(&lds_next, lane);  // the wave's first unit
    if (b0 < nb) {
      uint32_t bn = tp_ticket(&lds_next, lane);  // the next ticket (>= nb: none)
      PGA_RTP_RESOLVE(b0, 0u)
      uint32_t slot = 0, i = 0, bs = rbeg + b0 * U;  // breed cursor
      uint32_t nst = ((bs + U < rend ? bs + U : rend) - bs + NG - 1) / NG;
      uint32_t lslot = 0, li = 0, lbs = bs, lnst = nst;  // load cursor
      bool lpend = false, lmore = true, done = false;

#define PGA_RTP_LOAD(YA, YB)                                                                                \
  {                                                                                                         \
    if (lpend) { /* entering the next unit */                                                               \
      PGA_RTP_RESOLVE(bn, lslot ^ 1u)                                                                       \
      lslot ^= 1u;                                                                                          \
      li = 0;                                                                                               \
      lbs = rbeg + bn * U;                                                                                  \
      lnst = ((lbs + U < rend ? lbs + U : rend) - lbs + NG - 1) / NG;                                       \
      lpend = false;                                                                                        \
      bn = tp_ticket(&lds_next, lane);                                                                      \
    }                                                                                                       \
    const uint4 r = rec[lmore ? lslot : slot][(lmore ? li : i) * NG + g][0];                                \
    YA = RROW(cur, r.x, qq);                                                                                \
    YB = RROW(cur, r.y, qq);                                                                                \
    if (lmore && ++li == lnst) {                                                                            \
      lpend = bn < nb;                                                                                      \
      lmore = lpend;                                                                                        \
    }                                                                                                       \
  }

#define PGA_RTP_STEP(XA, XB, YA, YB)                                                                        \
  {                                                                                                         \
    PGA_RTP_LOAD(YA, YB)                                                                                    \
    const uint32_t c = bs + i * NG + g;                                                                     \
    const uint4 r0 = rec[slot][i * NG + g][0];                                                              \
    const uint32_t meta = r0.w;                                                                             \
    const uint4 r1 = rec[slot][i * NG + g][1];                                                              \
    const float A_[4] = {XA.x, XA.y, XA.z, XA.w}, B_[4] = {XB.x, XB.y, XB.z, XB.w};                         \
    float v[4];                                                                                             \
    {                                                                                                       \
      uint32_t ub = 0;                                                                                      \
      if (uniform_xo) {                                                                                     \
        if (u_word0) ub = (r0.z >> ((4u * q) & 31u)) & 0xFu;                                                \
        else if ((meta >> 29) & 1u) /* real_uniform_bits from the record's block */                         \
          ub = (sel4(u32x4{r1.x, r1.y, r1.z, r1.w}, (q >> 3) & 3u) >> ((4u * q) & 31u)) & 0xFu;              \
        else ub = real_uniform_bits<true>(a.key, c, q);                                                     \
      }                                                                                                     \
      real_cross_chunk<true>(a, c, q, A_, B_, (meta >> 30) & 1u, r0.z, ub, v);                             \
    }                                                                                                       \
    const uint32_t K = meta & 0xFFu;                                                                        \
    if (K > 0u) { /* group-uniform */                                                                       \
      uint32_t mm = 0;                                                                                      \
      _Pragma("unroll") for (uint32_t k = 0; k < 3; ++k) {                                                  \
        const uint32_t p = (r1.x >> (8u * k)) & 0xFFu;                                                      \
        const uint32_t dk = k == 0 ? r1.y : (k == 1 ? r1.z : r1.w);                                         \
        if (k < K && (p >> 2) == q) {                                                                       \
          set_gene4(v, p & 3u, real_mut_apply(a, u2f(dk), gene4(v, p & 3u)));                               \
          mm |= 1u << (p & 3u);                                                                             \
        }                                                                                                   \
      }                                                                                                     \
      if (K > 3u) real_sparse_group<GS, true>(a, c, K, 3, (meta >> 8) & 0xFFFFu, mm, q, gbase, v);          \
    } else if (dense && !(meta >> 31)) { /* elites are not mutated */                                       \
      real_mutate_chunk(a, c, q, clen, bin_chunk_mut_word<true>(a.key, c, q), lds_thr, v);                  \
    }                                                                                                       \
    _Pragma("unroll") for (uint32_t j = 0; j < 4; ++j) v[j] = j < clen ? v[j] : 0.f;                        \
    if (have) RROW(nxt, c, q) = make_float4(v[0], v[1], v[2], v[3]);                                        \
    if constexpr (JIT) {                                                                                    \
      lds_stage[(i % kJitStageSteps) * 64u + lane] = make_float4(v[0], v[1], v[2], v[3]);                   \
      if (i % kJitStageSteps == kJitStageSteps - 1u || i + 1u == nst) PGA_RTP_JIT_EVAL                      \
    }                                                                                                       \
    if constexpr (BUILTIN) {                                                                                \
      float z[4], zn[4];                                                                                    \
      _Pragma("unroll") for (uint32_t j = 0; j < 4; ++j) z[j] = 4 * q + j < L ? v[j] - sh[j] : 0.f;         \
      if constexpr (ROT) rot_tile4<GS>(xw, ms, z);                                                          \
      zn[0] = z[1];                                                                                         \
      zn[1] = z[2];                                                                                         \
      zn[2] = z[3];                                                                                         \
      zn[3] = OBJ == OBJ_ROSENBROCK ? __shfl(z[0], (int)lane + 1, 64) : 0.f;                                \
      RealAcc acc{0.f, 0.f, 1.f};                                                                           \
      _Pragma("unroll") for (uint32_t j = 0; j < 4; ++j) {                                                  \
        if (j < clen) real_obj_term_w(a, 4 * q + j, z[j], zn[j], v[j], w0[j], w1[j], acc);                  \
      }                                                                                                     \
      acc.s0 = group_sum<GS>(acc.s0);                                                                       \
      acc.s1 = group_sum<GS>(acc.s1);                                                                       \
      acc.s2 = group_prod<GS>(acc.s2);                                                                      \
      const float sc = real_obj_finish(a, acc);                                                             \
      RELEM(float, a.score_next, c) = sc; /* every lane of the group stores the same score */              \
      RELEM(uint16_t, a.key_next, c) = (uint16_t)qkey(sc, qlo, qscale);                                     \
      const unsigned long long pk = c < S ? pack_best(sc, c) : 0ull;                                        \
      my_best = pk > my_best ? pk : my_best;                                                                \
      st.add_if(q == 0u && c < S, sc);                                                                      \
    }                                                                                                       \
    if (++i == nst) {                                                                                       \
      if (lbs == bs) { /* the load cursor never left this unit: it was the wave's last */                   \
        done = true;                                                                                        \
      } else {                                                                                              \
        slot ^= 1u;                                                                                         \
        i = 0;                                                                                              \
        bs = lbs;                                                                                           \
        nst = lnst;                                                                                         \
      }                                                                                                     \
    }                                                                                                       \
  }

      // JIT: the staged steps s0..i of the unit (binary_dev.hpp PGA_TP_JIT_EVAL)
#define PGA_RTP_JIT_EVAL                                                                                    \
  {                                                                                                         \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");                                                  \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");                                                  \
    const uint32_t s0 = i - i % kJitStageSteps, ns = i - s0 + 1u;                                           \
    const uint32_t cj = bs + s0 * NG + lane;                                                                \
    const uint32_t ue = bs + U < rend ? bs + U : rend;                                                      \
    if (lane < ns * NG && cj < ue) {                                                                        \
      const uint32_t js = lane / NG, jg = lane % NG;                                                        \
      float sj;                                                                                             \
      if constexpr (UFN)                                                                                    \
        sj = ((float (*)(float*, unsigned))a.user_fn)((float*)(lds_stage + js * 64u + jg * GS), L);          \
      else                                                                                                  \
        sj = pga_user_objective_f32((pga_lds_floats)(lds_stage + js * 64u + jg * GS), L, a.obj_data);       \
      RELEM(float, a.score_next, cj) = sj;                                                                  \
      my_best = pack_best(sj, cj) > my_best ? pack_best(sj, cj) : my_best;                                  \
      st.add(sj);                                                                                           \
    }                                                                                                       \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");                                                  \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");                                                  \
  }

      float4 A0, B0, A1, B1, A2, B2, A3, B3;  // PD + 1 register sets, rotated statically
      (void)A2; (void)B2; (void)A3; (void)B3;
      if constexpr (PD == 1) {
        PGA_RTP_LOAD(A0, B0)
        for (;;) {
          PGA_RTP_STEP(A0, B0, A1, B1)
          if (done) break;
          PGA_RTP_STEP(A1, B1, A0, B0)
          if (done) break;
        }
      } else if constexpr (PD == 2) {
        PGA_RTP_LOAD(A0, B0)
        PGA_RTP_LOAD(A1, B1)
        for (;;) {
          PGA_RTP_STEP(A0, B0, A2, B2)
          if (done) break;
          PGA_RTP_STEP(A1, B1, A0, B0)
          if (done) break;
          PGA_RTP_STEP(A2, B2, A1, B1)
          if (done) break;
        }
      } else {
        PGA_RTP_LOAD(A0, B0)
        PGA_RTP_LOAD(A1, B1)
        PGA_RTP_LOAD(A2, B2)
        for (;;) {
          PGA_RTP_STEP(A0, B0, A3, B3)
          if (done) break;
          PGA_RTP_STEP(A1, B1, A0, B0)
          if (done) break;
          PGA_RTP_STEP(A2, B2, A1, B1)
          if (done) break;
          PGA_RTP_STEP(A3, B3, A2, B2)
          if (done) break;
        }
      }
#undef PGA_RTP_STEP
#undef PGA_RTP_LOAD
#undef PGA_RTP_JIT_EVAL
    }
#undef PGA_RTP_RESOLVE
    __syncthreads();  // every wave out of the round's counters before they are reset
    if (threadIdx.x == 0) lds_next = lds_tnext = 0;
    if (threadIdx.x < kTpMaxSegs) lds_ready[threadIdx.x] = 0;
  }
#undef RROW
#undef RELEM
  if (EVALS && best_parts && PGA_RTP_PROBE != 2) {  // block-uniform
    unsigned long long bb = block_max_u64_n(my_best, lds_red, NW);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = bb;
    if (a.stats_parts) block_stats_store_n(st, a.stats_parts, NW);
  }
}

template <int GS, int OBJ, bool ROT>
__global__ __launch_bounds__(kTpMaxWaves * 64) void real_gen_tp(GenArgs a, unsigned long long* best_parts) {
  real_gen_tp_body<GS, OBJ, ROT>(a, best_parts);
}

// Batched islands: up to kRealMaxBatch same-shape islands of one device in
// ONE launch, island = blockIdx.y (binary_gen_tp_batch's scheme, real.hip
// real_launch_batch).  The reference's islands are at most MAX_POPULATIONS =
// 10 per solver (include/pga.h:44), run one after another (src/pga.cu:272-276).
constexpr uint32_t kRealMaxBatch = 10;
struct RealBatch {
  GenArgs a[kRealMaxBatch];
  unsigned long long* parts[kRealMaxBatch];
};
template <int GS, int OBJ>
__global__ __launch_bounds__(kTpMaxWaves * 64) void real_gen_tp_batch(RealBatch b) {
  real_gen_tp_body<GS, OBJ, false>(b.a[blockIdx.y], b.parts[blockIdx.y]);
}

}  // namespace (jitgen / anonymous)
}  // namespace pga
