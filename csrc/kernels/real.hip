// real.hip — f32 REAL encoding on gfx950, including MFMA-batched rotated
// objectives.
//
// Geometry: one individual = `chunks` 16-byte chunks of 4 genes; a group of
// GS = group_size(chunks) lanes owns one individual (lane q holds genes
// 4q..4q+3), for genomes up to 256 genes (GS <= 64); longer genomes use
// real_long_kernel (a chunk-segment loop, one wave per individual).  The
// randomness layout (real_ops.hpp) is the BINARY one: ST_SEL selection words,
// one misc block per child, sparse mutation positions from ST_BMUT.
//
// Kernels:
//   real_gen_tp<GS,OBJ,ROT>     the hot generation path (transposed tournaments,
//                               per-child records, see below)
//   real_kernel<GS,MODE,ROT,UFN> every mode / selection / objective, one child
//                               per lane group at a time; rotated objectives
//                               on MFMA 16x16x4 f32 tiles staged in LDS
//   real_long_kernel<MODE>      genomes beyond 256 genes
//
// Rotated objectives (CEC-style f(M (x - o)), the "MFMA batched fitness" of
// BASELINE config 3) multiply child tiles by M^T on the matrix cores, exact
// f32 (bit-for-bit a k-ordered fma chain, so the CPU reference reproduces it).
//
// Reference parity: float genes, user objective via device function pointer
// (OBJ_USER_FNPTR, include/pga.h:46 obj_f), E1 sum / E2 knapsack / E3 random-key
// TSP objectives (test*/test.cu) are built in; the reference's evaluate /
// crossover / mutate kernels (src/pga.cu:250-347) become one launch.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/real_ops.hpp"
#include "pga/tp.hpp"

namespace pga {
namespace {

using namespace dev;
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float (*obj_fn_t)(float*, unsigned);

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

struct RealGeom {
  uint32_t tw;   // X/Z tile row stride (floats)
  uint32_t xr;   // tile rows (>= 16 for MFMA)
  uint32_t dp;   // padded dims for MFMA (multiple of 16)
};

__host__ __device__ inline RealGeom real_geom(uint32_t GS, uint32_t chunks) {
  RealGeom g;
  const uint32_t w = 4 * GS > 16 ? 4 * GS : 16;
  g.tw = w + 1;
  const uint32_t gpb = 256 / GS;
  g.xr = gpb > 16 ? gpb : 16;
  g.dp = ((4 * chunks + 15) / 16) * 16;
  return g;
}

// dynamic LDS layout (floats): [hdr 144][X xr*tw][Z xr*tw (rotation)][M dp*(dp+1) (rotation)]
constexpr uint32_t kHdr = 144;  // thr[128] u32 | red[4] u64 (8) | elite u32 | pad  (576 B, 16-aligned)

__host__ __device__ inline size_t real_lds_floats(uint32_t GS, uint32_t chunks, bool rot) {
  RealGeom g = real_geom(GS, chunks);
  size_t n = kHdr + (size_t)g.xr * g.tw;
  if (rot) n += (size_t)g.xr * g.tw + (size_t)g.dp * (g.dp + 1);
  return n;
}

// ---------------------------------------------------------------------------
// Generic kernel: every mode, selection and objective, one child per group.
// UFN: the user-objective instantiation is the only one that contains the
// indirect call (an indirect call forces a scratch stack and a conservative
// register allocation on every instantiation that can reach it).
// ---------------------------------------------------------------------------
template <int GS, int MODE, bool ROT, bool UFN>
__global__ __launch_bounds__(kBlock) void real_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  float* smem = (float*)pga_dyn_lds;
  uint32_t* lds_thr = (uint32_t*)smem;
  unsigned long long* lds_red = (unsigned long long*)(smem + 128);
  uint32_t* lds_elite = (uint32_t*)(smem + 136);
  const RealGeom G = real_geom(GS, a.chunks);
  float* X = smem + kHdr;
  float* Z = X + G.xr * G.tw;
  float* MS = Z + G.xr * G.tw;

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  constexpr uint32_t GPB = kBlock / GS;
  const uint32_t g = threadIdx.x / GS;
  const uint64_t rs = a.row_words >> 2;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L;
  const bool have = q < a.chunks;
  const uint32_t clen = have ? (L - 4 * q >= 4 ? 4u : L - 4 * q) : 0u;
  constexpr bool MUTATES = MODE == MODE_GEN || MODE == MODE_MUTATE;
  constexpr bool CROSSES = MODE == MODE_GEN || MODE == MODE_CROSS;
  constexpr bool EVALS = MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL;
  const bool evals = EVALS && a.objective != OBJ_NONE;
  const bool per_gene = MUTATES && real_per_gene_mutation(a);
  const bool sparse = per_gene && a.mut_sparse;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  const bool tile_needed = ROT || a.objective == OBJ_TSP_RANDOM_KEY || a.objective == OBJ_USER_FNPTR ||
                           a.objective == OBJ_ROSENBROCK;
  float qlo = 0.f, qscale = 0.f;  // quantized tournament keys of the children (GEN, when kept)
  if (MODE == MODE_GEN && a.key_next && a.qk) qkey_params(a.qk[0], a.qk[1], qlo, qscale);

  // ---- per-block setup ----
  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  for (uint32_t i = threadIdx.x; i < G.xr * G.tw; i += kBlock) X[i] = 0.f;
  if (ROT) {
    for (uint32_t i = threadIdx.x; i < G.xr * G.tw; i += kBlock) Z[i] = 0.f;
    for (uint32_t i = threadIdx.x; i < G.dp * (G.dp + 1); i += kBlock) {
      const uint32_t n = i / (G.dp + 1), k = i % (G.dp + 1);
      MS[i] = (n < L && k < L) ? a.obj_data[n * L + k] : 0.f;  // MS[n][k] = M[n][k]
    }
  }
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t base = (uint64_t)blockIdx.x * GPB; base < a.S; base += (uint64_t)gridDim.x * GPB) {  // block-uniform
    const uint64_t child = base + g;
    const bool valid = child < a.S;  // group-uniform
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    float score = 0.f;
    if (valid) {
      // elitism: child = copy of the elite row (no variation), re-evaluated like every child
      const bool elite = MODE == MODE_GEN && child < a.n_elite;
      const u32x4 misc = (CROSSES || MUTATES) ? real_misc(a.key, child) : u32x4{0, 0, 0, 0};
      if (elite) {
        const uint32_t src = a.elite_idx ? a.elite_idx[child] : *lds_elite;
        if (have) {
          const float4 e = cur[(uint64_t)src * rs + q];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        }
      } else if (MODE == MODE_INIT) {
        if (have) real_init_chunk(a, child, q, v);
      } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
        if (have) {
          const float4 e = cur[child * rs + q];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        }
      }
      if (CROSSES && !elite) {
        uint32_t pa, pb;
        st_select_parents(a, child, pa, pb);
        const bool xo = a.crossover != XO_NONE && do_crossover(a, misc.x);
        const uint32_t cut = real_cut_word(a, misc);
        if (have) {
          const float4 A4 = cur[(uint64_t)pa * rs + q], B4 = cur[(uint64_t)pb * rs + q];
          const float A[4] = {A4.x, A4.y, A4.z, A4.w}, B[4] = {B4.x, B4.y, B4.z, B4.w};
          const uint32_t ub = (xo && a.crossover == XO_UNIFORM) ? real_uniform_bits(a.key, child, q) : 0u;
          real_cross_chunk(a, child, q, A, B, xo, cut, ub, v);
        }
      }
      if (MUTATES && !elite) {
        if (sparse || reset_one) {
          const uint32_t K = sparse ? binom_count(misc.w, lds_thr) : (misc.w < a.mut_ind_thresh ? 1u : 0u);
          uint32_t mm = 0;
          real_sparse_group<GS>(a, child, K, 0, 0, mm, q, gbase, v);
        } else if (per_gene && have) {
          real_mutate_chunk(a, child, q, clen, bin_chunk_mut_word(a.key, child, q), lds_thr, v);
        }
      }
      // padding genes of the last chunk stay zero
      for (uint32_t j = 0; j < 4; ++j) v[j] = j < clen ? v[j] : 0.f;  // static indices: no scratch
      if (MODE != MODE_EVAL && have) nxt[child * rs + q] = make_float4(v[0], v[1], v[2], v[3]);
    }

    if (evals) {
      // x (shifted) -> LDS tile row
      float x[4];
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = 4 * q + j;
        x[j] = (shift && d < L) ? v[j] - a.obj_data2[d] : v[j];
        if (d >= L) x[j] = 0.f;
      }
      if (tile_needed) {
        float* row = X + g * G.tw + 4 * q;
        row[0] = x[0]; row[1] = x[1]; row[2] = x[2]; row[3] = x[3];
      }
      float z[4] = {x[0], x[1], x[2], x[3]};
      if (ROT) {
        __syncthreads();
        // Z = X M^T on MFMA: tile (rt, ct) = rows 16rt.., dims 16ct..; B[k][n] = M[n][k]
        const uint32_t w = threadIdx.x >> 6;
        const uint32_t nrt = (GPB + 15) / 16, nct = G.dp / 16;
        for (uint32_t t = w; t < nrt * nct; t += kBlock / 64) {
          const uint32_t rt = t / nct, ct = t % nct;
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* xa = X + (rt * 16 + (lane & 15)) * G.tw + (lane >> 4);
          const float* mb = MS + (ct * 16 + (lane & 15)) * (G.dp + 1) + (lane >> 4);
          for (uint32_t k0 = 0; k0 < G.dp; k0 += 4)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[k0], mb[k0], acc, 0, 0, 0);
          float* zo = Z + (rt * 16 + (lane >> 4) * 4) * G.tw + ct * 16 + (lane & 15);
          zo[0] = acc[0];
          zo[G.tw] = acc[1];
          zo[2 * G.tw] = acc[2];
          zo[3 * G.tw] = acc[3];
        }
        __syncthreads();
        const float* zr = Z + g * G.tw + 4 * q;
        z[0] = zr[0]; z[1] = zr[1]; z[2] = zr[2]; z[3] = zr[3];
      } else if (tile_needed) {
        __syncthreads();
      }
      if (valid) {
        if (UFN) {
          // reference ABI: obj_f(gene*, unsigned) on the child's genome (LDS row)
          float s = 0.f;
          if (q == 0) s = ((obj_fn_t)a.user_fn)(X + g * G.tw, L);
          score = __shfl(s, (int)gbase, 64);
        } else if (a.objective == OBJ_TSP_RANDOM_KEY) {
          // reference E3: path over consecutive decoded cities + 10000 per duplicate pair
          const float* row = X + g * G.tw;
          float len = 0.f;
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t i = 4 * q + j;
            if (i >= L) break;
            const uint32_t ci = random_key_city(row[i], L);
            if (i > 0) len += a.obj_data[random_key_city(row[i - 1], L) * L + ci];
            uint32_t dups = 0;
            for (uint32_t k = 0; k < L; ++k) dups += (k != i && random_key_city(row[k], L) == ci) ? 1u : 0u;
            len += 10000.f * (float)dups;
          }
          score = -group_sum<GS>(len);
        } else {
          RealAcc acc{0.f, 0.f, 1.f};
          const float* zrow = (ROT ? Z : X) + g * G.tw + 4 * q;
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t d = 4 * q + j;
            if (d < L) {
              const float zn = (j < 3) ? z[j + 1] : zrow[4];
              real_obj_term(a, d, z[j], zn, v[j], acc);
            }
          }
          acc.s0 = group_sum<GS>(acc.s0);
          acc.s1 = group_sum<GS>(acc.s1);
          acc.s2 = group_prod<GS>(acc.s2);
          score = real_obj_finish(a, acc);
        }
      }
      if (valid && q == 0) {
        a.score_next[child] = score;
        if (MODE == MODE_GEN && a.key_next) a.key_next[child] = (uint16_t)qkey(score, qlo, qscale);
        const unsigned long long pb = pack_best(score, child);
        my_best = pb > my_best ? pb : my_best;
        st.add(score);
      }
      if (tile_needed) __syncthreads();  // tiles are rewritten next iteration
    }
  }
  if (evals && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}

// ---------------------------------------------------------------------------
// Long genomes (L > 256 genes, more than 64 chunks): one wave per individual,
// lane q owns chunks q, q+64, q+128, ... (a segment loop, the BINARY generic
// kernel's layout), per-lane partial sums in gene order, one 64-lane
// butterfly.  Element-wise objectives and Rosenbrock: the neighbour of a
// segment's last gene is the next segment's first, so lane 63 defers that
// term to the next segment (added before that segment's own terms: the CPU's
// gene-order accumulation per lane).  Sparse mutation positions are listed
// once per child in the wave's LDS (distinct by a wave-wide compare).
// Rotation (M is L x L), the reference-E3 random-key TSP (O(L^2)) and device
// function pointers stay <= 256 genes.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void real_long_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ uint32_t lds_mpos[kBlock / 64][kMutCap];
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  constexpr uint32_t GS = 64, GPB = kBlock / 64;
  const uint32_t q = lane_id(), g = threadIdx.x >> 6;
  const uint64_t rs = a.row_words >> 2;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L, nchunks = a.chunks;
  constexpr bool MUTATES = MODE == MODE_GEN || MODE == MODE_MUTATE;
  constexpr bool CROSSES = MODE == MODE_GEN || MODE == MODE_CROSS;
  constexpr bool EVALS = MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL;
  const bool evals = EVALS && a.objective != OBJ_NONE;
  const bool per_gene = MUTATES && real_per_gene_mutation(a);
  const bool sparse = per_gene && a.mut_sparse;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  const bool rosen = a.objective == OBJ_ROSENBROCK;
  uint32_t* mpos = lds_mpos[g];
  float qlo = 0.f, qscale = 0.f;  // quantized tournament keys of the children (GEN, when kept)
  if (MODE == MODE_GEN && a.key_next && a.qk) qkey_params(a.qk[0], a.qk[1], qlo, qscale);

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t child = (uint64_t)blockIdx.x * GPB + g; child < a.S; child += (uint64_t)gridDim.x * GPB) {
    const bool elite = MODE == MODE_GEN && child < a.n_elite;  // wave-uniform
    const uint32_t src = elite ? (a.elite_idx ? a.elite_idx[child] : lds_elite) : 0u;
    const u32x4 misc = (CROSSES || MUTATES) ? real_misc(a.key, child) : u32x4{0, 0, 0, 0};
    uint32_t pa = 0, pb = 0, cut = 0, nm = 0;
    bool xo = false;
    if (CROSSES && !elite) {
      st_select_parents(a, child, pa, pb);
      xo = a.crossover != XO_NONE && do_crossover(a, misc.x);
      cut = real_cut_word(a, misc);
    }
    if (MUTATES && !elite && (sparse || reset_one)) {
      // the first K distinct positions (sequential definition), listed in LDS
      nm = sparse ? binom_count(misc.w, lds_thr) : (misc.w < a.mut_ind_thresh ? 1u : 0u);
      u32x4 blk{0u, 0u, 0u, 0u};
      for (uint32_t n = 0, j = 0; n < nm;) {  // wave-uniform
        if ((j & 3u) == 0u) blk = draw(a.key, ST_BMUT, child, j >> 2);
        const uint32_t p = word_to_index(sel4(blk, j & 3u), L);
        ++j;
        bool dup = false;
        for (uint32_t i = q; i < n; i += 64) dup |= mpos[i] == p;
        if (__any(dup)) continue;
        if (q == 0) mpos[n] = p;
        wave_lds_sync();
        ++n;
      }
    }
    RealAcc acc{0.f, 0.f, 1.f};
    float dz = 0.f, dx = 0.f;  // lane 63: the deferred Rosenbrock term of its last gene
    uint32_t dd = 0xFFFFFFFFu;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += GS) {  // wave-uniform
      const uint32_t c = c0 + q;
      const bool have = c < nchunks;
      const uint32_t clen = have ? (L - 4 * c >= 4 ? 4u : L - 4 * c) : 0u;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (have) {
        if (elite) {
          const float4 e = cur[(uint64_t)src * rs + c];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        } else if (MODE == MODE_INIT) {
          real_init_chunk(a, child, c, v);
        } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
          const float4 e = cur[child * rs + c];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        }
        if (CROSSES && !elite) {
          const float4 A4 = cur[(uint64_t)pa * rs + c], B4 = cur[(uint64_t)pb * rs + c];
          const float A[4] = {A4.x, A4.y, A4.z, A4.w}, B[4] = {B4.x, B4.y, B4.z, B4.w};
          const uint32_t ub = (xo && a.crossover == XO_UNIFORM) ? real_uniform_bits(a.key, child, c) : 0u;
          real_cross_chunk(a, child, c, A, B, xo, cut, ub, v);
        }
        if (MUTATES && !elite) {
          if (nm > 0) {
            for (uint32_t i = 0; i < nm; ++i) {
              const uint32_t p = mpos[i];
              if ((p >> 2) == c) set_gene4(v, p & 3u, real_mut_apply(a, real_mut_draw(a, child, i), gene4(v, p & 3u)));
            }
          } else if (per_gene && !sparse) {
            real_mutate_chunk(a, child, c, clen, bin_chunk_mut_word(a.key, child, c), lds_thr, v);
          }
        }
        for (uint32_t j = 0; j < 4; ++j) v[j] = j < clen ? v[j] : 0.f;
        if (MODE != MODE_EVAL) nxt[child * rs + c] = make_float4(v[0], v[1], v[2], v[3]);
      }
      if (evals) {
        float x[4];
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t d = 4 * c + j;
          x[j] = (shift && d < L) ? v[j] - a.obj_data2[d] : v[j];
          if (d >= L) x[j] = 0.f;
        }
        const float nx0 = __shfl_down(x[0], 1, 64);  // first gene of chunk c + 1 (lanes < 63)
        if (rosen) {
          const float first = __shfl(x[0], 0, 64);  // this segment's chunk c0 = previous lane 63's c + 1
          if (q == 63 && dd != 0xFFFFFFFFu) real_obj_term(a, dd, dz, first, dx, acc);
          dd = 0xFFFFFFFFu;
        }
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t d = 4 * c + j;
          if (d >= L) continue;
          if (rosen && j == 3 && q == 63) {  // neighbour in the next segment
            dd = d;
            dz = x[3];
            dx = v[3];
            continue;
          }
          const float zn = j < 3 ? x[j + 1] : nx0;
          real_obj_term(a, d, x[j], zn, v[j], acc);
        }
      }
    }
    if (MUTATES && nm > 0) wave_lds_sync();  // the list is rewritten for the next child
    float score = 0.f;
    if (evals) {
      acc.s0 = group_sum<GS>(acc.s0);
      acc.s1 = group_sum<GS>(acc.s1);
      acc.s2 = group_prod<GS>(acc.s2);
      score = real_obj_finish(a, acc);
    }
    if (evals && q == 0) {
      a.score_next[child] = score;
      if (MODE == MODE_GEN && a.key_next) a.key_next[child] = (uint16_t)qkey(score, qlo, qscale);
      const unsigned long long pk = pack_best(score, child);
      my_best = pk > my_best ? pk : my_best;
      st.add(score);
    }
  }
  if (evals && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}

template <typename K>
uint32_t launch_occ(K k, uint32_t children_per_block, size_t lds, const GenArgs& a, unsigned long long* parts,
                    hipStream_t s, bool& configured) {
  if (!configured) {
    // only the dynamic-LDS kernels may need more than the default 64 KiB
    if (lds > 0) allow_dynamic_lds((const void*)k);
    configured = true;
  }
  uint64_t need = (a.S + children_per_block - 1) / children_per_block;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, kBlock, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  uint64_t cap = (uint64_t)device_cu_count() * per_cu;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t grid = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL(k, grid, kBlock, lds, s, a, parts);
  return grid;
}

template <int GS, int MODE, bool ROT>
uint32_t go(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  const size_t lds = real_lds_floats(GS, a.chunks, ROT) * sizeof(float);
  if (a.objective == OBJ_USER_FNPTR) {
    static bool c1 = false;
    return launch_occ(real_kernel<GS, MODE, false, true>, kBlock / GS, lds, a, parts, s, c1);
  }
  static bool c0 = false;  // one per instantiation
  return launch_occ(real_kernel<GS, MODE, ROT, false>, kBlock / GS, lds, a, parts, s, c0);
}

// ---------------------------------------------------------------------------
// The hot generation kernel: transposed tournaments (the binary_gen_tp design,
// binary_dev.hpp).  A wave breeds NG = 64/GS children per STEP; a block owns
// a contiguous share of the population, in rounds (tp.hpp tp_block_range):
//   TOURNAMENTS  tp_select_segment (tp.hpp): one lane per child, every f32
//                score load of a 256-child segment in flight together
//   BREED        after one block barrier, UNITS of U <= 64 children pulled
//                from the block's LDS counter; per unit, RESOLVE (one lane
//                per child): the misc block
//                (crossover test, cut points / arithmetic u, mutation count
//                K), the first min(K, 3) distinct mutation positions and
//                their values (gaussian z by gauss_z) -> a 32-byte child
//                RECORD in the wave's LDS ring (2 units); per step: parent
//                rows loaded one step ahead, crossover (BLX: one Philox block
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

template <int GS, int OBJ, bool ROT>
__global__ __launch_bounds__(kTpMaxWaves * 64) void real_gen_tp(GenArgs a, unsigned long long* best_parts) {
  static_assert(!ROT || GS == 4 || GS == 8, "wave-local rotation: 16 or 32 padded dims");
  resolve_gen(a);
  a.objective = OBJ;  // compile-time objective: the term switches fold away
  const uint32_t NW = blockDim.x >> 6;  // 4 or 16 waves (tp_geometry)
  constexpr uint32_t NG = 64 / GS;      // children per wave per step
  constexpr uint32_t PD = tp_prefetch_depth(GS);  // steps of parent rows in flight (tp.hpp)
  constexpr uint32_t PSEG = ROT ? 6 : 7;  // tp_par_cap segments: the rotation tiles take static LDS
  constexpr bool EVALS = OBJ != OBJ_NONE;
  // dynamic LDS: per wave 2 units x 64 records x 32 B, then the round's parents
  uint4(*lds_rec)[2][64][2] = (uint4(*)[2][64][2])pga_dyn_lds;
  uint2* lds_par = (uint2*)(pga_dyn_lds + NW * 4096u);
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ uint32_t lds_el[kTpMaxElite];  // elite sources
  __shared__ unsigned long long lds_red[kTpMaxWaves];
  __shared__ uint32_t lds_next;  // the round's next unbred unit
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
    if (EVALS && d < L) real_obj_data(a, d, w0[j], w1[j]);
  }
  // quantization of the next generation's tournament keys
  float qlo = 0.f, qscale = 0.f;
  if (EVALS) qkey_params(a.qk[0], a.qk[1], qlo, qscale);
  // 32-bit offsets (the launcher checks (S + pad) rows < 4 GiB)
  const uint32_t rb = a.row_words * 4u;
#define RROW(base, row, ch) (*(float4*)((char*)(base) + ((uint32_t)(row) * rb + (uint32_t)(ch) * 16u)))
#define RELEM(T, base, i) (*(T*)((char*)(base) + (uint32_t)(i) * (uint32_t)sizeof(T)))

  const uint32_t U = tp_unit(a, NG);  // children per breed unit (tp.hpp)
  uint32_t bbegin, bend;              // this block's children
  tp_block_range(S, U, bbegin, bend);
  const uint32_t pcap = tp_par_cap(NW, PSEG);

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
  if (threadIdx.x == 0) lds_next = 0;

  unsigned long long my_best = 0;
  ScoreStats st;
  uint4(*rec)[64][2] = lds_rec[wid];
  static_assert(sizeof(lds_rec[0]) >= kSegBatches * 64 * sizeof(uint4), "contestant staging");
  for (uint32_t rbeg = bbegin; rbeg < bend; rbeg += pcap) {  // block-uniform rounds
    const uint32_t rend = rbeg + pcap < bend ? rbeg + pcap : bend;
    const uint32_t nb = (rend - rbeg + U - 1) / U;                                  // the round's units
    const uint32_t nseg = (rend - rbeg + kSegBatches * 64 - 1) / (kSegBatches * 64);  // its tournament segments
    __syncthreads();  // tables / elites / M / counter visible; the previous round's records and parents released

    // TOURNAMENTS of the round (contestants wait in the wave's record ring),
    // on the quantized u16 keys when the objective scores the children here
    for (uint32_t sg = wid; sg < nseg; sg += NW) {
      const uint32_t begin = rbeg + sg * kSegBatches * 64u;
      const uint32_t end = begin + kSegBatches * 64u < rend ? begin + kSegBatches * 64u : rend;
      tp_select_segment<EVALS ? TP_QKEY16 : TP_F32>(a, begin, end, lane, &rec[0][0][0],
                                                    lds_par + sg * kSegBatches * 64u);
    }
    __syncthreads();  // every parent of the round in LDS

    // RESOLVE: parents, crossover plan, mutation positions and draws of the
    // round's unit BI -> the records of ring slot SL
#define PGA_RTP_RESOLVE(BI, SL)                                                                              \
  {                                                                                                          \
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
    const uint32_t meta =                                                                                    \
        (K > 255u ? 255u : K) | ((jn > 0xFFFFu ? 0xFFFFu : jn) << 8) | (xo ? 1u << 30 : 0u) | (elite ? 1u << 31 : 0u); \
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
    uint32_t tk = 0;
    if (lane == 0) tk = __hip_atomic_fetch_add(&lds_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(tk);  // the wave's first unit
    if (b0 < nb) {
      if (lane == 0) tk = __hip_atomic_fetch_add(&lds_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint32_t bn = __builtin_amdgcn_readfirstlane(tk);  // the next ticket (>= nb: none)
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
      if (lane == 0)                                                                                        \
        tk = __hip_atomic_fetch_add(&lds_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);         \
      bn = __builtin_amdgcn_readfirstlane(tk);                                                              \
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
    const float A_[4] = {XA.x, XA.y, XA.z, XA.w}, B_[4] = {XB.x, XB.y, XB.z, XB.w};                         \
    float v[4];                                                                                             \
    {                                                                                                       \
      uint32_t ub = 0;                                                                                      \
      if (uniform_xo) ub = u_word0 ? (r0.z >> ((4u * q) & 31u)) & 0xFu : real_uniform_bits<true>(a.key, c, q); \
      real_cross_chunk<true>(a, c, q, A_, B_, (meta >> 30) & 1u, r0.z, ub, v);                             \
    }                                                                                                       \
    const uint32_t K = meta & 0xFFu;                                                                        \
    if (K > 0u) { /* group-uniform */                                                                       \
      const uint4 r1 = rec[slot][i * NG + g][1];                                                            \
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
    if constexpr (EVALS) {                                                                                  \
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
    }
#undef PGA_RTP_RESOLVE
    __syncthreads();  // every wave out of the round's counter before it is reset
    if (threadIdx.x == 0) lds_next = 0;
  }
#undef RROW
#undef RELEM
  if (EVALS && best_parts) {  // block-uniform
    unsigned long long bb = block_max_u64_n(my_best, lds_red, NW);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = bb;
    if (a.stats_parts) block_stats_store_n(st, a.stats_parts, NW);
  }
}

template <typename K>
uint32_t go_tp(K kernel, const GenArgs& a0, unsigned long long* parts, hipStream_t s, bool rot) {
  const TpGeom t = tp_geometry(a0.S, 1, (const void*)kernel, 64 / group_size(a0.chunks), rot ? 6 : 7);
  GenArgs a = a0;
  a.tp_unit = t.unit;
  hipLaunchKernelGGL(kernel, t.grid, t.block, t.lds, s, a, parts);
  return t.grid;
}

// Below ~64 children per CU the two-phase kernel has too few units to fill
// the device and the generic kernel is as fast (bench/real_size_sweep.py,
// round 4, breed units of U < 64 children: SumGenes-100 at S = 40,000 20.8 vs
// 35.2 us generic, Rastrigin-30 18.8 vs 20.6; at S = 10,000 14.2 vs 15.2 and
// 14.2 vs 13.0).  PGA_TP_MIN_S overrides (the tests pin 0 to cover the
// two-phase kernel at small sizes).
uint64_t real_tp_min_population() {
  if (const char* e = std::getenv("PGA_TP_MIN_S")) return std::strtoull(e, nullptr, 10);
  return 64ull * (uint64_t)device_cu_count();
}

bool real_tp_eligible(const GenArgs& a, uint32_t GS, bool rot) {
  if (force_generic_kernels()) return false;
  if (a.S < real_tp_min_population()) return false;
  if (a.objective == OBJ_USER_FNPTR || a.objective == OBJ_TSP_RANDOM_KEY) return false;
  if (rot && GS != 4 && GS != 8) return false;
  const bool sel_ok = (a.selection == SEL_TOURNAMENT && a.tour_k == 2) || a.selection == SEL_RANDOM ||
                      (a.selection == SEL_RANK && a.rank_order != nullptr) ||
                      (a.selection == SEL_ROULETTE && a.cumfit != nullptr && a.roul_guide != nullptr);
  if (!sel_ok) return false;
  if (a.n_elite > kTpMaxElite || (a.n_elite > 1 && a.elite_idx == nullptr)) return false;
  // evaluating instances tournament on quantized keys (the Island keeps them)
  if (a.objective != OBJ_NONE && (!a.key_cur || !a.key_next || !a.qk)) return false;
  // 32-bit offsets: the (S + kRowPad)-row buffers must stay below 4 GiB
  return (a.S + kRowPad) * (uint64_t)a.row_words * 4u <= 0xFFFFFFFFull;
}

template <int GS, bool ROT>
uint32_t launch_tp(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  if constexpr (ROT) {
    if constexpr (GS == 4 || GS == 8) {
      switch (a.objective) {
        case OBJ_SPHERE: return go_tp(real_gen_tp<GS, OBJ_SPHERE, true>, a, parts, s, ROT);
        case OBJ_RASTRIGIN: return go_tp(real_gen_tp<GS, OBJ_RASTRIGIN, true>, a, parts, s, ROT);
        case OBJ_ROSENBROCK: return go_tp(real_gen_tp<GS, OBJ_ROSENBROCK, true>, a, parts, s, ROT);
        case OBJ_ACKLEY: return go_tp(real_gen_tp<GS, OBJ_ACKLEY, true>, a, parts, s, ROT);
        case OBJ_GRIEWANK: return go_tp(real_gen_tp<GS, OBJ_GRIEWANK, true>, a, parts, s, ROT);
        default: return go_tp(real_gen_tp<GS, OBJ_SCHWEFEL, true>, a, parts, s, ROT);
      }
    }
    return 0;
  } else {
    switch (a.objective) {
      case OBJ_SPHERE: return go_tp(real_gen_tp<GS, OBJ_SPHERE, false>, a, parts, s, ROT);
      case OBJ_RASTRIGIN: return go_tp(real_gen_tp<GS, OBJ_RASTRIGIN, false>, a, parts, s, ROT);
      case OBJ_ROSENBROCK: return go_tp(real_gen_tp<GS, OBJ_ROSENBROCK, false>, a, parts, s, ROT);
      case OBJ_ACKLEY: return go_tp(real_gen_tp<GS, OBJ_ACKLEY, false>, a, parts, s, ROT);
      case OBJ_GRIEWANK: return go_tp(real_gen_tp<GS, OBJ_GRIEWANK, false>, a, parts, s, ROT);
      case OBJ_SCHWEFEL: return go_tp(real_gen_tp<GS, OBJ_SCHWEFEL, false>, a, parts, s, ROT);
      case OBJ_LINEAR: return go_tp(real_gen_tp<GS, OBJ_LINEAR, false>, a, parts, s, ROT);
      case OBJ_KNAPSACK_REAL: return go_tp(real_gen_tp<GS, OBJ_KNAPSACK_REAL, false>, a, parts, s, ROT);
      default: return go_tp(real_gen_tp<GS, OBJ_NONE, false>, a, parts, s, ROT);
    }
  }
}

template <int GS, bool ROT>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (mode) {
    case MODE_GEN:
      if (real_tp_eligible(a, GS, ROT)) return launch_tp<GS, ROT>(a, parts, s);
      return go<GS, MODE_GEN, ROT>(a, parts, s);
    case MODE_INIT: return go<GS, MODE_INIT, ROT>(a, parts, s);
    case MODE_EVAL: return go<GS, MODE_EVAL, ROT>(a, parts, s);
    case MODE_CROSS: return go<GS, MODE_CROSS, false>(a, parts, s);
    default: return go<GS, MODE_MUTATE, false>(a, parts, s);
  }
}

template <int GS>
uint32_t launch_rot(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  const bool rot = (a.obj_i & 2) && a.obj_data && real_obj_rotatable(a.objective);
  return rot ? launch_mode<GS, true>(mode, a, parts, s) : launch_mode<GS, false>(mode, a, parts, s);
}

}  // namespace

uint32_t real_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  const bool rot = (a.obj_i & 2) && real_obj_rotatable(a.objective);
  if (rot && a.L > 128) throw std::invalid_argument("rotated objectives support at most 128 dimensions");
  if (a.chunks > 64) {
    if (a.objective == OBJ_TSP_RANDOM_KEY || a.objective == OBJ_USER_FNPTR)
      throw std::invalid_argument("the random-key TSP and function-pointer objectives support at most 256 genes");
    static bool c[5] = {false, false, false, false, false};
    constexpr uint32_t per_block = kBlock / 64;
    uint32_t grid = 0;
    switch (mode) {
      case MODE_GEN: grid = launch_occ(real_long_kernel<MODE_GEN>, per_block, 0, a, best_parts, s, c[0]); break;
      case MODE_INIT: grid = launch_occ(real_long_kernel<MODE_INIT>, per_block, 0, a, best_parts, s, c[1]); break;
      case MODE_EVAL: grid = launch_occ(real_long_kernel<MODE_EVAL>, per_block, 0, a, best_parts, s, c[2]); break;
      case MODE_CROSS: grid = launch_occ(real_long_kernel<MODE_CROSS>, per_block, 0, a, best_parts, s, c[3]); break;
      default: grid = launch_occ(real_long_kernel<MODE_MUTATE>, per_block, 0, a, best_parts, s, c[4]); break;
    }
    PGA_HIP_CHECK(hipGetLastError());
    return grid;
  }
  uint32_t grid = 0;
  switch (group_size(a.chunks)) {
    case 1: grid = launch_rot<1>(mode, a, best_parts, s); break;
    case 2: grid = launch_rot<2>(mode, a, best_parts, s); break;
    case 4: grid = launch_rot<4>(mode, a, best_parts, s); break;
    case 8: grid = launch_rot<8>(mode, a, best_parts, s); break;
    case 16: grid = launch_rot<16>(mode, a, best_parts, s); break;
    case 32: grid = launch_rot<32>(mode, a, best_parts, s); break;
    default: grid = launch_rot<64>(mode, a, best_parts, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace pga
