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
#include "pga/real_dev.hpp"

namespace pga {
namespace {

using namespace dev;
typedef float (*obj_fn_t)(float*, unsigned);

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
__device__ __forceinline__ void real_generic_body(GenArgs& a, unsigned long long* best_parts) {
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

template <int GS, int MODE, bool ROT, bool UFN>
__global__ __launch_bounds__(kBlock) void real_kernel(GenArgs a, unsigned long long* best_parts) {
  real_generic_body<GS, MODE, ROT, UFN>(a, best_parts);
}

// ---------------------------------------------------------------------------
// Tiny populations (every child in one block, e.g. the reference's E2 at
// S = 100): n generations in ONE launch with the population resident in LDS.
// As one launch per generation, 100 children cost a chain of dependent global
// round trips (best partial -> scores -> parent rows -> stores drained) plus
// the launch: 7.1 us/gen on hipGraph replay; one launch re-reading global
// memory each generation still 4.6 us.  Here generation 0 reads the global
// population and writes LDS, the middle ones run LDS -> LDS (rows, scores,
// best partial: no global access but the mutation table's first copy), the
// last writes the global buffers of its parity, its best partial and stats.
// Each generation is the generic kernel's generation gen + g, bit for bit.
// Three call sites of the generic body, so each sees its pointers' address
// space (global or LDS) after inlining.
// ---------------------------------------------------------------------------
struct RealMulti {
  void* rows_out;                 // the last generation's children (its parity's buffers)
  float* scores_out;
  uint16_t* keys_out;
  unsigned long long* parts_out;  // its best partial
  float* stats_out;               // its stats partials (or null)
  uint32_t n;                     // generations (>= 2)
  uint32_t lds_off;               // floats: the population region after the body's LDS
};

// LDS floats of the resident population: 2 best partials, 2 x S rows, 2 x S scores
__host__ __device__ inline uint32_t real_multi_floats(uint32_t S, uint32_t row_words) {
  return 4u + 2u * S * row_words + 2u * S;
}

template <int GS, bool UFN>
__global__ __launch_bounds__(kBlock) void real_multi_kernel(GenArgs a, RealMulti m) {
  const uint32_t S = (uint32_t)a.S, rf = a.row_words;
  float* pop = (float*)pga_dyn_lds + m.lds_off;
  unsigned long long* bl = (unsigned long long*)pop;
  float* rows0 = pop + 4;
  float* rows1 = rows0 + S * rf;
  float* sc0 = rows1 + S * rf;
  float* sc1 = sc0 + S;
  const uint32_t* thr = (const uint32_t*)pga_dyn_lds;  // the body's copy of the mutation table
  {  // generation 0: global -> LDS buffer 0
    GenArgs b = a;
    b.next = rows0;
    b.score_next = sc0;
    b.key_next = nullptr;
    b.stats_parts = nullptr;
    real_generic_body<GS, MODE_GEN, false, UFN>(b, &bl[0]);
    __syncthreads();
  }
  for (uint32_t g = 1; g + 1 < m.n; ++g) {  // LDS -> LDS
    GenArgs b = a;
    const bool odd = g & 1u;
    b.cur = odd ? rows0 : rows1;
    b.next = odd ? rows1 : rows0;
    b.score_cur = odd ? sc0 : sc1;
    b.score_next = odd ? sc1 : sc0;
    b.best_cur = odd ? &bl[0] : &bl[1];
    b.n_best_cur = 1;
    b.mut_thr = thr;
    b.key_cur = nullptr;
    b.key_next = nullptr;
    b.stats_parts = nullptr;
    b.key.gen = a.key.gen + g;
    real_generic_body<GS, MODE_GEN, false, UFN>(b, odd ? &bl[1] : &bl[0]);
    __syncthreads();
  }
  {  // the last generation: LDS -> the global buffers of its parity
    const uint32_t g = m.n - 1;
    const bool odd = g & 1u;
    GenArgs b = a;
    b.cur = odd ? rows0 : rows1;
    b.score_cur = odd ? sc0 : sc1;
    b.best_cur = odd ? &bl[0] : &bl[1];
    b.n_best_cur = 1;
    b.mut_thr = thr;
    b.key_cur = nullptr;
    b.next = m.rows_out;
    b.score_next = m.scores_out;
    b.key_next = m.keys_out;
    b.stats_parts = m.stats_out;
    b.key.gen = a.key.gen + g;
    real_generic_body<GS, MODE_GEN, false, UFN>(b, m.parts_out);
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
  (void)configured;
  // only the dynamic-LDS kernels may need more than the default 64 KiB (per device)
  if (lds > 0) (void)allow_dynamic_lds((const void*)k);
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

template <typename K>
uint32_t go_tp(K kernel, const GenArgs& a0, unsigned long long* parts, hipStream_t s, bool rot, bool stage = false) {
  const TpGeom t = tp_geometry(a0.S, 1, (const void*)kernel, 64 / group_size(a0.chunks), rot ? 6 : 7);
  GenArgs a = a0;
  a.tp_unit = t.unit;
  a.tp_skew = tp_skew_units(t, a.S);
  // stage: the children's rows are staged in LDS for an out-of-line objective
  const uint32_t lds = t.lds + (stage ? tp_jit_stage_bytes(t.block / 64) : 0u);
  hipLaunchKernelGGL(kernel, t.grid, t.block, lds, s, a, parts);
  return t.grid;
}

// Below ~64 children per CU the two-phase kernel has too few units to fill
// the device and the generic kernel is as fast (bench/real_size_sweep.py,
// round 4, breed units of U < 64 children: SumGenes-100 at S = 40,000 20.8 vs
// 35.2 us generic, Rastrigin-30 18.8 vs 20.6; at S = 10,000 14.2 vs 15.2 and
// 14.2 vs 13.0).  PGA_TP_MIN_S overrides (the tests pin 0 to cover the
// two-phase kernel at small sizes).
}  // namespace

uint64_t real_tp_min_population() {
  if (const char* e = std::getenv("PGA_TP_MIN_S")) return std::strtoull(e, nullptr, 10);
  return 64ull * (uint64_t)device_cu_count();
}

namespace {

bool real_tp_eligible(const GenArgs& a, uint32_t GS, bool rot) {
  if (force_generic_kernels()) return false;
  if (a.S < real_tp_min_population()) return false;
  if (a.objective == OBJ_TSP_RANDOM_KEY) return false;
  // the user function pointer: a user mutation / crossover callback runs the
  // compat kernels instead; tournaments on the f32 scores (no keys)
  const bool ufn = a.objective == OBJ_USER_FNPTR;
  if (ufn && (rot || a.user_fn == nullptr || a.user_xo_fn || a.user_mut_fn)) return false;
  if (rot && GS != 4 && GS != 8) return false;
  const bool sel_ok = (a.selection == SEL_TOURNAMENT && a.tour_k == 2) || a.selection == SEL_RANDOM ||
                      (a.selection == SEL_RANK && a.rank_order != nullptr) ||
                      (a.selection == SEL_ROULETTE && a.cumfit != nullptr && a.roul_guide != nullptr);
  if (!sel_ok) return false;
  if (a.n_elite > kTpMaxElite || (a.n_elite > 1 && a.elite_idx == nullptr)) return false;
  // evaluating instances tournament on quantized keys (the Island keeps them)
  if (a.objective != OBJ_NONE && !ufn && (!a.key_cur || !a.key_next || !a.qk)) return false;
  // 32-bit offsets: the (S + kRowPad)-row buffers must stay below 4 GiB
  return (a.S + kRowPad) * (uint64_t)a.row_words * 4u <= 0xFFFFFFFFull;
}

}  // namespace

bool real_tp_batchable(const GenArgs& a, uint32_t n) {
  // real_tp_eligible for one of n batched islands: the batch fills the
  // device, so the population threshold applies to all n together; no
  // rotation (rotated objectives run their islands on streams)
  if (a.chunks > 64u || n == 0) return false;
  if ((a.obj_i & 2) && a.obj_data && real_obj_rotatable(a.objective)) return false;
  GenArgs b = a;
  b.S = a.S * n;  // only the threshold reads it below
  if (!real_tp_eligible(b, group_size(a.chunks), false)) return false;
  return (a.S + kRowPad) * (uint64_t)a.row_words * 4u <= 0xFFFFFFFFull;
}

bool real_tp_plan(const GenArgs& a, uint32_t& gs) {
  gs = group_size(a.chunks);
  return a.chunks <= 64u && real_tp_eligible(a, gs, false);
}

namespace {

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
      case OBJ_USER_FNPTR: return go_tp(real_gen_tp<GS, kObjUserFn, false>, a, parts, s, ROT, true);
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

namespace {
template <int GS>
void go_multi(const GenArgs& a, const RealMulti& m, hipStream_t s) {
  const size_t lds = ((size_t)m.lds_off + real_multi_floats((uint32_t)a.S, a.row_words)) * sizeof(float);
  if (a.objective == OBJ_USER_FNPTR) hipLaunchKernelGGL((real_multi_kernel<GS, true>), 1, kBlock, lds, s, a, m);
  else hipLaunchKernelGGL((real_multi_kernel<GS, false>), 1, kBlock, lds, s, a, m);
}
}  // namespace

bool real_launch_multi(const GenArgs& a, unsigned long long* const parts[2], float* const stats[2], uint32_t n,
                       hipStream_t s) {
  static const bool on = [] {
    const char* e = std::getenv("PGA_TINY_MULTI");
    return !(e && e[0] == '0');
  }();
  if (!on || n < 2 || a.chunks == 0 || a.chunks > 64 || force_generic_kernels()) return false;
  const uint32_t gs = group_size(a.chunks);
  if (a.S == 0 || a.S > kBlock / gs) return false;  // one block holds every child
  if (a.objective == OBJ_NONE || ((a.obj_i & 2) && real_obj_rotatable(a.objective))) return false;
  if (a.selection != SEL_TOURNAMENT && a.selection != SEL_RANDOM) return false;
  if (a.n_elite > 1 || a.elite_idx || a.qk || a.gen_dev) return false;
  if (a.user_xo_fn || a.user_mut_fn) return false;  // the compat operators draw a host-filled buffer
  if (!parts[0] || !parts[1]) return false;
  RealMulti m;
  // per-generation parity: generation g writes buffer set (cur + g + 1) & 1,
  // so the last one (n - 1) writes `next` for odd n and `cur` for even n
  const bool odd = n & 1u;
  m.rows_out = odd ? a.next : const_cast<void*>(a.cur);
  m.scores_out = odd ? a.score_next : const_cast<float*>(a.score_cur);
  m.keys_out = odd ? a.key_next : const_cast<uint16_t*>(a.key_cur);
  m.parts_out = parts[odd ? 0 : 1];
  m.stats_out = stats[odd ? 0 : 1];
  m.n = n;
  m.lds_off = (uint32_t)((real_lds_floats(gs, a.chunks, false) + 3) & ~(size_t)3);
  switch (gs) {
    case 1: go_multi<1>(a, m, s); break;
    case 2: go_multi<2>(a, m, s); break;
    case 4: go_multi<4>(a, m, s); break;
    case 8: go_multi<8>(a, m, s); break;
    case 16: go_multi<16>(a, m, s); break;
    case 32: go_multi<32>(a, m, s); break;
    default: go_multi<64>(a, m, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace pga
