// real.hip — f32 REAL encoding on gfx950, including MFMA-batched rotated
// objectives.
//
// Geometry: one individual = `chunks` 16-byte chunks of 4 genes; a group of
// GS = group_size(chunks) lanes owns one individual (lane q holds genes
// 4q..4q+3), GPB = 256/GS individuals per block iteration, for genomes up to
// 256 genes (GS <= 64); longer genomes use real_long_kernel (a chunk-segment
// loop, one wave per individual).  Per iteration every child's genes are also staged in an
// LDS tile X[GPB][TW] (TW = max(4 GS, 16) + 1: the +1 breaks the 16-way bank
// conflict of the MFMA A-operand column reads).
//
// Rotated objectives (CEC-style f(M (x - o)), the "MFMA batched fitness" of
// BASELINE config 3) multiply the whole child tile by M^T with
// v_mfma_f32_16x16x4_f32: 16 children x 16 dims per wave tile, K = 4 per
// instruction, exact f32 (bit-for-bit a k-ordered fma chain, so the CPU
// reference reproduces it), M staged once per block in LDS (real_gen_fast,
// L <= 128).  For L <= 32 (the 30-D Rastrigin config) the software-pipelined
// kernel does the rotation wave-locally instead, with v_mfma_f32_4x4x1_16b_f32
// (64/GS children x 4 GS dims = 16 blocks of 4x4 per wave, no empty rows),
// the same exact fma chain, and no block barrier (real_gen_pipe, ROT).
//
// Reference parity: float genes, user objective via device function pointer
// (OBJ_USER_FNPTR, include/pga.h:46 obj_f), E1 sum / E2 knapsack / E3 random-key
// TSP objectives (test*/test.cu) are built in.
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/real_ops.hpp"

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

// UFN: the user-objective instantiation is the only one that contains the
// indirect call (an indirect call forces a scratch stack and a conservative
// register allocation on every instantiation that can reach it)
template <int GS, int MODE, bool ROT, bool UFN>
__global__ __launch_bounds__(kBlock) void real_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  extern __shared__ __attribute__((aligned(16))) float smem[];
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
  constexpr bool EVALS = MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL;
  const bool evals = EVALS && a.objective != OBJ_NONE;
  const bool per_gene_mut = MUTATES && (a.mutation == MUT_GAUSSIAN || a.mutation == MUT_UNIFORM) && a.mut_rate > 0.f;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  const bool tile_needed = ROT || a.objective == OBJ_TSP_RANDOM_KEY || a.objective == OBJ_USER_FNPTR ||
                           a.objective == OBJ_ROSENBROCK;

  // ---- per-block setup ----
  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene_mut)
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
    bool elite = false;
    float score = 0.f;
    if (valid) {
      if (MODE == MODE_GEN && child < a.n_elite) {
        elite = true;
        const uint32_t src = a.elite_idx ? a.elite_idx[child] : *lds_elite;
        if (have) {
          const float4 e = cur[(uint64_t)src * rs + q];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        }
        score = a.score_cur[src];
      } else if (MODE == MODE_INIT) {
        if (have) real_init_chunk(a, child, q, v);
      } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
        if (have) {
          const float4 e = cur[child * rs + q];
          v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
        }
      }
      if (!elite && (MODE == MODE_GEN || MODE == MODE_CROSS || MODE == MODE_MUTATE)) {
        Pool<GS> pool{draw(a.key, ST_CHILD, child, q), gbase};
        if (MODE == MODE_GEN || MODE == MODE_CROSS) {
          uint32_t pa, pb;
          select_parents<GS>(a, pool, child, pa, pb);
          const bool xo = a.crossover != XO_NONE && do_crossover(a, pool.get(W_XOPROB, a.key, child));
          uint32_t blo = 0, bhi = 0;
          float ua = 0.f;
          if (a.crossover == XO_ONE_POINT) {
            blo = word_to_index(pool.get(W_CUT1, a.key, child), L);
            bhi = L;
          } else if (a.crossover == XO_TWO_POINT) {
            const uint32_t c1 = word_to_index(pool.get(W_CUT1, a.key, child), L);
            const uint32_t c2 = word_to_index(pool.get(W_CUT2, a.key, child), L);
            blo = c1 < c2 ? c1 : c2;
            bhi = c1 < c2 ? c2 : c1;
          } else if (a.crossover == XO_ARITHMETIC) {
            ua = word_to_unit(pool.get(W_CUT1, a.key, child));
          }
          if (have) {
            const float4 A4 = cur[(uint64_t)pa * rs + q], B4 = cur[(uint64_t)pb * rs + q];
            const float A[4] = {A4.x, A4.y, A4.z, A4.w}, B[4] = {B4.x, B4.y, B4.z, B4.w};
            real_cross_chunk(a, child, q, A, B, xo, blo, bhi, ua, v);
          }
        }
        if (per_gene_mut && have) {
          real_mutate_chunk(a, child, q, clen, pool.w.w, lds_thr, v);
        } else if (reset_one && pool.get(W_MUTIND, a.key, child) < a.mut_ind_thresh) {
          const uint32_t pos = word_to_index(pool.get(W_MUTPOS, a.key, child), L);
          const float x = real_reset_value(a, pool.get(W_SEL + sel_words(a), a.key, child));
          if ((pos >> 2) == q) {
            const uint32_t j = pos & 3u;
            v[0] = j == 0 ? x : v[0];
            v[1] = j == 1 ? x : v[1];
            v[2] = j == 2 ? x : v[2];
            v[3] = j == 3 ? x : v[3];
          }
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
      if (valid && !elite) {
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
// gene-order accumulation per lane).  Rotation (M is L x L), the reference-E3
// random-key TSP (O(L^2)) and device function pointers stay <= 256 genes.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void real_long_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  constexpr uint32_t GS = 64, GPB = kBlock / 64;
  const uint32_t q = lane_id(), g = threadIdx.x >> 6;
  const uint64_t rs = a.row_words >> 2;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L, nchunks = a.chunks;
  constexpr bool MUTATES = MODE == MODE_GEN || MODE == MODE_MUTATE;
  constexpr bool EVALS = MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL;
  const bool evals = EVALS && a.objective != OBJ_NONE;
  const bool per_gene_mut = MUTATES && (a.mutation == MUT_GAUSSIAN || a.mutation == MUT_UNIFORM) && a.mut_rate > 0.f;
  const bool reset_one = MUTATES && a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  const bool rosen = a.objective == OBJ_ROSENBROCK;

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene_mut)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t child = (uint64_t)blockIdx.x * GPB + g; child < a.S; child += (uint64_t)gridDim.x * GPB) {
    const bool elite = MODE == MODE_GEN && child < a.n_elite;  // wave-uniform
    const uint32_t src = elite ? (a.elite_idx ? a.elite_idx[child] : lds_elite) : 0u;
    const bool breeds = !elite && (MODE == MODE_GEN || MODE == MODE_CROSS || MODE == MODE_MUTATE);
    Pool<GS> pool{u32x4{0, 0, 0, 0}, 0u};
    uint32_t pa = 0, pb = 0, blo = 0, bhi = 0, rpos = 0xFFFFFFFFu;
    bool xo = false;
    float ua = 0.f, rval = 0.f;
    if (breeds) {
      pool.w = draw(a.key, ST_CHILD, child, q);
      if (MODE == MODE_GEN || MODE == MODE_CROSS) {
        select_parents<GS>(a, pool, child, pa, pb);
        xo = a.crossover != XO_NONE && do_crossover(a, pool.get(W_XOPROB, a.key, child));
        if (a.crossover == XO_ONE_POINT) {
          blo = word_to_index(pool.get(W_CUT1, a.key, child), L);
          bhi = L;
        } else if (a.crossover == XO_TWO_POINT) {
          const uint32_t c1 = word_to_index(pool.get(W_CUT1, a.key, child), L);
          const uint32_t c2 = word_to_index(pool.get(W_CUT2, a.key, child), L);
          blo = c1 < c2 ? c1 : c2;
          bhi = c1 < c2 ? c2 : c1;
        } else if (a.crossover == XO_ARITHMETIC) {
          ua = word_to_unit(pool.get(W_CUT1, a.key, child));
        }
      }
      if (reset_one && pool.get(W_MUTIND, a.key, child) < a.mut_ind_thresh) {
        rpos = word_to_index(pool.get(W_MUTPOS, a.key, child), L);
        rval = real_reset_value(a, pool.get(W_SEL + sel_words(a), a.key, child));
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
        if (breeds && (MODE == MODE_GEN || MODE == MODE_CROSS)) {
          const float4 A4 = cur[(uint64_t)pa * rs + c], B4 = cur[(uint64_t)pb * rs + c];
          const float A[4] = {A4.x, A4.y, A4.z, A4.w}, B[4] = {B4.x, B4.y, B4.z, B4.w};
          real_cross_chunk(a, child, c, A, B, xo, blo, bhi, ua, v);
        }
        if (breeds && per_gene_mut) {
          real_mutate_chunk(a, child, c, clen, c == q ? pool.w.w : chunk_mut_word(a.key, child, c), lds_thr, v);
        } else if (breeds && (rpos >> 2) == c) {
          const uint32_t j = rpos & 3u;
          v[0] = j == 0 ? rval : v[0];
          v[1] = j == 1 ? rval : v[1];
          v[2] = j == 2 ? rval : v[2];
          v[3] = j == 3 ? rval : v[3];
        }
        for (uint32_t j = 0; j < 4; ++j) v[j] = j < clen ? v[j] : 0.f;
        if (MODE != MODE_EVAL) nxt[child * rs + c] = make_float4(v[0], v[1], v[2], v[3]);
      }
      if (evals && !elite) {
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
    float score = 0.f;
    if (evals) {
      acc.s0 = group_sum<GS>(acc.s0);
      acc.s1 = group_sum<GS>(acc.s1);
      acc.s2 = group_prod<GS>(acc.s2);
      score = elite ? a.score_cur[src] : real_obj_finish(a, acc);
    }
    if (evals && q == 0) {
      a.score_next[child] = score;
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
// Fast GEN path.  The generic kernel above walks one child per group per block
// iteration through a strictly serial chain (pool draw -> 4 score loads ->
// 2 parent-row loads -> crossover/mutation -> store -> objective), so with a
// few waves per SIMD it is latency bound (rocprof: ~5.7 us per iteration,
// 1.1 TB/s effective on Rastrigin-30D @ 1M).  Here every group carries U
// children through each phase together: U x 4 tournament loads are in flight
// at once, then U x 2 parent rows, then the U children are finished back to
// back — U-fold memory-level parallelism per wave with no extra waves.
// Semantics (RNG words, operators, elitism, MFMA order) are exactly the
// generic kernel's, so rows stay bit-identical to the CPU reference.
// Eligible: MODE_GEN, tournament-2 or random selection, built-in objectives
// that need no neighbour dimension (not Rosenbrock without rotation, not
// random-key TSP, not user fn-ptrs).
template <int GS, int U, bool ROT>
__global__ __launch_bounds__(kBlock) void real_gen_fast(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint32_t* lds_thr = (uint32_t*)smem;
  unsigned long long* lds_red = (unsigned long long*)(smem + 128);
  uint32_t* lds_elite = (uint32_t*)(smem + 136);
  constexpr uint32_t GPB = kBlock / GS;
  constexpr uint32_t ROWS = GPB * U;
  constexpr uint32_t XR = ROWS > 16 ? ROWS : 16;
  constexpr uint32_t TW = (4 * GS > 16 ? 4 * GS : 16) + 1;
  const uint32_t dp = ((4 * a.chunks + 15) / 16) * 16;
  float* X = smem + kHdr;  // [XR][TW] shifted x (ROT)
  float* Z = X + XR * TW;  // [XR][TW] rotated z (ROT)
  float* MS = Z + XR * TW; // [dp][dp+1]

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  const uint32_t g = threadIdx.x / GS;
  const uint64_t rs = a.row_words >> 2;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L;
  const uint32_t S32 = (uint32_t)a.S;
  const bool have = q < a.chunks;
  const uint32_t qc = have ? q : a.chunks - 1;  // unconditional loads, clamped chunk
  const uint32_t clen = have ? (L - 4 * q >= 4 ? 4u : L - 4 * q) : 0u;
  const bool evals = a.objective != OBJ_NONE;
  const bool tour2 = a.selection == SEL_TOURNAMENT;
  const bool per_gene_mut = (a.mutation == MUT_GAUSSIAN || a.mutation == MUT_UNIFORM) && a.mut_rate > 0.f;
  const bool reset_one = a.mutation == MUT_RESET_ONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);

  if (a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene_mut)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  if (ROT) {
    for (uint32_t i = threadIdx.x; i < 2 * XR * TW; i += kBlock) X[i] = 0.f;
    for (uint32_t i = threadIdx.x; i < dp * (dp + 1); i += kBlock) {
      const uint32_t n = i / (dp + 1), k = i % (dp + 1);
      MS[i] = (n < L && k < L) ? a.obj_data[n * L + k] : 0.f;
    }
  }
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t base = (uint64_t)blockIdx.x * ROWS; base < a.S; base += (uint64_t)gridDim.x * ROWS) {
    uint64_t ch[U];
    u32x4 pw[U];
    uint32_t pa[U], pb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ch[u] = base + u * GPB + g;
      pw[u] = draw(a.key, ST_CHILD, ch[u], q);
    }
    // ---- phase 1: selection (all U x 4 score loads in flight together) ----
    if (tour2) {
      uint32_t i0[U], i1[U], i2[U], i3[U];
      float s0[U], s1[U], s2[U], s3[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const Pool<GS> pool{pw[u], gbase};
        i0[u] = word_to_index(pool.get(W_SEL + 0, a.key, ch[u]), S32);
        i1[u] = word_to_index(pool.get(W_SEL + 1, a.key, ch[u]), S32);
        i2[u] = word_to_index(pool.get(W_SEL + 2, a.key, ch[u]), S32);
        i3[u] = word_to_index(pool.get(W_SEL + 3, a.key, ch[u]), S32);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s0[u] = a.score_cur[i0[u]];
        s1[u] = a.score_cur[i1[u]];
        s2[u] = a.score_cur[i2[u]];
        s3[u] = a.score_cur[i3[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pa[u] = (s0[u] < s1[u]) ? i1[u] : i0[u];
        pb[u] = (s2[u] < s3[u]) ? i3[u] : i2[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const Pool<GS> pool{pw[u], gbase};
        pa[u] = word_to_index(pool.get(W_SEL + 0, a.key, ch[u]), S32);
        pb[u] = word_to_index(pool.get(W_SEL + 1, a.key, ch[u]), S32);
      }
    }
    bool el[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      el[u] = ch[u] < a.n_elite;
      if (el[u]) {
        pa[u] = a.elite_idx ? a.elite_idx[ch[u]] : *lds_elite;
        pb[u] = pa[u];
      }
    }
    // ---- phase 2: parent rows (U x 2 dwordx4 loads in flight) ----
    float4 A4[U], B4[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      A4[u] = cur[(uint64_t)pa[u] * rs + qc];
      B4[u] = cur[(uint64_t)pb[u] * rs + qc];
    }
    // ---- phase 3: variation + store ----
    float v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float A[4] = {A4[u].x, A4[u].y, A4[u].z, A4[u].w}, B[4] = {B4[u].x, B4[u].y, B4[u].z, B4[u].w};
      if (el[u]) {
        for (int j = 0; j < 4; ++j) v[u][j] = A[j];
      } else {
        const Pool<GS> pool{pw[u], gbase};
        const bool xo = a.crossover != XO_NONE && do_crossover(a, pool.get(W_XOPROB, a.key, ch[u]));
        uint32_t blo = 0, bhi = 0;
        float ua = 0.f;
        if (a.crossover == XO_ONE_POINT) {
          blo = word_to_index(pool.get(W_CUT1, a.key, ch[u]), L);
          bhi = L;
        } else if (a.crossover == XO_TWO_POINT) {
          const uint32_t c1 = word_to_index(pool.get(W_CUT1, a.key, ch[u]), L);
          const uint32_t c2 = word_to_index(pool.get(W_CUT2, a.key, ch[u]), L);
          blo = c1 < c2 ? c1 : c2;
          bhi = c1 < c2 ? c2 : c1;
        } else if (a.crossover == XO_ARITHMETIC) {
          ua = word_to_unit(pool.get(W_CUT1, a.key, ch[u]));
        }
        real_cross_chunk(a, ch[u], q, A, B, xo, blo, bhi, ua, v[u]);
        if (per_gene_mut) {
          if (have) real_mutate_chunk(a, ch[u], q, clen, pw[u].w, lds_thr, v[u]);
        } else if (reset_one && pool.get(W_MUTIND, a.key, ch[u]) < a.mut_ind_thresh) {
          const uint32_t pos = word_to_index(pool.get(W_MUTPOS, a.key, ch[u]), L);
          const float x = real_reset_value(a, pool.get(W_SEL + sel_words(a), a.key, ch[u]));
          if ((pos >> 2) == q) {
            const uint32_t j = pos & 3u;
            v[u][0] = j == 0 ? x : v[u][0];
            v[u][1] = j == 1 ? x : v[u][1];
            v[u][2] = j == 2 ? x : v[u][2];
            v[u][3] = j == 3 ? x : v[u][3];
          }
        }
      }
      for (uint32_t j = 0; j < 4; ++j) v[u][j] = j < clen ? v[u][j] : 0.f;
      if (ch[u] < a.S && have) nxt[ch[u] * rs + q] = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
    }
    if (!evals) continue;
    // ---- phase 4: objective (rotated: one MFMA pass over the U*GPB-row tile) ----
    float z[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = 4 * q + j;
        z[u][j] = d < L ? ((shift) ? v[u][j] - a.obj_data2[d] : v[u][j]) : 0.f;
      }
    if (ROT) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float* row = X + (u * GPB + g) * TW + 4 * q;
        row[0] = z[u][0]; row[1] = z[u][1]; row[2] = z[u][2]; row[3] = z[u][3];
      }
      __syncthreads();
      const uint32_t w = threadIdx.x >> 6;
      const uint32_t nct = dp / 16;
      for (uint32_t t = w; t < (XR / 16) * nct; t += kBlock / 64) {
        const uint32_t rt = t / nct, ct = t % nct;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* xa = X + (rt * 16 + (lane & 15)) * TW + (lane >> 4);
        const float* mb = MS + (ct * 16 + (lane & 15)) * (dp + 1) + (lane >> 4);
        for (uint32_t k0 = 0; k0 < dp; k0 += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[k0], mb[k0], acc, 0, 0, 0);
        float* zo = Z + (rt * 16 + (lane >> 4) * 4) * TW + ct * 16 + (lane & 15);
        zo[0] = acc[0];
        zo[TW] = acc[1];
        zo[2 * TW] = acc[2];
        zo[3 * TW] = acc[3];
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float score;
      if (el[u]) {
        score = a.score_cur[pa[u]];
      } else {
        RealAcc acc{0.f, 0.f, 1.f};
        const float* zrow = Z + (u * GPB + g) * TW + 4 * q;
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t d = 4 * q + j;
          if (d < L) {
            const float zj = ROT ? zrow[j] : z[u][j];
            const float zn = ROT ? zrow[j + 1] : 0.f;  // Rosenbrock only reaches here rotated
            real_obj_term(a, d, zj, zn, v[u][j], acc);
          }
        }
        acc.s0 = group_sum<GS>(acc.s0);
        acc.s1 = group_sum<GS>(acc.s1);
        acc.s2 = group_prod<GS>(acc.s2);
        score = real_obj_finish(a, acc);
      }
      if (ch[u] < a.S && q == 0) {
        a.score_next[ch[u]] = score;
        const unsigned long long pb2 = pack_best(score, ch[u]);
        my_best = pb2 > my_best ? pb2 : my_best;
        st.add(score);
      }
    }
    if (ROT) __syncthreads();  // X/Z are rewritten next iteration
  }
  if (evals && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}


// ---------------------------------------------------------------------------
// Software-pipelined GEN kernel, the REAL analogue of
// binary_gen_pipe: three children per lane group in flight — contestant score
// loads of c+2, parent-row loads of c+1 and the variation / objective of c in
// one loop body, three static register sets rotating X -> Y -> Z so hipcc's
// vmcnt waits stay exact (every load is issued unconditionally; tail children
// are clamped, lanes without a chunk re-read the last chunk).  Tournament-2 or
// random selection, any crossover / mutation, objectives that need no
// neighbouring dimension.  Same semantics as real_kernel (bit-exact).
//
// ROT (GS 4 or 8, i.e. L <= 16 / 32): rotated objective f(M (x - o)) with the
// rotation on the matrix cores, wave-local — no block barrier in the loop.
// Per stage 3 the wave's 64/GS children are transposed through a private
// 16 x 36 LDS tile, multiplied by M^T (rot_tile4), and the outputs go back
// through the same tile to the lanes' own 4-gene chunks.  Same k-ordered
// accumulation as real_gen_fast (bit-exact).  The loop condition is
// wave-uniform here: every lane of the wave takes part in the tile even when
// its own child is past S.  4 waves/SIMD (launch bounds; 3 without them:
// rastrigin30_rot 211 -> 193 us/gen).
constexpr uint32_t kRotTW = 36;  // tile row stride (floats): conflict-free column reads, 16-byte rows

__device__ __forceinline__ void rot_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// z (4 genes of this lane's chunk, shifted) -> rotated z, in place, with
// v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4 blocks, K = 1): the wave's
// C = 64/GS children x DP = 4 GS dims are exactly 16 blocks (C/4 row groups x
// GS column groups), so no tile row is wasted — a 16x16x4 tile leaves half its
// rows empty at GS 8 and measured 4% slower (rastrigin30_rot 201 vs 193 us/gen).
// One k per instruction: each output is the same sequential fma chain as the
// CPU reference.  A = X[child][k] and B = M[n][k] come from LDS as dwordx4 runs
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
  rot_wave_sync();
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
  rot_wave_sync();
#pragma unroll
  for (int i = 0; i < 4; ++i) xw[(4 * rg + i) * kRotTW + nb] = acc[i];
  rot_wave_sync();
  const float4 r = *(const float4*)(xw + row * kRotTW + 4 * q);
  z[0] = r.x;
  z[1] = r.y;
  z[2] = r.z;
  z[3] = r.w;
  rot_wave_sync();
}

template <int GS, int OBJ, bool ROT = false>
__global__ __launch_bounds__(kBlock, ROT ? 4 : 1) void real_gen_pipe(GenArgs a, unsigned long long* best_parts) {
  static_assert(!ROT || GS == 4 || GS == 8, "wave-local rotation: 16 or 32 padded dims");
  resolve_gen(a);
  a.objective = OBJ;  // compile-time objective: the term switches fold away
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  __shared__ uint32_t lds_thr[kMutCap];
  __shared__ __attribute__((aligned(16))) float lds_rot[ROT ? (kBlock / 64 + 2) * 16 * kRotTW : 1];  // 4 wave tiles + M

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  constexpr uint32_t GPB = kBlock / GS;
  const uint64_t rs = a.row_words >> 2;
  const float4* cur = (const float4*)a.cur;
  float4* nxt = (float4*)a.next;
  const uint32_t L = a.L;
  const uint32_t S32 = (uint32_t)a.S;
  const bool have = q < a.chunks;
  const uint32_t qc = have ? q : a.chunks - 1;
  const uint32_t clen = have ? (L - 4 * q >= 4 ? 4u : L - 4 * q) : 0u;
  const bool tour2 = a.selection == SEL_TOURNAMENT;
  const bool xo_on = a.crossover != XO_NONE;
  const bool per_gene_mut = (a.mutation == MUT_GAUSSIAN || a.mutation == MUT_UNIFORM) && a.mut_rate > 0.f;
  const bool reset_one = a.mutation == MUT_RESET_ONE;
  const bool evals = a.objective != OBJ_NONE;
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  // loop-invariant per-lane problem data (no conditional loads inside the pipeline)
  float sh[4], w0[4], w1[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t d = 4 * q + j;
    sh[j] = (shift && d < L) ? a.obj_data2[d] : 0.f;
    w0[j] = 1.f;
    w1[j] = 0.f;
    if (evals && d < L) real_obj_data(a, d, w0[j], w1[j]);
  }
  float* xw = lds_rot + (ROT ? (threadIdx.x >> 6) * 16 * kRotTW : 0);  // this wave's X/Z tile
  float* ms = lds_rot + (ROT ? (kBlock / 64) * 16 * kRotTW : 0);        // M[n][k], block-shared
  if (ROT)
    for (uint32_t i = threadIdx.x; i < 32 * kRotTW; i += kBlock) {
      const uint32_t n = i / kRotTW, k = i % kRotTW;
      ms[i] = (n < L && k < L) ? a.obj_data[n * L + k] : 0.f;
    }

  if (a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
  }
  if (per_gene_mut)
    for (uint32_t i = threadIdx.x; i < kMutCap; i += kBlock) lds_thr[i] = a.mut_thr[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  const uint64_t stride = (uint64_t)gridDim.x * GPB;
  uint64_t c0 = (uint64_t)blockIdx.x * GPB + threadIdx.x / GS;
  while (c0 < a.n_elite && c0 < a.S) {  // elites: copy row and score
    const uint32_t src = a.elite_idx ? a.elite_idx[c0] : lds_elite;
    if (have) nxt[c0 * rs + q] = cur[(uint64_t)src * rs + q];
    const float sc = a.score_cur[src];
    if (q == 0) {
      a.score_next[c0] = sc;
      const unsigned long long pb = pack_best(sc, c0);
      my_best = pb > my_best ? pb : my_best;
      st.add(sc);
    }
    c0 += stride;
  }

#define R_SET(P)                                                      \
  u32x4 P##w{0, 0, 0, 0};                                             \
  uint32_t P##i0 = 0, P##i1 = 0, P##i2 = 0, P##i3 = 0;                \
  float P##t0 = 0.f, P##t1 = 0.f, P##t2 = 0.f, P##t3 = 0.f;           \
  float4 P##A = make_float4(0.f, 0.f, 0.f, 0.f), P##B = P##A;         \
  bool P##xo = false;
  R_SET(X)
  R_SET(Y)
  R_SET(Z)
#undef R_SET

#define R_STAGE1(c, P)                                                 \
  {                                                                    \
    const uint64_t cc_ = (c) < a.S ? (c) : a.S - 1;                    \
    P##w = draw(a.key, ST_CHILD, cc_, q);                              \
    const Pool<GS> pool_{P##w, gbase};                                 \
    P##i0 = word_to_index(pool_.get(W_SEL + 0, a.key, cc_), S32);      \
    P##i1 = word_to_index(pool_.get(W_SEL + 1, a.key, cc_), S32);      \
    P##i2 = word_to_index(pool_.get(W_SEL + 2, a.key, cc_), S32);      \
    P##i3 = word_to_index(pool_.get(W_SEL + 3, a.key, cc_), S32);      \
    P##t0 = a.score_cur[P##i0];                                        \
    P##t1 = a.score_cur[P##i1];                                        \
    P##t2 = a.score_cur[P##i2];                                        \
    P##t3 = a.score_cur[P##i3];                                        \
  }

#define R_STAGE2(c, P)                                                                          \
  {                                                                                             \
    const uint64_t cc_ = (c) < a.S ? (c) : a.S - 1;                                             \
    uint32_t pa_, pb_;                                                                          \
    if (tour2) {                                                                                \
      pa_ = P##i0 ^ ((P##i0 ^ P##i1) & (0u - (uint32_t)(P##t0 < P##t1)));                       \
      pb_ = P##i2 ^ ((P##i2 ^ P##i3) & (0u - (uint32_t)(P##t2 < P##t3)));                       \
    } else {                                                                                    \
      pa_ = P##i0;                                                                              \
      pb_ = P##i1;                                                                              \
    }                                                                                           \
    const Pool<GS> pool_{P##w, gbase};                                                          \
    P##xo = xo_on && do_crossover(a, pool_.get(W_XOPROB, a.key, cc_));                          \
    P##A = cur[(uint64_t)pa_ * rs + qc];                                                        \
    P##B = cur[(uint64_t)pb_ * rs + qc];                                                        \
  }

#define R_VARY(c, P)                                                                            \
  const Pool<GS> pool_{P##w, gbase};                                                            \
  uint32_t lo_ = 0, hi_ = 0;                                                                    \
  float ua_ = 0.f;                                                                              \
  if (a.crossover == XO_ONE_POINT) {                                                            \
    lo_ = word_to_index(pool_.get(W_CUT1, a.key, (c)), L);                                      \
    hi_ = L;                                                                                    \
  } else if (a.crossover == XO_TWO_POINT) {                                                     \
    const uint32_t x1_ = word_to_index(pool_.get(W_CUT1, a.key, (c)), L);                       \
    const uint32_t x2_ = word_to_index(pool_.get(W_CUT2, a.key, (c)), L);                       \
    lo_ = x1_ < x2_ ? x1_ : x2_;                                                                \
    hi_ = x1_ < x2_ ? x2_ : x1_;                                                                \
  } else if (a.crossover == XO_ARITHMETIC) {                                                    \
    ua_ = word_to_unit(pool_.get(W_CUT1, a.key, (c)));                                          \
  }                                                                                             \
  const float A_[4] = {P##A.x, P##A.y, P##A.z, P##A.w};                                         \
  const float B_[4] = {P##B.x, P##B.y, P##B.z, P##B.w};                                         \
  real_cross_chunk(a, (c), q, A_, B_, P##xo, lo_, hi_, ua_, v_);                                \
  if (per_gene_mut) {                                                                           \
    if (have) real_mutate_chunk(a, (c), q, clen, P##w.w, lds_thr, v_);                          \
  } else if (reset_one && pool_.get(W_MUTIND, a.key, (c)) < a.mut_ind_thresh) {                 \
    const uint32_t pos_ = word_to_index(pool_.get(W_MUTPOS, a.key, (c)), L);                    \
    const float x_ = real_reset_value(a, pool_.get(W_SEL + sel_words(a), a.key, (c)));          \
    if ((pos_ >> 2) == q) {                                                                     \
      v_[0] = fsel(pos_ == 4 * q + 0, x_, v_[0]);                                               \
      v_[1] = fsel(pos_ == 4 * q + 1, x_, v_[1]);                                               \
      v_[2] = fsel(pos_ == 4 * q + 2, x_, v_[2]);                                               \
      v_[3] = fsel(pos_ == 4 * q + 3, x_, v_[3]);                                               \
    }                                                                                           \
  }                                                                                             \
  for (uint32_t j = 0; j < 4; ++j) v_[j] = j < clen ? v_[j] : 0.f;                              \
  if (have) nxt[(c) * rs + q] = make_float4(v_[0], v_[1], v_[2], v_[3]);

#define R_EVAL(c, ZE, ZN)                                                                       \
  {                                                                                             \
    RealAcc acc_{0.f, 0.f, 1.f};                                                                \
    _Pragma("unroll") for (uint32_t j = 0; j < 4; ++j) {                                        \
      const uint32_t d_ = 4 * q + j;                                                            \
      if (d_ < L) real_obj_term_w(a, d_, ZE, ZN, v_[j], w0[j], w1[j], acc_);                    \
    }                                                                                           \
    acc_.s0 = group_sum<GS>(acc_.s0);                                                           \
    acc_.s1 = group_sum<GS>(acc_.s1);                                                           \
    acc_.s2 = group_prod<GS>(acc_.s2);                                                          \
    const float sc_ = real_obj_finish(a, acc_);                                                 \
    if (q == 0) {                                                                               \
      a.score_next[(c)] = sc_;                                                                  \
      const unsigned long long pb_ = pack_best(sc_, (c));                                       \
      my_best = pb_ > my_best ? pb_ : my_best;                                                  \
      st.add(sc_);                                                                              \
    }                                                                                           \
  }

#define R_STAGE3(c, P)                                                                               \
  if constexpr (!ROT) {                                                                              \
    if ((c) < a.S) {                                                                                 \
      float v_[4];                                                                                   \
      R_VARY(c, P)                                                                                   \
      if (evals) R_EVAL(c, v_[j] - sh[j], 0.f)                                                       \
    }                                                                                                \
  } else { /* wave-uniform: every lane joins the rotation tile */                                    \
    float v_[4] = {0.f, 0.f, 0.f, 0.f};                                                              \
    const bool live_ = (c) < a.S;                                                                    \
    if (live_) {                                                                                     \
      R_VARY(c, P)                                                                                   \
    }                                                                                                \
    float z_[4], zn_[4];                                                                             \
    _Pragma("unroll") for (uint32_t j = 0; j < 4; ++j) z_[j] = 4 * q + j < L ? v_[j] - sh[j] : 0.f;  \
    rot_tile4<GS>(xw, ms, z_);                                                                       \
    zn_[0] = z_[1];                                                                                  \
    zn_[1] = z_[2];                                                                                  \
    zn_[2] = z_[3];                                                                                  \
    zn_[3] = OBJ == OBJ_ROSENBROCK ? __shfl(z_[0], (int)lane + 1, 64) : 0.f;                         \
    if (live_) R_EVAL(c, z_[j], zn_[j])                                                              \
  }

  // ROT: a wave stays in the loop while any of its groups has a child left
#define R_MORE(c) (ROT ? __any((c) < a.S) != 0 : (c) < a.S)
  R_STAGE1(c0, X)
  R_STAGE2(c0, X)
  R_STAGE1(c0 + stride, Y)
  while (R_MORE(c0)) {  // group-uniform (ROT: wave-uniform)
    R_STAGE1(c0 + 2 * stride, Z)
    R_STAGE2(c0 + stride, Y)
    R_STAGE3(c0, X)
    c0 += stride;
    if (!R_MORE(c0)) break;
    R_STAGE1(c0 + 2 * stride, X)
    R_STAGE2(c0 + stride, Z)
    R_STAGE3(c0, Y)
    c0 += stride;
    if (!R_MORE(c0)) break;
    R_STAGE1(c0 + 2 * stride, Y)
    R_STAGE2(c0 + stride, X)
    R_STAGE3(c0, Z)
    c0 += stride;
  }
#undef R_STAGE1
#undef R_MORE
#undef R_STAGE2
#undef R_STAGE3
#undef R_VARY
#undef R_EVAL

  if (evals && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}

template <int GS, int U, bool ROT>
uint32_t go_fast(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  constexpr uint32_t ROWS = (kBlock / GS) * U;
  constexpr uint32_t XR = ROWS > 16 ? ROWS : 16;
  constexpr uint32_t TW = (4 * GS > 16 ? 4 * GS : 16) + 1;
  const uint32_t dp = ((4 * a.chunks + 15) / 16) * 16;
  const size_t lds = (kHdr + (ROT ? 2 * XR * TW + (size_t)dp * (dp + 1) : 0)) * sizeof(float);
  static bool c = false;
  return launch_occ(real_gen_fast<GS, U, ROT>, ROWS, lds, a, parts, s, c);
}

bool real_fast_eligible(int mode, const GenArgs& a, bool rot) {
  if (mode != MODE_GEN || force_generic_kernels()) return false;
  if (a.objective == OBJ_USER_FNPTR || a.objective == OBJ_TSP_RANDOM_KEY) return false;
  if (a.objective == OBJ_ROSENBROCK && !rot) return false;
  if (!(a.selection == SEL_RANDOM || (a.selection == SEL_TOURNAMENT && a.tour_k == 2))) return false;
  if (a.n_elite > 1 && a.elite_idx == nullptr) return false;
  return true;
}

template <int GS, bool ROT>
uint32_t launch_fast(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  if constexpr (ROT && (GS == 4 || GS == 8)) {
    {
      static bool c[6] = {false, false, false, false, false, false};
      switch (a.objective) {
        case OBJ_SPHERE: return launch_occ(real_gen_pipe<GS, OBJ_SPHERE, true>, kBlock / GS, 0, a, parts, s, c[0]);
        case OBJ_RASTRIGIN:
          return launch_occ(real_gen_pipe<GS, OBJ_RASTRIGIN, true>, kBlock / GS, 0, a, parts, s, c[1]);
        case OBJ_ROSENBROCK:
          return launch_occ(real_gen_pipe<GS, OBJ_ROSENBROCK, true>, kBlock / GS, 0, a, parts, s, c[2]);
        case OBJ_ACKLEY: return launch_occ(real_gen_pipe<GS, OBJ_ACKLEY, true>, kBlock / GS, 0, a, parts, s, c[3]);
        case OBJ_GRIEWANK:
          return launch_occ(real_gen_pipe<GS, OBJ_GRIEWANK, true>, kBlock / GS, 0, a, parts, s, c[4]);
        case OBJ_SCHWEFEL:
          return launch_occ(real_gen_pipe<GS, OBJ_SCHWEFEL, true>, kBlock / GS, 0, a, parts, s, c[5]);
        default: break;
      }
    }
  }
  if (!ROT) {
    static bool c[8] = {false, false, false, false, false, false, false, false};
    switch (a.objective) {
      case OBJ_SPHERE: return launch_occ(real_gen_pipe<GS, OBJ_SPHERE>, kBlock / GS, 0, a, parts, s, c[0]);
      case OBJ_RASTRIGIN: return launch_occ(real_gen_pipe<GS, OBJ_RASTRIGIN>, kBlock / GS, 0, a, parts, s, c[1]);
      case OBJ_ACKLEY: return launch_occ(real_gen_pipe<GS, OBJ_ACKLEY>, kBlock / GS, 0, a, parts, s, c[2]);
      case OBJ_GRIEWANK: return launch_occ(real_gen_pipe<GS, OBJ_GRIEWANK>, kBlock / GS, 0, a, parts, s, c[3]);
      case OBJ_SCHWEFEL: return launch_occ(real_gen_pipe<GS, OBJ_SCHWEFEL>, kBlock / GS, 0, a, parts, s, c[4]);
      case OBJ_LINEAR: return launch_occ(real_gen_pipe<GS, OBJ_LINEAR>, kBlock / GS, 0, a, parts, s, c[5]);
      case OBJ_KNAPSACK_REAL:
        return launch_occ(real_gen_pipe<GS, OBJ_KNAPSACK_REAL>, kBlock / GS, 0, a, parts, s, c[6]);
      case OBJ_NONE: return launch_occ(real_gen_pipe<GS, OBJ_NONE>, kBlock / GS, 0, a, parts, s, c[7]);
      default: break;  // Rosenbrock needs the neighbouring dimension: fast path below
    }
  }
  return go_fast<GS, 1, ROT>(a, parts, s);
}

template <int GS, bool ROT>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (mode) {
    case MODE_GEN:
      if (real_fast_eligible(mode, a, ROT)) return launch_fast<GS, ROT>(a, parts, s);
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
