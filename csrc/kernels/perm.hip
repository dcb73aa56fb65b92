// perm.hip — PERMUTATION encoding (u16 city ids) on gfx950: TSP with PMX /
// OX1 crossover and swap / inversion (2-opt) mutation.
//
// Geometry: a chunk is 8 genes (16 B); a group of GS = group_size(chunks)
// lanes owns one individual (lane q holds chunks q, q+GS, ...); GPB = 256/GS
// individuals per block iteration.  Crossover needs random access to both
// parents and a city->position map, so each child gets four u16 arrays in LDS
// (parent A, parent B, child C, map M; 8 L bytes; 16 KB per block for TSP-256)
// filled by dwordx4 row loads.  OX1 is parallel: keep flags -> group-wide
// prefix scan (ranks in "B order starting at the segment end") -> scatter.
// PMX follows the mapping chains per position.  Tour length: every lane sums
// its own edges (distance matrix from L2, or Euclidean from city coordinates
// staged in LDS), then a GS-lane butterfly.
//
// Reference: the reference has no permutation type; its TSP example encodes
// tours as float random keys and repairs them with a custom crossover that
// keeps an int[110] table per thread (test3/test.cu:48-64).  That semantics is
// kept as OBJ_TSP_RANDOM_KEY in real.hip; this file is the native encoding of
// BASELINE config 5.
#include <hip/hip_runtime.h>

#include <string>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/perm_ops.hpp"

namespace pga {
namespace {

using namespace dev;
constexpr uint16_t kNone = 0xFFFF;
constexpr uint32_t kHdrF = 144;  // floats: red u64[4] (8 floats) | elite | pad  (16-aligned)

inline uint32_t perm_max_length(bool euc) {  // longest genome the one-individual-per-block kernel holds in LDS
  return (uint32_t)((160 * 1024 - 4 * kHdrF - 64 /* static LDS */) / (euc ? 16 : 8)) / 8 * 8;
}

__host__ __device__ inline size_t perm_lds_bytes(uint32_t GS, uint32_t chunks, bool euc, uint32_t blk = 256) {
  const uint32_t gpb = blk / GS;
  const size_t lp = 8ull * chunks;  // genes per padded row
  return 4ull * kHdrF + (euc ? 8ull * chunks * 8 : 0) + (size_t)gpb * 4 * lp * 2;
}

template <int GS>
__device__ __forceinline__ uint32_t group_excl_scan(uint32_t v, uint32_t q, uint32_t& total) {
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < GS; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)inc, o, GS);
    if (q >= (uint32_t)o) inc += t;
  }
  total = (uint32_t)__shfl((int)inc, GS - 1, GS);
  return inc - v;
}

__device__ __forceinline__ void ld8(const uint16_t* p, uint32_t e[8]) {
  const uint4 v = *(const uint4*)p;
  e[0] = v.x & 0xFFFF; e[1] = v.x >> 16; e[2] = v.y & 0xFFFF; e[3] = v.y >> 16;
  e[4] = v.z & 0xFFFF; e[5] = v.z >> 16; e[6] = v.w & 0xFFFF; e[7] = v.w >> 16;
}

template <int GS, int MODE, int OBJ, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void perm_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  float* smem = (float*)pga_dyn_lds;
  unsigned long long* lds_red = (unsigned long long*)smem;
  uint32_t* lds_elite = (uint32_t*)(smem + 8);
  const uint32_t L = a.L, nch = a.chunks, lp = 8 * nch;
  float* coords = smem + kHdrF;  // 2L floats (EUC)
  uint16_t* arena = (uint16_t*)(coords + (OBJ == OBJ_TSP_EUC ? 16 * nch : 0));  // 2L <= 16 nch floats

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  constexpr uint32_t GPB = BLK / GS;
  const uint32_t g = threadIdx.x / GS;
  uint16_t* A = arena + (size_t)g * 4 * lp;
  uint16_t* B = A + lp;
  uint16_t* Cc = B + lp;
  uint16_t* Mp = Cc + lp;
  const uint64_t rs = a.row_words >> 2;
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  constexpr bool CROSSES = MODE == MODE_GEN || MODE == MODE_CROSS;
  constexpr bool MUTATES = MODE == MODE_GEN || MODE == MODE_MUTATE;
  constexpr bool EVALS = OBJ != OBJ_NONE && (MODE == MODE_GEN || MODE == MODE_INIT || MODE == MODE_EVAL);
  const bool mut_on = MUTATES && (a.mutation == MUT_SWAP || a.mutation == MUT_INVERSION);

  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts<BLK>(a.best_cur, a.n_best_cur, lds_red);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (OBJ == OBJ_TSP_EUC)
    for (uint32_t i = threadIdx.x; i < 2 * L; i += BLK) coords[i] = a.obj_data[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t base = (uint64_t)blockIdx.x * GPB; base < a.S; base += (uint64_t)gridDim.x * GPB) {  // block-uniform
    const uint64_t child = base + g;
    const bool valid = child < a.S;  // group-uniform
    bool elite = false, xo = false;
    uint32_t lo = 0, hi = 0;
    float score = 0.f;
    Pool<GS> pool{u32x4{0, 0, 0, 0}, gbase};

    // ---- stage 1: rows -> LDS ----
    if (valid) {
      if (MODE == MODE_GEN && child < a.n_elite) {
        elite = true;
        const uint32_t src = a.elite_idx ? a.elite_idx[child] : *lds_elite;
        for (uint32_t c = q; c < nch; c += GS) *(uint4*)(Cc + 8 * c) = cur[(uint64_t)src * rs + c];
        score = a.score_cur[src];
      } else if (MODE == MODE_INIT) {
        if (q == 0) {  // Durstenfeld shuffle, one lane per child
          for (uint32_t i = 0; i < lp; ++i) Cc[i] = i < L ? (uint16_t)i : (uint16_t)0;
          for (uint32_t i = L - 1; i >= 1; --i) {
            const uint32_t j = word_to_index(perm_init_word(a.key, child, i), i + 1);
            const uint16_t t = Cc[i];
            Cc[i] = Cc[j];
            Cc[j] = t;
          }
        }
      } else if (MODE == MODE_EVAL || MODE == MODE_MUTATE) {
        for (uint32_t c = q; c < nch; c += GS) *(uint4*)(Cc + 8 * c) = cur[child * rs + c];
      }
      if (!elite && (CROSSES || MUTATES)) pool.w = draw(a.key, ST_CHILD, child, q);
      if (!elite && CROSSES) {
        uint32_t pa, pb;
        select_parents<GS>(a, pool, child, pa, pb);
        xo = (a.crossover == XO_PMX || a.crossover == XO_OX) && do_crossover(a, pool.get(W_XOPROB, a.key, child));
        perm_segment(pool.get(W_CUT1, a.key, child), pool.get(W_CUT2, a.key, child), L, lo, hi);
        for (uint32_t c = q; c < nch; c += GS) {
          *(uint4*)(A + 8 * c) = cur[(uint64_t)pa * rs + c];
          if (xo) *(uint4*)(B + 8 * c) = cur[(uint64_t)pb * rs + c];
        }
      }
    }
    __syncthreads();
    // ---- stage 2: crossover into C ----
    if (CROSSES) {
      if (valid && !elite) {
        for (uint32_t c = q; c < nch; c += GS) {
          if (xo) {
            for (uint32_t e = 0; e < 8; ++e) Mp[8 * c + e] = kNone;  // map indexed by city
          } else {
            *(uint4*)(Cc + 8 * c) = *(const uint4*)(A + 8 * c);
          }
        }
      }
      __syncthreads();
      if (valid && !elite && xo)
        for (uint32_t c = q; c < nch; c += GS)
          for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t k = 8 * c + e;
            if (k >= lo && k < hi) Mp[A[k]] = (uint16_t)k;  // city -> its position in A's segment
          }
      __syncthreads();
      if (valid && !elite && xo) {
        if (a.crossover == XO_PMX) {
          for (uint32_t c = q; c < nch; c += GS)
            for (uint32_t e = 0; e < 8; ++e) {
              const uint32_t p = 8 * c + e;
              if (p >= L) {
                Cc[p] = 0;  // row padding
                continue;
              }
              if (p >= lo && p < hi) {
                Cc[p] = A[p];
              } else {
                uint32_t v = B[p];
                for (uint32_t guard = 0; Mp[v] != kNone && guard < L; ++guard) v = B[Mp[v]];
                Cc[p] = (uint16_t)v;
              }
            }
        } else {  // OX1
          // Eb = kept genes of B in [0, hi); K = L - (hi - lo)
          uint32_t eb_part = 0;
          for (uint32_t c = q; c < nch; c += GS)
            for (uint32_t e = 0; e < 8; ++e) {
              const uint32_t p = 8 * c + e;
              if (p < L && p < hi && Mp[B[p]] == kNone) ++eb_part;
            }
          const uint32_t Eb = group_sum_u<GS>(eb_part);
          const uint32_t K = L - (hi - lo), tail = L - hi;
          uint32_t carry = 0;
          for (uint32_t c0 = 0; c0 < nch; c0 += GS) {  // group-uniform
            const uint32_t c = c0 + q;
            uint32_t keep = 0;
            if (c < nch)
              for (uint32_t e = 0; e < 8; ++e) {
                const uint32_t p = 8 * c + e;
                keep |= (p < L && Mp[B[p]] == kNone) ? (1u << e) : 0u;
              }
            uint32_t seg_total;
            const uint32_t ex = group_excl_scan<GS>(__popc(keep), q, seg_total);
            uint32_t run = carry + ex;
            for (uint32_t e = 0; e < 8; ++e) {
              const uint32_t p = 8 * c + e;
              if (c < nch && p >= L) Cc[p] = 0;  // row padding
              if (c < nch && p < L && p >= lo && p < hi) Cc[p] = A[p];
              if ((keep >> e) & 1u) {
                const uint32_t r = p >= hi ? run - Eb : (K - Eb) + run;
                const uint32_t pos = r < tail ? hi + r : r - tail;
                Cc[pos] = B[p];
                ++run;
              }
            }
            carry += seg_total;
          }
        }
      }
      __syncthreads();
    }
    // ---- stage 3: mutation on C ----
    if (MUTATES) {
      if (valid && !elite && mut_on && pool.get(W_MUTIND, a.key, child) < a.mut_ind_thresh) {
        uint32_t i, j;
        perm_mut_positions(pool.get(W_MUTPOS, a.key, child), pool.get(W_SEL + sel_words(a), a.key, child), L, i, j);
        if (a.mutation == MUT_SWAP) {
          if (q == 0) {
            const uint16_t t = Cc[i];
            Cc[i] = Cc[j];
            Cc[j] = t;
          }
        } else {  // reverse C[i..j]
          const uint32_t half = (j - i + 1) / 2;
          for (uint32_t t = q; t < half; t += GS) {
            const uint16_t x = Cc[i + t];
            Cc[i + t] = Cc[j - t];
            Cc[j - t] = x;
          }
        }
      }
      __syncthreads();
    }
    // ---- stage 4: store + evaluate ----
    if (valid) {
      if (MODE != MODE_EVAL)
        for (uint32_t c = q; c < nch; c += GS) nxt[child * rs + c] = *(const uint4*)(Cc + 8 * c);
      if (EVALS && !elite) {
        float len = 0.f;
        const uint32_t last = (OBJ == OBJ_TSP_OPEN) ? L - 1 : L;
        for (uint32_t c = q; c < nch; c += GS) {
          uint32_t e8[8];
          ld8(Cc + 8 * c, e8);
          for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t p = 8 * c + e;
            if (p >= last) break;
            // min(): a forged row (e.g. a corrupted migrant) can never index out of bounds
            const uint32_t u = min(e8[e], L - 1),
                           w = min((e < 7 && p + 1 < L) ? e8[e + 1] : (uint32_t)Cc[(p + 1 == L) ? 0 : p + 1], L - 1);
            if (OBJ == OBJ_TSP_EUC) {
              const float dx = coords[2 * u] - coords[2 * w], dy = coords[2 * u + 1] - coords[2 * w + 1];
              len += sqrtf(fmaf(dx, dx, dy * dy));
            } else {
              len += a.obj_data[u * L + w];
            }
          }
        }
        score = -group_sum<GS>(len);
      }
      if (EVALS && q == 0) {
        a.score_next[child] = score;
        const unsigned long long pb = pack_best(score, child);
        my_best = pb > my_best ? pb : my_best;
        st.add(score);
      }
    }
    __syncthreads();  // C is rewritten next iteration
  }
  if (EVALS && best_parts) {
    unsigned long long b = block_max_u64<BLK>(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store<BLK>(st, a.stats_parts);
  }
}


// ---------------------------------------------------------------------------
// Fast GEN path for rows of at most 64 chunks (L <= 512 cities): one chunk per
// lane, so a child never leaves its wave.  Everything a child needs from LDS
// (parent B for PMX chains, the city -> position map, the OX scatter target)
// is exchanged inside the wave with wave-level barriers instead of
// __syncthreads: the four waves of a block drift independently and hide each
// other's latency.  Parent chunks, the child chunk and the tour edges live in
// registers (one dwordx4 per row per lane; the edge to the next lane's first
// city is a shuffle).  Same operator semantics as perm_kernel (bit-exact).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// u16 gene e (0..7, a compile-time constant after unrolling) of a packed chunk
__device__ __forceinline__ uint32_t get16(const uint4& v, uint32_t e) {
  const uint32_t w = e < 2 ? v.x : (e < 4 ? v.y : (e < 6 ? v.z : v.w));
  return (e & 1u) ? (w >> 16) : (w & 0xFFFFu);
}
__device__ __forceinline__ uint4 set16(uint4 v, uint32_t e, uint32_t x) {
  const uint32_t sh = (e & 1u) * 16u, m = 0xFFFFu << sh;
  if (e < 2) v.x = (v.x & ~m) | (x << sh);
  else if (e < 4) v.y = (v.y & ~m) | (x << sh);
  else if (e < 6) v.z = (v.z & ~m) | (x << sh);
  else v.w = (v.w & ~m) | (x << sh);
  return v;
}

// TBL (integer distance matrices, the launcher's choice): the matrix as u16
// in LDS (GenArgs::obj_aux, staged once per block) instead of an f32 L2
// gather per edge — 1 = a symmetric matrix's strict lower triangle plus its
// diagonal (65 KB at L = 256, so 1024-thread blocks still fit: 16 waves share
// one table per CU), 2 = the full matrix.  Entries are exact (u16 -> f32),
// so the tour sums equal the f32-matrix kernel's bit for bit.
template <int GS, int OBJ, int TBL = 0>
__device__ __forceinline__ void perm_gen_fast_body(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  float* smem = (float*)pga_dyn_lds;
  unsigned long long* lds_red = (unsigned long long*)smem;  // 16 entries: kHdrF holds them
  uint32_t* lds_elite = (uint32_t*)(smem + 32);
  const uint32_t L = a.L, nch = a.chunks, lp = 8 * nch;
  const uint32_t BLK = blockDim.x, NWv = BLK >> 6;
  float* coords = smem + kHdrF;
  uint16_t* arena = (uint16_t*)(coords + (OBJ == OBJ_TSP_EUC ? 16 * nch : 0));
  // the table after the groups' arrays (16-byte aligned: lp is a multiple of 8)
  uint16_t* tab = arena + (size_t)(BLK / GS) * 4 * lp;
  const uint32_t tri = L * (L - 1) / 2;  // TBL 1: the diagonal's offset

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  const uint32_t GPB = BLK / GS;
  const uint32_t g = threadIdx.x / GS;
  uint16_t* B = arena + (size_t)g * 4 * lp + lp;
  uint16_t* Cc = B + lp;
  uint16_t* Mp = Cc + lp;
  const uint64_t rs = a.row_words >> 2;
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  const bool have = q < nch;
  const uint32_t qc = have ? q : nch - 1;
  const bool mut_on = a.mutation == MUT_SWAP || a.mutation == MUT_INVERSION;
  const bool xo_kind = a.crossover == XO_PMX || a.crossover == XO_OX;
  const bool pmx = a.crossover == XO_PMX;
  const uint32_t S32 = (uint32_t)a.S;

  if (a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts_n(a.best_cur, a.n_best_cur, lds_red, NWv);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (OBJ == OBJ_TSP_EUC)
    for (uint32_t i = threadIdx.x; i < 2 * L; i += BLK) coords[i] = a.obj_data[i];
  if (TBL)
    for (uint32_t i = threadIdx.x; i < a.obj_aux_bytes / 16; i += BLK) ((uint4*)tab)[i] = ((const uint4*)a.obj_aux)[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  for (uint64_t base = (uint64_t)blockIdx.x * GPB; base < a.S; base += (uint64_t)gridDim.x * GPB) {
    const uint64_t child = base + g;
    const bool valid = child < a.S;  // group-uniform
    const uint64_t ch = valid ? child : a.S - 1;
    const Pool<GS> pool{draw(a.key, ST_CHILD, ch, q), gbase};
    uint32_t pa, pb;
    select_parents<GS>(a, pool, ch, pa, pb);
    const bool elite = ch < a.n_elite;
    if (elite) {
      pa = a.elite_idx ? a.elite_idx[ch] : *lds_elite;
      pb = pa;
    }
    const bool xo = !elite && xo_kind && do_crossover(a, pool.get(W_XOPROB, a.key, ch));
    uint32_t lo, hi;
    perm_segment(pool.get(W_CUT1, a.key, ch), pool.get(W_CUT2, a.key, ch), L, lo, hi);
    // parent / child chunks stay packed (8 x u16 in 4 VGPRs each)
    const uint4 Av = cur[(uint64_t)pa * rs + qc];
    const uint4 Bv = cur[(uint64_t)pb * rs + qc];
    uint4 Cv = Av;
    float score = 0.f;
    if (elite) score = a.score_cur[pa];

    if (xo) {  // group-uniform
      if (have) {
        *(uint4*)(Mp + 8 * q) = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (pmx) *(uint4*)(B + 8 * q) = Bv;  // PMX follows chains through B
      }
      wave_sync();
#pragma unroll
      for (uint32_t e = 0; e < 8; ++e) {
        const uint32_t k = 8 * q + e;
        if (have && k >= lo && k < hi) Mp[get16(Av, e)] = (uint16_t)k;  // city -> its position in A's segment
      }
      wave_sync();
      if (pmx) {
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t p = 8 * q + e;
          uint32_t v = get16(Bv, e);
          if (p < L && !(p >= lo && p < hi))
            for (uint32_t guard = 0; Mp[v] != kNone && guard < L; ++guard) v = B[Mp[v]];
          Cv = set16(Cv, e, p >= L ? 0u : ((p >= lo && p < hi) ? get16(Av, e) : v));
        }
      } else {  // OX1 (same ranks as perm_kernel)
        uint32_t keep = 0, eb_part = 0;
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t p = 8 * q + e;
          const bool k = have && p < L && Mp[get16(Bv, e)] == kNone;
          keep |= k ? (1u << e) : 0u;
          eb_part += (k && p < hi) ? 1u : 0u;
        }
        const uint32_t Eb = group_sum_u<GS>(eb_part);
        const uint32_t K = L - (hi - lo), tail = L - hi;
        uint32_t seg_total;
        uint32_t run = group_excl_scan<GS>(__popc(keep), q, seg_total);
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t p = 8 * q + e;
          if (have && p >= L) Cc[p] = 0;
          if (have && p < L && p >= lo && p < hi) Cc[p] = (uint16_t)get16(Av, e);
          if ((keep >> e) & 1u) {
            const uint32_t r = p >= hi ? run - Eb : (K - Eb) + run;
            const uint32_t pos = r < tail ? hi + r : r - tail;
            Cc[pos] = (uint16_t)get16(Bv, e);
            ++run;
          }
        }
        wave_sync();
        Cv = *(const uint4*)(Cc + 8 * qc);
      }
    }

    if (!elite && mut_on && pool.get(W_MUTIND, a.key, ch) < a.mut_ind_thresh) {  // group-uniform
      uint32_t i, j;
      perm_mut_positions(pool.get(W_MUTPOS, a.key, ch), pool.get(W_SEL + sel_words(a), a.key, ch), L, i, j);
      wave_sync();  // earlier readers of C are done
      if (have) *(uint4*)(Cc + 8 * q) = Cv;
      wave_sync();
      if (a.mutation == MUT_SWAP) {
        if (q == 0) {
          const uint16_t t = Cc[i];
          Cc[i] = Cc[j];
          Cc[j] = t;
        }
      } else {
        const uint32_t half = (j - i + 1) / 2;
        for (uint32_t t = q; t < half; t += GS) {
          const uint16_t x = Cc[i + t];
          Cc[i + t] = Cc[j - t];
          Cc[j - t] = x;
        }
      }
      wave_sync();
      Cv = *(const uint4*)(Cc + 8 * qc);
    }
    wave_sync();  // the next child of this group rewrites B / C / M

    if (valid && have) nxt[child * rs + q] = Cv;
    if (!elite) {
      // edges (p, p+1) and the closing edge; the city after a lane's chunk is
      // the next lane's first city
      const uint32_t c0 = Cv.x & 0xFFFFu;
      const uint32_t next_first = (uint32_t)__shfl((int)c0, (int)(gbase + ((q + 1) & (GS - 1))), 64);
      const uint32_t first = (uint32_t)__shfl((int)c0, (int)gbase, 64);
      const uint32_t last = (OBJ == OBJ_TSP_OPEN) ? L - 1 : L;
      float len = 0.f;
      if (OBJ == OBJ_TSP_EUC) {
        // one float2 per city of the chunk (+ the following city), reused by both edge ends
        const float2* xy = (const float2*)coords;
        float2 pu = xy[min(get16(Cv, 0), L - 1)];
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t p = 8 * q + e;
          const uint32_t nx = p + 1 < L ? (e < 7 ? get16(Cv, e + 1) : next_first) : first;
          const float2 pw = xy[min(nx, L - 1)];
          if (have && p < last) {
            const float dx = pu.x - pw.x, dy = pu.y - pw.y;
            len += sqrtf(fmaf(dx, dx, dy * dy));
          }
          pu = pw;
        }
      } else {
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t p = 8 * q + e;
          if (have && p < last) {
            const uint32_t nx = p + 1 < L ? (e < 7 ? get16(Cv, e + 1) : next_first) : first;
            const uint32_t u = min(get16(Cv, e), L - 1), w = min(nx, L - 1);
            if constexpr (TBL == 1) {
              const uint32_t hi_ = u > w ? u : w, lo_ = u > w ? w : u;
              len += (float)tab[hi_ == lo_ ? tri + u : hi_ * (hi_ - 1) / 2 + lo_];
            } else if constexpr (TBL == 2) {
              len += (float)tab[u * L + w];
            } else {
              len += a.obj_data[u * L + w];
            }
          }
        }
      }
      score = -group_sum<GS>(len);
    }
    if (valid && q == 0) {
      a.score_next[child] = score;
      const unsigned long long pb2 = pack_best(score, child);
      my_best = pb2 > my_best ? pb2 : my_best;
      st.add(score);
    }
  }
  if (best_parts) {
    unsigned long long b = block_max_u64_n(my_best, lds_red, NWv);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store_n(st, a.stats_parts, NWv);
  }
}

// the LDS-table variants launch up to 1024 threads (one table per CU); the L2
// path and the batch kernel launch kBlock, so they keep kBlock's register cap
template <int GS, int OBJ, int TBL = 0>
__global__ __launch_bounds__(TBL ? 1024 : kBlock) void perm_gen_fast(GenArgs a, unsigned long long* best_parts) {
  perm_gen_fast_body<GS, OBJ, TBL>(a, best_parts);
}

// Batched islands: up to kPermMaxBatch same-shape islands in ONE launch,
// island = blockIdx.y (the binary / real batched kernels' scheme; the tour
// evaluation from each island's f32 matrix or coordinates).  Reference: at
// most MAX_POPULATIONS = 10 islands per solver (include/pga.h:44), run one
// after another (src/pga.cu:272-276).
constexpr uint32_t kPermMaxBatch = 10;
struct PermBatch {
  GenArgs a[kPermMaxBatch];
  unsigned long long* parts[kPermMaxBatch];
};
template <int GS, int OBJ>
__global__ __launch_bounds__(kBlock) void perm_gen_fast_batch(PermBatch b) {
  perm_gen_fast_body<GS, OBJ, 0>(b.a[blockIdx.y], b.parts[blockIdx.y]);
}

// Genomes beyond kPermMaxL genes: one 64-lane block per individual, so the
// four per-child LDS arrays (8 L bytes, +8 L of EUC coordinates) fit in
// 160 KiB up to ~20 000 cities (u16 ids cap L at 65 535 anyway)
template <int MODE, int OBJ>
uint32_t go_long(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  const size_t lds = perm_lds_bytes(64, a.chunks, OBJ == OBJ_TSP_EUC, 64);
  auto k = perm_kernel<64, MODE, OBJ, 64>;
  const size_t avail = allow_dynamic_lds((const void*)k);
  if (lds > avail)
    throw std::invalid_argument("PERMUTATION genome too long for the LDS-resident crossover (" + std::to_string(a.L) +
                                " genes; at most " + std::to_string(perm_max_length(OBJ == OBJ_TSP_EUC)) + ")");
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, 64, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  uint64_t cap = (uint64_t)device_cu_count() * per_cu;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t grid = (uint32_t)(a.S < cap ? a.S : cap);
  hipLaunchKernelGGL(k, grid, 64, lds, s, a, parts);
  return grid;
}

template <int GS, int MODE, int OBJ>
uint32_t go(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  if (GS == 64 && a.L > kPermMaxL) return go_long<MODE, OBJ>(a, parts, s);
  const size_t lds = perm_lds_bytes(GS, a.chunks, OBJ == OBJ_TSP_EUC);
  auto k = perm_kernel<GS, MODE, OBJ>;
  (void)allow_dynamic_lds((const void*)k);
  const uint32_t gpb = kBlock / GS;
  const uint64_t need = (a.S + gpb - 1) / gpb;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, kBlock, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  uint64_t cap = (uint64_t)device_cu_count() * per_cu;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t grid = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL(k, grid, kBlock, lds, s, a, parts);
  return grid;
}

template <int GS, int OBJ, int TBL>
uint32_t go_fast_blk(const GenArgs& a, unsigned long long* parts, hipStream_t s, uint32_t blk) {
  const size_t lds = perm_lds_bytes(GS, a.chunks, OBJ == OBJ_TSP_EUC, blk) + (TBL ? a.obj_aux_bytes : 0);
  auto k = perm_gen_fast<GS, OBJ, TBL>;
  const size_t avail = allow_dynamic_lds((const void*)k);
  if constexpr (TBL != 0) {  // the table did not fit this device's limit: the L2 matrix path
    if (lds > avail) return go_fast_blk<GS, OBJ, 0>(a, parts, s, kBlock);
  }
  const uint32_t gpb = blk / GS;
  const uint64_t need = (a.S + gpb - 1) / gpb;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, (int)blk, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  uint64_t cap = (uint64_t)device_cu_count() * per_cu;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t grid = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL(k, grid, blk, lds, s, a, parts);
  return grid;
}

template <int GS, int OBJ>
uint32_t go_fast(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  if constexpr (OBJ == OBJ_TSP || OBJ == OBJ_TSP_OPEN) {
    // an integer matrix as u16 in LDS: the largest block (up to 16 waves,
    // one table per CU) whose group arrays fit beside it
    // (OX / no crossover: TSP-256 OX 3,265 -> 4,013 gens/s; PMX's chain
    // walks want the 256-thread occupancy more: 2,793 vs 2,650, L2 path kept)
    if (a.obj_aux && (a.obj_aux_kind == 1 || a.obj_aux_kind == 2) && a.obj_aux_bytes % 16 == 0 &&
        a.crossover != XO_PMX) {
      const size_t avail = 160 * 1024 - 1024;  // less the static LDS (block reductions)
      for (uint32_t blk : {1024u, 512u, 256u}) {
        if (perm_lds_bytes(GS, a.chunks, false, blk) + a.obj_aux_bytes > avail) continue;
        if (a.obj_aux_kind == 1) return go_fast_blk<GS, OBJ, 1>(a, parts, s, blk);
        return go_fast_blk<GS, OBJ, 2>(a, parts, s, blk);
      }
    }
  }
  return go_fast_blk<GS, OBJ, 0>(a, parts, s, kBlock);
}

template <int GS, int OBJ>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (mode) {
    case MODE_GEN:
      if (OBJ != OBJ_NONE && a.chunks <= (uint32_t)GS && !force_generic_kernels()) return go_fast<GS, OBJ>(a, parts, s);
      return go<GS, MODE_GEN, OBJ>(a, parts, s);
    case MODE_INIT: return go<GS, MODE_INIT, OBJ>(a, parts, s);
    case MODE_EVAL: return go<GS, MODE_EVAL, OBJ>(a, parts, s);
    case MODE_CROSS: return go<GS, MODE_CROSS, OBJ_NONE>(a, parts, s);
    default: return go<GS, MODE_MUTATE, OBJ_NONE>(a, parts, s);
  }
}

template <int GS>
uint32_t launch_obj(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (a.objective) {
    case OBJ_TSP: return launch_mode<GS, OBJ_TSP>(mode, a, parts, s);
    case OBJ_TSP_OPEN: return launch_mode<GS, OBJ_TSP_OPEN>(mode, a, parts, s);
    case OBJ_TSP_EUC: return launch_mode<GS, OBJ_TSP_EUC>(mode, a, parts, s);
    default: return launch_mode<GS, OBJ_NONE>(mode, a, parts, s);
  }
}

template <int GS, int OBJ>
uint32_t batch_go(PermBatch& b, uint32_t n, hipStream_t s) {
  const GenArgs& a0 = b.a[0];
  const size_t lds = perm_lds_bytes(GS, a0.chunks, OBJ == OBJ_TSP_EUC);
  const void* k = (const void*)perm_gen_fast_batch<GS, OBJ>;
  static bool configured = false;
  if (!configured) {
    allow_dynamic_lds(k);
    configured = true;
  }
  const uint32_t gpb = kBlock / GS;
  const uint64_t need = (a0.S + gpb - 1) / gpb;
  uint64_t cap = (uint64_t)device_cu_count() * occupancy_blocks(k, kBlock, lds) / n;  // the device split
  if (cap < 1) cap = 1;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t gx = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL((perm_gen_fast_batch<GS, OBJ>), dim3(gx, n), kBlock, lds, s, b);
  PGA_HIP_CHECK(hipGetLastError());
  return gx;
}

template <int GS>
uint32_t batch_obj(PermBatch& b, uint32_t n, hipStream_t s) {
  switch (b.a[0].objective) {
    case OBJ_TSP: return batch_go<GS, OBJ_TSP>(b, n, s);
    case OBJ_TSP_OPEN: return batch_go<GS, OBJ_TSP_OPEN>(b, n, s);
    case OBJ_TSP_EUC: return batch_go<GS, OBJ_TSP_EUC>(b, n, s);
    default: return 0;
  }
}

}  // namespace

uint32_t perm_max_batch() { return kPermMaxBatch; }

uint32_t perm_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s) {
  if (n == 0 || n > kPermMaxBatch || force_generic_kernels()) return 0;
  const GenArgs& a0 = args[0];
  if (a0.objective != OBJ_TSP && a0.objective != OBJ_TSP_OPEN && a0.objective != OBJ_TSP_EUC) return 0;
  if (a0.chunks > 64u || a0.L > 65535) return 0;  // the fast kernel: one chunk per lane
  PermBatch b;
  for (uint32_t i = 0; i < n; ++i) {
    const GenArgs& a = args[i];
    if (a.S != a0.S || a.L != a0.L || a.chunks != a0.chunks || a.objective != a0.objective) return 0;
    b.a[i] = a;
    b.parts[i] = parts[i];
  }
  switch (group_size(a0.chunks)) {
    case 1: return batch_obj<1>(b, n, s);
    case 2: return batch_obj<2>(b, n, s);
    case 4: return batch_obj<4>(b, n, s);
    case 8: return batch_obj<8>(b, n, s);
    case 16: return batch_obj<16>(b, n, s);
    case 32: return batch_obj<32>(b, n, s);
    default: return batch_obj<64>(b, n, s);
  }
}

uint32_t perm_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  if (a.L > 65535) throw std::invalid_argument("PERMUTATION encoding supports at most 65535 genes (u16 city ids)");
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
