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

#include <cstdlib>
#include <string>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/perm_ops.hpp"

namespace pga {
namespace {

using namespace dev;
constexpr uint16_t kNone = 0xFFFF;
// experiment builds only (tools/variants.sh): tournaments, crossover or the
// tour evaluation switched off in perm_gen_fast, to split its time
#ifndef PGA_PERM_NOSEL
#define PGA_PERM_NOSEL 0
#endif
#ifndef PGA_PERM_NOXO
#define PGA_PERM_NOXO 0
#endif
#ifndef PGA_PERM_PF  // parent rows one step ahead
#define PGA_PERM_PF 1
#endif
#ifndef PGA_PERM_NOEVAL
#define PGA_PERM_NOEVAL 0
#endif
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

// The same exclusive scan for groups of 16, 32 or 64 lanes on DPP row
// shifts and row broadcasts (VALU, no LDS crossbar round trip per level);
// smaller groups take group_excl_scan.  Integer sums: any order is exact.
template <int GS>
__device__ __forceinline__ uint32_t group_excl_scan_dpp(uint32_t v, uint32_t q, uint32_t& total) {
  if constexpr (GS < 16) {
    return group_excl_scan<GS>(v, q, total);
  } else {
    int inc = (int)v;
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xf, 0xf, false);  // row_shr:1
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xf, 0xf, false);  // row_shr:2
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xf, 0xf, false);  // row_shr:4
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xf, 0xf, false);  // row_shr:8
    if constexpr (GS >= 32) inc += __builtin_amdgcn_update_dpp(0, inc, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    if constexpr (GS == 64) inc += __builtin_amdgcn_update_dpp(0, inc, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    if constexpr (GS == 16) {
      total = (uint32_t)__shfl(inc, (int)((lane_id() & ~15u) | 15u), 64);
    } else if constexpr (GS == 32) {
      const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane(inc, 31), t1 = (uint32_t)__builtin_amdgcn_readlane(inc, 63);
      total = lane_id() < 32u ? t0 : t1;
    } else {
      total = (uint32_t)__builtin_amdgcn_readlane(inc, 63);
    }
    (void)q;
    return (uint32_t)inc - v;
  }
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
    bool forged = false;
    if constexpr (MODE == MODE_EVAL) {
      // a row that is not a permutation of 0..L-1 (a corrupted or forged
      // migrant) becomes the identity tour and is scored as one: Mp[city] =
      // a position holding it; a duplicate city leaves one of its positions
      // unclaimed, a city >= L is rejected outright (cpu_perm.cpp: the same)
      if (valid)
        for (uint32_t c = q; c < nch; c += GS) *(uint4*)(Mp + 8 * c) = make_uint4(~0u, ~0u, ~0u, ~0u);
      __syncthreads();
      uint32_t bad = 0;
      if (valid)
        for (uint32_t p = q; p < L; p += GS) {
          const uint32_t v = Cc[p];
          if (v >= L) bad = 1;
          else Mp[v] = (uint16_t)p;
        }
      __syncthreads();
      if (valid)
        for (uint32_t p = q; p < L; p += GS) {
          const uint32_t v = Cc[p];
          if (v < L && Mp[v] != p) bad = 1;
        }
      forged = valid && group_sum_u<GS>(bad) != 0;  // group-uniform
      if (forged)
        for (uint32_t p = q; p < lp; p += GS) Cc[p] = p < L ? (uint16_t)p : (uint16_t)0;
      __syncthreads();
    }
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
      if (MODE != MODE_EVAL || forged)
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
// lane, so a child never leaves its wave.  Two phases per BATCH of 64
// consecutive children (a wave's unit of work, wave-strided over the grid):
//   SELECT  one lane per child: the child's selection words (its ST_CHILD
//           Philox blocks, the words select_parents reads from the group's
//           pool) and every score load of the 64 tournaments in flight at once;
//           the parents stay in two VGPRs (lane j: child j of the batch)
//   BREED   NG = 64 / GS children per step, one chunk per lane; the parent
//           rows of step t + 1 are loaded before step t's crossover, so a
//           step waits for no load of its own
// (before round 5 every step drew its selection words, waited for its four
// scores, then for its rows: tournaments measured 92 of 273 us per
// generation at TSP-256 OX).  Everything a child needs from LDS (the PMX
// mapping, the OX membership bits and scatter target) is exchanged inside the
// wave with wave-level barriers instead of __syncthreads.  Parent chunks, the
// child chunk and the tour edges live in registers (one dwordx4 per row per
// lane; the edge to the next lane's first city is a shuffle).  Same operator
// semantics as perm_kernel (bit-exact).
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

// bit e set when position base + e lies in [a, b) (a lane's 8 genes)
__device__ __forceinline__ uint32_t range8(uint32_t base, uint32_t a, uint32_t b) {
  const uint32_t lo = a > base ? min(a - base, 8u) : 0u;
  const uint32_t hi = b > base ? min(b - base, 8u) : 0u;
  return ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}
// 8 gene bits -> the 16-bit lanes of a packed chunk (0xFFFF where set)
__device__ __forceinline__ uint4 mask16x8(uint32_t m) {
  const auto w = [m](uint32_t i) {
    return (((m >> (2 * i)) & 1u) ? 0xFFFFu : 0u) | (((m >> (2 * i + 1)) & 1u) ? 0xFFFF0000u : 0u);
  };
  return make_uint4(w(0), w(1), w(2), w(3));
}
// per 16-bit lane: a where the mask is set, else b (v_bfi_b32)
__device__ __forceinline__ uint4 bfi4(const uint4& m, const uint4& a, const uint4& b) {
  return make_uint4((a.x & m.x) | (b.x & ~m.x), (a.y & m.y) | (b.y & ~m.y), (a.z & m.z) | (b.z & ~m.z),
                    (a.w & m.w) | (b.w & ~m.w));
}
__device__ __forceinline__ uint4 pack16x8(const uint32_t v[8]) {
  return make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
}

// One lane's view of its own child's ST_CHILD words (the pool's words, core.hpp
// child_word): blocks 1 and 2 hold the selection words W_SEL .. W_SEL + 3 of
// tournament-2, roulette and uniform selection; other words are drawn on demand
template <int GS>
struct LanePool {
  u32x4 b1, b2;
  __device__ __forceinline__ uint32_t get(uint32_t t, const RngKey& key, uint64_t child) const {
    if (t / 3u == 1u) return sel3(b1, t % 3u);
    if (t / 3u == 2u) return sel3(b2, t % 3u);
    return child_word(key, child, t);
  }
};

// Per-group LDS of the fast kernel: one lp-gene u16 array (PMX: the mapping
// T, then the child for mutation; OX: the scatter target) and 64 bytes of OX
// membership bits (one per city) — a quarter of perm_kernel's four arrays,
// so a 16-wave block keeps its 32 groups beside a 131.6 KB f32 triangle
__host__ __device__ inline size_t perm_fast_group_bytes(uint32_t chunks) { return 16ull * chunks + 64; }
__host__ __device__ inline size_t perm_fast_lds_bytes(uint32_t GS, uint32_t chunks, bool euc, uint32_t blk) {
  return 4ull * kHdrF + (euc ? 8ull * chunks * 8 : 0) + (size_t)(blk / GS) * perm_fast_group_bytes(chunks);
}

// TBL (the launcher's choice from GenArgs::obj_aux): the distance matrix in
// LDS (staged once per block) instead of an f32 L2 gather per edge — 1 = a
// symmetric integer matrix's lower triangle with the diagonal as u16, row by
// row (entry (i, j <= i) at i (i + 1) / 2 + j; 65 KB at L = 256), 2 = a full
// integer matrix as u16, 3 = a symmetric f32 matrix's lower triangle with the
// diagonal as f32 (131.6 KB at L = 256: the 16 waves of a CU share one).  Entries are the matrix's own values, so the tour sums
// equal the f32 L2 path's bit for bit.
// FULL (the launcher's choice when L = 8 GS: every lane holds a whole chunk,
// no padding): the lane masks below fold to constants, L is a compile-time
// constant, and for L <= 256 the tour's triangle indices are computed two
// edges per packed 16-bit instruction.
template <int GS, int OBJ, int TBL = 0, bool FULL = false>
__device__ __forceinline__ void perm_gen_fast_body(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  float* smem = (float*)pga_dyn_lds;
  unsigned long long* lds_red = (unsigned long long*)smem;  // 16 entries: kHdrF holds them
  uint32_t* lds_elite = (uint32_t*)(smem + 32);
  const uint32_t L = FULL ? 8u * GS : a.L, nch = FULL ? (uint32_t)GS : a.chunks, lp = 8 * nch;
  const uint32_t BLK = blockDim.x, NWv = BLK >> 6;
  constexpr uint32_t NG = 64 / GS;  // children per wave per step
  float* coords = smem + kHdrF;
  char* arena = (char*)(coords + (OBJ == OBJ_TSP_EUC ? 16 * nch : 0));
  const size_t gbytes = perm_fast_group_bytes(nch);
  // the table after the groups' arrays (16-byte aligned: gbytes is a multiple of 16)
  const uint16_t* tab = (const uint16_t*)(arena + (size_t)(BLK / GS) * gbytes);
  const float* ftab = (const float*)tab;

  const uint32_t lane = lane_id();
  const uint32_t q = lane & (GS - 1);
  const uint32_t gbase = lane & ~(uint32_t)(GS - 1);
  const uint32_t g = lane / GS;
  uint16_t* Cc = (uint16_t*)(arena + (size_t)(threadIdx.x / GS) * gbytes);  // PMX: T; OX: A's inverse; then the child
  const uint64_t rs = a.row_words >> 2;
  const uint4* cur = (const uint4*)a.cur;
  uint4* nxt = (uint4*)a.next;
  const bool have = FULL || q < nch;
  const uint32_t qc = have ? q : nch - 1;
  const bool mut_on = a.mutation == MUT_SWAP || a.mutation == MUT_INVERSION;
  const bool xo_kind = a.crossover == XO_PMX || a.crossover == XO_OX;
  const bool pmx = a.crossover == XO_PMX;
  const uint32_t S32 = (uint32_t)a.S;
  // the lane's genes (bit e: position 8 q + e), loop-invariant: padding
  // positions (all 8 for a lane without a chunk), the gene at position L - 1
  // (its successor is the tour's first city), genes whose edge counts
  // (FULL: no padding, and the last lane's successor lane is the group's
  // first, so the closing edge needs no select)
  const uint32_t base = 8u * q;
  const uint32_t padm8 = FULL ? 0u : (have ? range8(base, L, lp) : 0xFFu);
  const uint32_t wrapm8 = FULL ? 0u : (have ? range8(base, L - 1, L) : 0u);
  const uint32_t edgem8 = FULL ? (OBJ == OBJ_TSP_OPEN && q == GS - 1 ? 0x7Fu : 0xFFu)
                               : (have ? range8(base, 0, OBJ == OBJ_TSP_OPEN ? L - 1 : L) : 0u);
  // the LDS slot a padding gene writes instead of a city's (its own padding
  // position; a lane without a chunk: the group's spare words after C)
  const uint32_t dslot = have ? base : lp;

  if (a.n_elite > 0 && a.elite_idx == nullptr && blockIdx.x == 0) {
    unsigned long long b = block_reduce_parts_n(a.best_cur, a.n_best_cur, lds_red, NWv);
    if (threadIdx.x == 0) *lds_elite = (uint32_t)best_index(b);
  }
  if (OBJ == OBJ_TSP_EUC)
    for (uint32_t i = threadIdx.x; i < 2 * L; i += BLK) coords[i] = a.obj_data[i];
  if (TBL)
    for (uint32_t i = threadIdx.x; i < a.obj_aux_bytes / 16; i += BLK)
      ((uint4*)tab)[i] = ((const uint4*)a.obj_aux)[i];
  __syncthreads();

  unsigned long long my_best = 0;
  ScoreStats st;
  // batches of U children (the launcher's GenArgs::tp_unit: 64, or fewer for
  // small populations so that every wave gets one)
  const uint32_t U = a.tp_unit >= NG && a.tp_unit <= 64u && (a.tp_unit & (a.tp_unit - 1u)) == 0u ? a.tp_unit : 64u;
  const uint32_t TW = gridDim.x * NWv, Wg = blockIdx.x * NWv + (threadIdx.x >> 6);
  for (uint32_t bb = Wg * U; bb < S32; bb += TW * U) {  // wave-uniform batches (the launcher: S < 2^32)
    // ---- SELECT: lane j draws for child bb + j (its ST_CHILD words, core.hpp
    // child_word: block 0 = crossover test and cut words, block 1 = mutation
    // test and first position word, blocks 1-2 = the tournament words) and
    // picks its parents; the breed steps fetch the results by lane ----
    uint32_t PA, PB, PM, PX;  // parents; lo | hi << 10 | xo << 20 | mutate << 21 | elite << 22; i | j << 16
    {
      const uint32_t cj = lane < U && bb + lane < S32 ? bb + lane : bb;
      const u32x4 b0 = draw(a.key, ST_CHILD, cj, 0);
      const LanePool<GS> lpool{draw(a.key, ST_CHILD, cj, 1), draw(a.key, ST_CHILD, cj, 2)};
      select_parents<GS, LanePool<GS>>(a, lpool, cj, PA, PB);
#if PGA_PERM_NOSEL  // experiment builds: parents without tournaments
      PA = cj;
      PB = (cj ^ 1u) < S32 ? (cj ^ 1u) : cj;
#endif
      const bool elite = cj < a.n_elite;
      if (elite) {
        PA = a.elite_idx ? a.elite_idx[cj] : *lds_elite;
        PB = PA;
      }
      const bool xo = !PGA_PERM_NOXO && !elite && xo_kind && do_crossover(a, b0.x);  // W_XOPROB
      uint32_t lo, hi;
      perm_segment(b0.y, b0.z, L, lo, hi);  // W_CUT1, W_CUT2
      const bool mut = !elite && mut_on && lpool.b1.x < a.mut_ind_thresh;  // W_MUTIND
      uint32_t mi = 0, mj = 0;
      if (mut) perm_mut_positions(lpool.b1.y, child_word(a.key, cj, W_SEL + sel_words(a)), L, mi, mj);  // W_MUTPOS
      PM = lo | (hi << 10) | (xo ? 1u << 20 : 0u) | (mut ? 1u << 21 : 0u) | (elite ? 1u << 22 : 0u);
      PX = mi | (mj << 16);
    }
    const uint32_t nst = ((S32 - bb < U ? S32 - bb : U) + NG - 1) / NG;
    uint4 nA, nB;  // the next step's parent chunks
    if (PGA_PERM_PF) {
      const uint32_t pa = (uint32_t)__shfl((int)PA, (int)g, 64), pb = (uint32_t)__shfl((int)PB, (int)g, 64);
      nA = cur[(uint64_t)pa * rs + qc];
      nB = cur[(uint64_t)pb * rs + qc];
    }
    for (uint32_t t = 0; t < nst; ++t) {  // wave-uniform
      // ---- BREED step t: child bb + NG t + g ----
      const uint32_t child = bb + NG * t + g;
      const bool valid = child < S32;  // group-uniform
      const uint32_t jl = NG * t + g;   // the child's SELECT lane
      const uint32_t pa = (uint32_t)__shfl((int)PA, (int)jl, 64);
      if (!PGA_PERM_PF) {
        const uint32_t pb = (uint32_t)__shfl((int)PB, (int)jl, 64);
        nA = cur[(uint64_t)pa * rs + qc];
        nB = cur[(uint64_t)pb * rs + qc];
      }
      const uint4 Av = nA, Bv = nB;
      if (PGA_PERM_PF && t + 1 < nst) {  // wave-uniform: issue step t + 1's rows now
        const uint32_t j = jl + NG;
        const uint32_t na = (uint32_t)__shfl((int)PA, (int)j, 64), nb = (uint32_t)__shfl((int)PB, (int)j, 64);
        nA = cur[(uint64_t)na * rs + qc];
        nB = cur[(uint64_t)nb * rs + qc];
      }
      const uint32_t pm = (uint32_t)__shfl((int)PM, (int)jl, 64);
      const bool elite = (pm >> 22) & 1u, xo = (pm >> 20) & 1u;
      const uint32_t lo = pm & 1023u, hi = (pm >> 10) & 1023u;
      uint4 Cv = Av;
      float score = 0.f;
      if (elite) score = a.score_cur[pa];

      if (xo) {  // group-uniform
        // Branch-free per gene: every LDS access of the 8 genes is issued
        // unconditionally (a gene with nothing to write writes a slot the
        // result never reads), and the child is assembled with bit selects.
        // seg8: the lane's genes inside A's segment; from A: segment and padding
        const uint32_t seg8 = range8(base, lo, hi);
        const uint4 fromA = mask16x8(seg8 | padm8);
        if (pmx) {
          // T[city] = B's gene at the city's position in A's segment, kNone
          // elsewhere: A holds every city once, so T needs no clearing
          uint16_t* T = Cc;
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t ta = ((padm8 >> e) & 1u) ? dslot + e : min(get16(Av, e), lp - 1);
            T[ta] = (uint16_t)(((seg8 >> e) & 1u) ? get16(Bv, e) : (uint32_t)kNone);
          }
          wave_sync();
          // a gene of B outside the segment follows T until it leaves A's
          // segment (at most L links); the first link of all 8 in one batch
          uint32_t y0[8], v[8];
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) y0[e] = T[min(get16(Bv, e), lp - 1)];
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            v[e] = get16(Bv, e);
            if (!(((seg8 | padm8) >> e) & 1u)) {
              uint32_t y = y0[e];
              for (uint32_t guard = 0; y != kNone && guard < L;) {
                v[e] = y;
                if (++guard >= L) break;
                y = T[min(v[e], lp - 1)];
              }
            }
          }
          Cv = bfi4(fromA, Av, pack16x8(v));
        } else {  // OX1 (the ranks of perm_kernel): Cc first holds A's inverse, then the child
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t ia = ((padm8 >> e) & 1u) ? dslot + e : min(get16(Av, e), lp - 1);
            Cc[ia] = (uint16_t)(base + e);  // city -> its position in A
          }
          wave_sync();
          uint32_t pa8[8];
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) pa8[e] = Cc[min(get16(Bv, e), lp - 1)];
          // keep: B's genes outside A's segment, in B order
          uint32_t keep = 0;
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e)
            keep |= (!((padm8 >> e) & 1u) && pa8[e] - lo >= hi - lo) ? (1u << e) : 0u;
          const uint32_t below = range8(base, 0, hi);  // B positions before the segment end
          // one scan of both counts (16 bits each: at most L <= 65535 genes): the
          // group's kept genes before this lane (low half) and, in total, the
          // kept genes before the segment end (high half)
          uint32_t both;
          const uint32_t ex2 = group_excl_scan_dpp<GS>(__popc(keep) | (__popc(keep & below) << 16), q, both);
          const uint32_t Eb = both >> 16;
          const uint32_t K = L - (hi - lo);
          uint32_t run = ex2 & 0xFFFFu;
          wave_sync();  // every read of A's inverse is done before the child overwrites it
          // kept gene of rank r (B order from position 0) -> child position
          // hi + ((r - Eb) mod K), wrapped at L; a gene not kept writes the
          // slot lo + (its rank among those), inside the segment, which the
          // result takes from A (padding: its own padding slot)
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t p = base + e;
            uint32_t x = run + hi - Eb + (((below >> e) & 1u) ? K : 0u);
            x = min(x, x - L);  // x mod L (x < 2 L): the unsigned wrap of x - L loses the min below L
            const uint32_t d = ((padm8 >> e) & 1u) ? dslot + e : lo + (p - run);
            const bool k = (keep >> e) & 1u;
            Cc[k ? x : d] = (uint16_t)get16(Bv, e);
            run += k ? 1u : 0u;
          }
          wave_sync();
          Cv = bfi4(fromA, Av, *(const uint4*)(Cc + 8 * qc));
        }
      }

      // (the shuffle before the branch: the SELECT lane may be outside it)
      const uint32_t px = (uint32_t)__shfl((int)PX, (int)jl, 64);
      if ((pm >> 21) & 1u) {  // group-uniform: mutation
        const uint32_t i = px & 0xFFFFu, j = px >> 16;
        wave_sync();  // earlier readers of C / T are done
        if (have) *(uint4*)(Cc + 8 * q) = Cv;
        wave_sync();
        if (a.mutation == MUT_SWAP) {
          if (q == 0) {
            const uint16_t t2 = Cc[i];
            Cc[i] = Cc[j];
            Cc[j] = t2;
          }
        } else {
          const uint32_t half = (j - i + 1) / 2;
          for (uint32_t t2 = q; t2 < half; t2 += GS) {
            const uint16_t x = Cc[i + t2];
            Cc[i + t2] = Cc[j - t2];
            Cc[j - t2] = x;
          }
        }
        wave_sync();
        Cv = *(const uint4*)(Cc + 8 * qc);
      }
      wave_sync();  // the next child of this group rewrites C / T

      if (valid && have) nxt[(uint64_t)child * rs + q] = Cv;
      if (!elite && !PGA_PERM_NOEVAL) {
        // edge of gene e: to gene e + 1, the next lane's first city (e = 7),
        // or the tour's first city (position L - 1); every lookup of the 8
        // issued before the sum, which keeps perm_kernel's order (e = 0..7
        // from 0.f, then the butterfly)
        const uint32_t c0 = Cv.x & 0xFFFFu;
        const uint32_t next_first = (uint32_t)__shfl((int)c0, (int)(gbase + ((q + 1) & (GS - 1))), 64);
        const uint32_t first = (uint32_t)__shfl((int)c0, (int)gbase, 64);
        uint32_t u[8], w[8];
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
          const uint32_t nx = ((wrapm8 >> e) & 1u) ? first : (e < 7 ? get16(Cv, e + 1) : next_first);
          u[e] = min(get16(Cv, e), L - 1);
          w[e] = min(nx, L - 1);
        }
        float dv[8];
        if (OBJ == OBJ_TSP_EUC) {
          const float2* xy = (const float2*)coords;
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            const float2 pu = xy[u[e]], pw = xy[w[e]];
            const float dx = pu.x - pw.x, dy = pu.y - pw.y;
            dv[e] = sqrtf(fmaf(dx, dx, dy * dy));
          }
        } else if constexpr (FULL && GS <= 32 && (TBL == 1 || TBL == 3)) {
          // L <= 256: hi (hi + 1) <= 65280 fits 16 bits, so each pair of
          // edges takes one packed clamp / max / min / multiply-add / shift /
          // add; (hi, lo) of edge e is (max, min) of gene e and its successor
          using us2 = unsigned short __attribute__((ext_vector_type(2)));
          const us2 lm = {(unsigned short)(L - 1), (unsigned short)(L - 1)};
          const uint32_t wv[4] = {Cv.x, Cv.y, Cv.z, Cv.w};
          uint32_t gw[4];
#pragma unroll
          for (uint32_t i = 0; i < 4; ++i)
            gw[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(us2, wv[i]), lm));
          const uint32_t nf = min(next_first, L - 1);
#pragma unroll
          for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t sw = i < 3 ? __builtin_amdgcn_alignbit(gw[i + 1], gw[i], 16) : ((gw[3] >> 16) | (nf << 16));
            const us2 a2 = __builtin_bit_cast(us2, gw[i]), b2 = __builtin_bit_cast(us2, sw);
            const us2 h2 = __builtin_elementwise_max(a2, b2), l2 = __builtin_elementwise_min(a2, b2);
            const uint32_t ix = __builtin_bit_cast(uint32_t, ((us2)(h2 * h2 + h2) >> (us2){1, 1}) + l2);
            dv[2 * i] = TBL == 1 ? (float)tab[ix & 0xFFFFu] : ftab[ix & 0xFFFFu];
            dv[2 * i + 1] = TBL == 1 ? (float)tab[ix >> 16] : ftab[ix >> 16];
          }
        } else {
#pragma unroll
          for (uint32_t e = 0; e < 8; ++e) {
            if constexpr (TBL == 1 || TBL == 3) {
              // rows of the lower triangle with the diagonal: (hi, lo) at hi (hi + 1) / 2 + lo
              const uint32_t hi_ = max(u[e], w[e]), lo_ = min(u[e], w[e]);
              const uint32_t ix = (__umul24(hi_, hi_ + 1u) >> 1) + lo_;
              dv[e] = TBL == 1 ? (float)tab[ix] : ftab[ix];
            } else if constexpr (TBL == 2) {
              dv[e] = (float)tab[__umul24(u[e], L) + w[e]];
            } else {
              dv[e] = a.obj_data[u[e] * L + w[e]];
            }
          }
        }
        float len = 0.f;
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e)
          if ((edgem8 >> e) & 1u) len += dv[e];
        score = -group_sum<GS>(len);
      }
      if (valid && q == 0) {
        a.score_next[child] = score;
        const unsigned long long pb2 = pack_best(score, child);
        my_best = pb2 > my_best ? pb2 : my_best;
        st.add(score);
      }
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
template <int GS, int OBJ, int TBL = 0, bool FULL = false>
__global__ __launch_bounds__(TBL ? 1024 : kBlock) void perm_gen_fast(GenArgs a, unsigned long long* best_parts) {
  perm_gen_fast_body<GS, OBJ, TBL, FULL>(a, best_parts);
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
template <int GS, int OBJ, int TBL = 0>
__global__ __launch_bounds__(kBlock) void perm_gen_fast_batch(PermBatch b) {
  perm_gen_fast_body<GS, OBJ, TBL>(b.a[blockIdx.y], b.parts[blockIdx.y]);
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

// children per wave batch (GenArgs::tp_unit of the fast kernel): 64, halved
// (down to one step) while the batches would leave waves of the grid idle
template <int GS>
uint32_t fast_unit(uint64_t S, uint64_t waves) {
  uint32_t u = 64;
  while (u > 64u / GS && (S + u - 1) / u < waves) u >>= 1;
  return u;
}

// the LDS matrix for PMX too (PGA_PERM_PMX_TBL=0: PMX keeps the L2 matrix
// path and its 256-thread blocks, for A/B runs)
inline bool perm_tbl_on(const GenArgs& a) {
  static const bool pmx_tbl = [] {
    const char* e = std::getenv("PGA_PERM_PMX_TBL");
    return !(e && e[0] == '0');
  }();
  return a.crossover != XO_PMX || pmx_tbl;
}

template <int GS, int OBJ, int TBL, bool FULL>
uint32_t go_fast_blk(const GenArgs& a0, unsigned long long* parts, hipStream_t s, uint32_t blk) {
  const size_t lds = perm_fast_lds_bytes(GS, a0.chunks, OBJ == OBJ_TSP_EUC, blk) + (TBL ? a0.obj_aux_bytes : 0);
  auto k = perm_gen_fast<GS, OBJ, TBL, FULL>;
  const size_t avail = allow_dynamic_lds((const void*)k);
  if constexpr (TBL != 0) {  // the table did not fit this device's limit: the L2 matrix path
    if (lds > avail) return go_fast_blk<GS, OBJ, 0, FULL>(a0, parts, s, kBlock);
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, (int)blk, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  uint64_t cap = (uint64_t)device_cu_count() * per_cu;
  if (cap > kMaxGrid) cap = kMaxGrid;
  GenArgs a = a0;
  const uint32_t nw = blk / 64;
  a.tp_unit = fast_unit<GS>(a.S, cap * nw);
  const uint64_t need = ((a.S + a.tp_unit - 1) / a.tp_unit + nw - 1) / nw;
  const uint32_t grid = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL(k, grid, blk, lds, s, a, parts);
  return grid;
}

template <int GS, int OBJ, bool FULL>
uint32_t go_fast_tbl(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  if constexpr (OBJ == OBJ_TSP || OBJ == OBJ_TSP_OPEN) {
    // the matrix in LDS (obj_aux): the largest block (up to 16 waves, one
    // table per CU) whose group arrays fit beside it
    if (a.obj_aux && a.obj_aux_kind >= 1 && a.obj_aux_kind <= 3 && a.obj_aux_bytes % 16 == 0 && perm_tbl_on(a)) {
      const size_t avail = 160 * 1024 - 1024;  // less the static LDS (block reductions)
      // populations that fill every wave of 16-wave blocks with 64-child
      // batches take the largest block that fits (one table per CU); smaller
      // ones the smallest, so that their few batches spread over every CU
      const bool big = a.S >= 1024ull * device_cu_count();
      const uint32_t order[3] = {big ? 1024u : 256u, 512u, big ? 256u : 1024u};
      for (uint32_t blk : order) {
        if (perm_fast_lds_bytes(GS, a.chunks, false, blk) + a.obj_aux_bytes > avail) continue;
        if (a.obj_aux_kind == 1) return go_fast_blk<GS, OBJ, 1, FULL>(a, parts, s, blk);
        if (a.obj_aux_kind == 2) return go_fast_blk<GS, OBJ, 2, FULL>(a, parts, s, blk);
        return go_fast_blk<GS, OBJ, 3, FULL>(a, parts, s, blk);
      }
    }
  }
  return go_fast_blk<GS, OBJ, 0, FULL>(a, parts, s, kBlock);
}

template <int GS, int OBJ>
uint32_t go_fast(const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  // whole chunks on every lane (L = 8 GS: TSP-64 / 128 / 256 / 512): the FULL variants
  if constexpr (GS >= 8) {
    static const bool off = std::getenv("PGA_PERM_NO_FULL") != nullptr;  // A/B runs: the general variants
    if (a.L == 8u * GS && a.chunks == (uint32_t)GS && !off)
      return go_fast_tbl<GS, OBJ, true>(a, parts, s);
  }
  return go_fast_tbl<GS, OBJ, false>(a, parts, s);
}

template <int GS, int OBJ>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (mode) {
    case MODE_GEN:
      // the fast kernel walks its batches with 32-bit child indices: the
      // batch base (at most S + grid * 16 waves * 64 past 0) must not wrap
      if (OBJ != OBJ_NONE && a.chunks <= (uint32_t)GS && !force_generic_kernels() &&
          a.S <= 0xFFFFFFFFull - (uint64_t)kMaxGrid * 16 * 64)
        return go_fast<GS, OBJ>(a, parts, s);
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

template <int GS, int OBJ, int TBL = 0>
uint32_t batch_go(PermBatch& b, uint32_t n, hipStream_t s) {
  const GenArgs& a0 = b.a[0];
  // TBL: every island's matrix in its blocks' LDS (the islands' tables have one kind and size)
  const size_t lds = perm_fast_lds_bytes(GS, a0.chunks, OBJ == OBJ_TSP_EUC, kBlock) + (TBL ? a0.obj_aux_bytes : 0);
  const void* k = (const void*)perm_gen_fast_batch<GS, OBJ, TBL>;
  (void)allow_dynamic_lds(k);  // cached per (kernel, device)
  uint64_t cap = (uint64_t)device_cu_count() * occupancy_blocks(k, kBlock, lds) / n;  // the device split
  if (cap < 1) cap = 1;
  if (cap > kMaxGrid) cap = kMaxGrid;
  const uint32_t nw = kBlock / 64, u = fast_unit<GS>(a0.S, cap * nw);
  for (uint32_t i = 0; i < n; ++i) b.a[i].tp_unit = u;
  const uint64_t need = ((a0.S + u - 1) / u + nw - 1) / nw;
  const uint32_t gx = (uint32_t)(need < cap ? need : cap);
  hipLaunchKernelGGL((perm_gen_fast_batch<GS, OBJ, TBL>), dim3(gx, n), kBlock, lds, s, b);
  PGA_HIP_CHECK(hipGetLastError());
  return gx;
}

template <int GS, int OBJ>
uint32_t batch_tbl(PermBatch& b, uint32_t n, hipStream_t s) {
  if constexpr (OBJ == OBJ_TSP || OBJ == OBJ_TSP_OPEN) {
    const GenArgs& a0 = b.a[0];
    bool same = a0.obj_aux && a0.obj_aux_kind >= 1 && a0.obj_aux_kind <= 3 && a0.obj_aux_bytes % 16 == 0 &&
                perm_tbl_on(a0) &&
                perm_fast_lds_bytes(GS, a0.chunks, false, kBlock) + a0.obj_aux_bytes <= 160 * 1024 - 1024;
    for (uint32_t i = 1; same && i < n; ++i)
      same = b.a[i].obj_aux && b.a[i].obj_aux_kind == a0.obj_aux_kind && b.a[i].obj_aux_bytes == a0.obj_aux_bytes;
    if (same) {
      if (a0.obj_aux_kind == 1) return batch_go<GS, OBJ, 1>(b, n, s);
      if (a0.obj_aux_kind == 2) return batch_go<GS, OBJ, 2>(b, n, s);
      return batch_go<GS, OBJ, 3>(b, n, s);
    }
  }
  return batch_go<GS, OBJ, 0>(b, n, s);
}

template <int GS>
uint32_t batch_obj(PermBatch& b, uint32_t n, hipStream_t s) {
  switch (b.a[0].objective) {
    case OBJ_TSP: return batch_tbl<GS, OBJ_TSP>(b, n, s);
    case OBJ_TSP_OPEN: return batch_tbl<GS, OBJ_TSP_OPEN>(b, n, s);
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
  if (a0.S > 0xFFFFFFFFull - (uint64_t)kMaxGrid * 16 * 64) return 0;  // its 32-bit batch walk (launch_mode)
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
