// cpu_perm.cpp — CPU reference backend for the PERMUTATION encoding; mirrors
// csrc/kernels/perm.hip.  PMX / OX1 / swap / inversion are deterministic
// functions of the parents and the child's words, and the tour-length sum
// follows the kernel's lane partition + butterfly, so children and scores
// are bit-identical to the GPU.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "pga/cpu.hpp"
#include "pga/perm_ops.hpp"

namespace pga {
namespace cpu {

// PMX / OX1 child of parents A and B with A's segment [lo, hi) (the kernels'
// LDS versions compute the same child; tests/test_perm.py pins both against
// the textbook examples)
void perm_crossover(int op, const uint16_t* A, const uint16_t* B, uint32_t L, uint32_t lo, uint32_t hi, uint16_t* C) {
  std::vector<int32_t> M(L, -1);  // city -> its position in A's segment
  for (uint32_t k = lo; k < hi; ++k) M[A[k]] = (int32_t)k;
  std::fill(C, C + L, 0);
  if (op == XO_PMX) {
    for (uint32_t p = 0; p < L; ++p) {
      if (p >= lo && p < hi) {
        C[p] = A[p];
      } else {
        uint32_t v = B[p];
        for (uint32_t guard = 0; M[v] >= 0 && guard < L; ++guard) v = B[M[v]];
        C[p] = (uint16_t)v;
      }
    }
  } else {  // OX1: fill from the segment end, B in order from the segment end
    for (uint32_t k = lo; k < hi; ++k) C[k] = A[k];
    uint32_t pos = hi % L;
    for (uint32_t t = 0; t < L; ++t) {
      const uint32_t p = (hi + t) % L;
      if (M[B[p]] >= 0) continue;
      C[pos] = B[p];  // free positions: hi .. L-1, then 0 .. lo-1 (exactly L - (hi - lo) of them)
      pos = (pos + 1) % L;
    }
  }
}

// every city 0..L-1 exactly once (seen: L scratch entries)
static bool perm_row_valid(const uint16_t* C, uint32_t L, std::vector<uint16_t>& seen) {
  std::fill(seen.begin(), seen.begin() + L, (uint16_t)0);
  for (uint32_t p = 0; p < L; ++p) {
    if (C[p] >= L || seen[C[p]]) return false;
    seen[C[p]] = 1;
  }
  return true;
}

uint32_t perm_run(int mode, const GenArgs& a, unsigned long long* best_parts) {
  if (a.L > 65535) throw std::invalid_argument("PERMUTATION encoding supports at most 65535 genes (u16 city ids)");
  const uint32_t L = a.L, nch = a.chunks, lp = 8 * nch, GS = group_size(nch);
  const uint64_t rw = a.row_words;
  const uint16_t* cur = (const uint16_t*)a.cur;
  uint16_t* nxt = (uint16_t*)a.next;
  const uint64_t rh = 2 * rw;  // u16 per row
  const bool gen = mode == MODE_GEN, crosses = gen || mode == MODE_CROSS, mutates = gen || mode == MODE_MUTATE;
  const bool evals = a.objective != OBJ_NONE && (gen || mode == MODE_INIT || mode == MODE_EVAL);
  const bool mut_on = mutates && (a.mutation == MUT_SWAP || a.mutation == MUT_INVERSION);
  uint32_t elite0 = 0;
  if (gen && a.n_elite > 0 && a.elite_idx == nullptr) elite0 = (uint32_t)best_index(reduce_best(a.best_cur, a.n_best_cur));

  std::vector<unsigned long long> bests(cpu_threads(), 0ull);
  parallel_for(a.S, 64, [&](uint64_t c_begin, uint64_t c_end, unsigned slot) {
  unsigned long long best = 0;
  std::vector<uint16_t> A(lp), B(lp), C(lp);
  for (uint64_t child = c_begin; child < c_end; ++child) {
    bool elite = false;
    float score = 0.f;
    std::fill(C.begin(), C.end(), 0);
    if (gen && child < a.n_elite) {
      elite = true;
      const uint32_t src = a.elite_idx ? a.elite_idx[child] : elite0;
      std::memcpy(C.data(), cur + (uint64_t)src * rh, 2ull * lp);
      score = a.score_cur[src];
    } else if (mode == MODE_INIT) {
      for (uint32_t i = 0; i < L; ++i) C[i] = (uint16_t)i;
      for (uint32_t i = L - 1; i >= 1; --i) {
        const uint32_t j = word_to_index(perm_init_word(a.key, child, i), i + 1);
        std::swap(C[i], C[j]);
      }
    } else if (mode == MODE_EVAL || mode == MODE_MUTATE) {
      std::memcpy(C.data(), cur + child * rh, 2ull * lp);
    }
    if (mode == MODE_EVAL && !perm_row_valid(C.data(), L, A)) {
      // not a permutation of 0..L-1 (a corrupted or forged migrant): the
      // identity tour replaces it, scored below like any other row
      for (uint32_t p = 0; p < lp; ++p) C[p] = p < L ? (uint16_t)p : (uint16_t)0;
      std::memcpy(nxt + child * rh, C.data(), 2ull * lp);
    }
    if (!elite && crosses) {
      uint32_t pa, pb;
      select_parents(a, child, pa, pb);
      const bool xo = (a.crossover == XO_PMX || a.crossover == XO_OX) && do_crossover(a, pool_word(a.key, child, W_XOPROB));
      uint32_t lo, hi;
      perm_segment(pool_word(a.key, child, W_CUT1), pool_word(a.key, child, W_CUT2), L, lo, hi);
      std::memcpy(A.data(), cur + (uint64_t)pa * rh, 2ull * lp);
      if (!xo) {
        C = A;
      } else {
        std::memcpy(B.data(), cur + (uint64_t)pb * rh, 2ull * lp);
        perm_crossover(a.crossover, A.data(), B.data(), L, lo, hi, C.data());
      }
    }
    if (!elite && mut_on && pool_word(a.key, child, W_MUTIND) < a.mut_ind_thresh) {
      uint32_t i, j;
      perm_mut_positions(pool_word(a.key, child, W_MUTPOS), pool_word(a.key, child, W_SEL + sel_words(a)), L, i, j);
      if (a.mutation == MUT_SWAP) std::swap(C[i], C[j]);
      else std::reverse(C.begin() + i, C.begin() + j + 1);
    }
    if (mode != MODE_EVAL) std::memcpy(nxt + child * rh, C.data(), 2ull * lp);
    if (evals && !elite) {
      float lane[64] = {0};
      const uint32_t last = a.objective == OBJ_TSP_OPEN ? L - 1 : L;
      for (uint32_t p = 0; p < last; ++p) {
        const uint32_t u = std::min<uint32_t>(C[p], L - 1), w = std::min<uint32_t>(C[(p + 1) % L], L - 1);
        float d;
        if (a.objective == OBJ_TSP_EUC) {
          const float dx = a.obj_data[2 * u] - a.obj_data[2 * w], dy = a.obj_data[2 * u + 1] - a.obj_data[2 * w + 1];
          d = std::sqrt(std::fma(dx, dx, dy * dy));  // explicit: same rounding as the kernels
        } else {
          d = a.obj_data[u * L + w];
        }
        lane[(p / 8) % GS] += d;
      }
      score = -butterfly_sum(lane, GS);
    }
    if (evals) {
      a.score_next[child] = score;
      best = std::max(best, pack_best(score, child));
    }
  }
  bests[slot] = best;
  });
  const unsigned long long best = *std::max_element(bests.begin(), bests.end());
  if (evals && best_parts) best_parts[0] = best;
  return 1;
}

}  // namespace cpu
}  // namespace pga
