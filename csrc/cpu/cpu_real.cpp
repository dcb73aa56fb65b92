// cpu_real.cpp — CPU reference backend for the REAL encoding; mirrors
// csrc/kernels/real.hip (same randomness layout and per-gene semantics from
// real_ops.hpp, same GS-lane butterfly reductions, rotation as a k-ordered fma
// chain = the MFMA result).  Rows are bit-identical to the GPU for every
// operator (gaussian included: real_ops.hpp gauss_z); scores of the
// polynomial objectives too, those of the transcendental ones to a few ulps.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "pga/cpu.hpp"
#include "pga/real_ops.hpp"

namespace pga {
namespace cpu {

static float butterfly_prod(float* v, uint32_t GS) {
  float t[64];
  for (uint32_t o = GS / 2; o > 0; o >>= 1) {
    for (uint32_t q = 0; q < GS; ++q) t[q] = v[q] * v[q ^ o];
    for (uint32_t q = 0; q < GS; ++q) v[q] = t[q];
  }
  return v[0];
}

uint32_t real_run(int mode, const GenArgs& a, unsigned long long* best_parts) {
  const uint32_t GS = group_size(a.chunks);  // 64 lanes own chunks c, c+64, ... of long genomes
  const uint64_t rw = a.row_words;
  const float* cur = (const float*)a.cur;
  float* nxt = (float*)a.next;
  const uint32_t L = a.L, nchunks = a.chunks;
  const bool gen = mode == MODE_GEN, cross = mode == MODE_CROSS, mutm = mode == MODE_MUTATE;
  const bool evals = a.objective != OBJ_NONE && (gen || mode == MODE_INIT || mode == MODE_EVAL);
  const bool per_gene = (gen || mutm) && real_per_gene_mutation(a);
  const bool sparse = per_gene && a.mut_sparse;
  const bool reset_one = (gen || mutm) && a.mutation == MUT_RESET_ONE;
  const bool rot = (a.obj_i & 2) && a.obj_data && real_obj_rotatable(a.objective);
  const bool shift = (a.obj_i & 1) && a.obj_data2 && real_obj_rotatable(a.objective);
  if (rot && L > 128) throw std::invalid_argument("rotated objectives support at most 128 dimensions");
  const uint32_t dp = ((4 * nchunks + 15) / 16) * 16;
  if (evals && a.objective == OBJ_USER_FNPTR)
    throw std::invalid_argument("device function-pointer objectives need the GPU backend");
  if (nchunks > 64 && evals && a.objective == OBJ_TSP_RANDOM_KEY)
    throw std::invalid_argument("the random-key TSP and function-pointer objectives support at most 256 genes");

  uint32_t elite0 = 0;
  if (gen && a.n_elite > 0 && a.elite_idx == nullptr) elite0 = (uint32_t)best_index(reduce_best(a.best_cur, a.n_best_cur));

  const uint32_t nv = 4 * std::max<uint32_t>(GS, nchunks);
  std::vector<unsigned long long> bests(cpu_threads(), 0ull);
  parallel_for(a.S, 64, [&](uint64_t c_begin, uint64_t c_end, unsigned slot) {
  unsigned long long best = 0;
  std::vector<float> v(nv), x(std::max<uint32_t>(nv, dp) + 4), z(std::max<uint32_t>(nv, dp) + 4);
  std::vector<uint32_t> pos;
  for (uint64_t child = c_begin; child < c_end; ++child) {
    std::fill(v.begin(), v.end(), 0.f);
    // elitism: child = copy of the elite row (no variation), re-evaluated like every child
    const bool elite = gen && child < a.n_elite;
    const u32x4 misc = real_misc(a.key, child);
    if (elite) {
      const uint32_t src = a.elite_idx ? a.elite_idx[child] : elite0;
      std::memcpy(v.data(), cur + (uint64_t)src * rw, 16ull * nchunks);
    } else if (mode == MODE_INIT) {
      for (uint32_t q = 0; q < nchunks; ++q) real_init_chunk(a, child, q, &v[4 * q]);
    } else if (mode == MODE_EVAL || mutm) {
      std::memcpy(v.data(), cur + child * rw, 16ull * nchunks);
    }
    if (!elite && (gen || cross)) {
      uint32_t pa, pb;
      bin_select_parents(a, child, pa, pb);
      const bool xo = a.crossover != XO_NONE && do_crossover(a, misc.x);
      const uint32_t cut = real_cut_word(a, misc);
      for (uint32_t q = 0; q < nchunks; ++q) {
        const uint32_t ub = (xo && a.crossover == XO_UNIFORM) ? real_uniform_bits(a.key, child, q) : 0u;
        real_cross_chunk(a, child, q, cur + (uint64_t)pa * rw + 4 * q, cur + (uint64_t)pb * rw + 4 * q, xo, cut, ub,
                         &v[4 * q]);
      }
    }
    if (!elite && (sparse || reset_one)) {
      // the first K distinct positions of the mutation words, the n-th takes value draw n
      const uint32_t K = sparse ? binom_count(misc.w, a.mut_thr) : (misc.w < a.mut_ind_thresh ? 1u : 0u);
      pos.clear();
      for (uint32_t j = 0; pos.size() < K; ++j) {
        const uint32_t p = word_to_index(bin_mut_word(a.key, child, j), L);
        if (std::find(pos.begin(), pos.end(), p) != pos.end()) continue;
        v[p] = real_mut_apply(a, real_mut_draw(a, child, (uint32_t)pos.size()), v[p]);
        pos.push_back(p);
      }
    } else if (!elite && per_gene) {
      for (uint32_t q = 0; q < nchunks; ++q) {
        const uint32_t clen = std::min(4u, L - 4 * q);
        real_mutate_chunk(a, child, q, clen, bin_chunk_mut_word(a.key, child, q), a.mut_thr, &v[4 * q]);
      }
    }
    for (uint32_t d = L; d < 4 * nchunks; ++d) v[d] = 0.f;
    if (mode != MODE_EVAL) std::memcpy(nxt + child * rw, v.data(), 16ull * nchunks);

    float score = 0.f;
    if (evals) {
      std::fill(x.begin(), x.end(), 0.f);
      for (uint32_t d = 0; d < L; ++d) x[d] = shift ? v[d] - a.obj_data2[d] : v[d];
      if (rot) {
        std::fill(z.begin(), z.end(), 0.f);
        for (uint32_t n = 0; n < L; ++n) {
          float acc = 0.f;
          for (uint32_t k = 0; k < dp; ++k) acc = std::fmaf(x[k], k < L ? a.obj_data[n * L + k] : 0.f, acc);
          z[n] = acc;
        }
      } else {
        z = x;
      }
      if (a.objective == OBJ_TSP_RANDOM_KEY) {
        float lane[64] = {0};
        for (uint32_t i = 0; i < L; ++i) {
          const uint32_t ci = random_key_city(x[i], L);
          if (i > 0) lane[i / 4] += a.obj_data[random_key_city(x[i - 1], L) * L + ci];
          uint32_t dups = 0;
          for (uint32_t k = 0; k < L; ++k) dups += (k != i && random_key_city(x[k], L) == ci) ? 1u : 0u;
          lane[i / 4] += 10000.f * (float)dups;
        }
        score = -butterfly_sum(lane, GS);
      } else {
        float s0[64] = {0}, s1[64] = {0}, s2[64];
        for (uint32_t q = 0; q < GS; ++q) s2[q] = 1.f;
        for (uint32_t d = 0; d < L; ++d) {
          const uint32_t ln = (d / 4) % GS;  // the lane owning gene d's chunk
          RealAcc acc{s0[ln], s1[ln], s2[ln]};
          real_obj_term(a, d, z[d], z[d + 1], v[d], acc);
          s0[ln] = acc.s0;
          s1[ln] = acc.s1;
          s2[ln] = acc.s2;
        }
        RealAcc t{butterfly_sum(s0, GS), butterfly_sum(s1, GS), butterfly_prod(s2, GS)};
        score = real_obj_finish(a, t);
      }
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
