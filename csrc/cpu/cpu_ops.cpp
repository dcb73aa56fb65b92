// cpu_ops.cpp — CPU reference backend: BINARY encoding + population utilities.
// Mirrors csrc/kernels/binary.hip and csrc/kernels/util.hip operation by
// operation (see the comments there for the semantics).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "pga/cpu.hpp"

namespace pga {
namespace cpu {

// x^T Q x of S bit rows with the kernels' coefficient rule (qubo_coef) and
// integer accumulation: bit-identical to qubo.hip
uint32_t qubo_eval(const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const float* q, float sign,
                   float* scores, unsigned long long* best_parts) {
  std::vector<int32_t> Q((size_t)L * L);
  for (size_t i = 0; i < Q.size(); ++i) Q[i] = qubo_coef(q[i]);
  const uint32_t* r = (const uint32_t*)rows;
  std::vector<uint32_t> on;
  unsigned long long best = 0;
  for (uint64_t c = 0; c < S; ++c) {
    on.clear();
    for (uint32_t k = 0; k < L; ++k)
      if ((r[c * row_words + k / 32] >> (k % 32)) & 1u) on.push_back(k);
    int64_t f = 0;
    for (uint32_t k : on)
      for (uint32_t n : on) f += Q[(size_t)k * L + n];
    const float sc = sign * (float)(int32_t)f;
    scores[c] = sc;
    const unsigned long long pb = pack_best(sc, c);
    best = pb > best ? pb : best;
  }
  if (best_parts) best_parts[0] = best;
  return 1;
}

uint32_t encoding_run(int mode, const GenArgs& a, unsigned long long* best_parts) {
  switch (a.encoding) {
    case ENC_BINARY:
      if (a.objective == OBJ_QUBO && (mode == MODE_GEN || mode == MODE_INIT || mode == MODE_EVAL)) {
        GenArgs b = a;
        b.objective = OBJ_NONE;
        b.key_next = nullptr;
        if (mode != MODE_EVAL) binary_run(mode, b, best_parts);
        return qubo_eval(a.next, a.row_words, a.S, a.L, a.obj_data, a.obj_f0, a.score_next, best_parts);
      }
      return binary_run(mode, a, best_parts);
    case ENC_REAL: return real_run(mode, a, best_parts);
    default: return perm_run(mode, a, best_parts);
  }
}

static uint32_t roulette_pick(const float* cumfit, uint32_t S, uint32_t w) {
  float total = cumfit[S - 1];
  if (!(total > 0.f)) return word_to_index(w, S);
  float target = word_to_unit(w) * total;
  uint32_t lo = 0, hi = S - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (cumfit[mid] < target) lo = mid + 1; else hi = mid;
  }
  return lo;
}

void select_parents(const GenArgs& a, uint64_t child, uint32_t& pa, uint32_t& pb) {
  const uint32_t S = (uint32_t)a.S;
  if (a.selection == SEL_TOURNAMENT) {
    const uint32_t k = a.tour_k;
    uint32_t best[2];
    for (uint32_t p = 0; p < 2; ++p) {
      uint32_t b = word_to_index(pool_word(a.key, child, W_SEL + p * k), S);
      float bs = a.score_cur[b];
      for (uint32_t j = 1; j < k; ++j) {
        uint32_t c = word_to_index(pool_word(a.key, child, W_SEL + p * k + j), S);
        float cs = a.score_cur[c];
        if (bs < cs) { bs = cs; b = c; }
      }
      best[p] = b;
    }
    pa = best[0];
    pb = best[1];
  } else if (a.selection == SEL_ROULETTE) {
    pa = roulette_pick(a.cumfit, S, pool_word(a.key, child, W_SEL + 0));
    pb = roulette_pick(a.cumfit, S, pool_word(a.key, child, W_SEL + 1));
  } else if (a.selection == SEL_RANK) {
    auto w = [&](uint32_t t) { return pool_word(a.key, child, W_SEL + t); };
    pa = a.rank_order[rank_pick(w(0), w(1), w(2), S, a.rank_thresh)];
    pb = a.rank_order[rank_pick(w(3), w(4), w(5), S, a.rank_thresh)];
  } else {
    pa = word_to_index(pool_word(a.key, child, W_SEL + 0), S);
    pb = word_to_index(pool_word(a.key, child, W_SEL + 1), S);
  }
}

static inline uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }

// BINARY / REAL parent choice from the ST_SEL words (core.hpp "BINARY randomness layout")
void bin_select_parents(const GenArgs& a, uint64_t child, uint32_t& pa, uint32_t& pb) {
  const uint32_t S = (uint32_t)a.S;
  auto w = [&](uint32_t t) { return bin_sel_word(a.key, child, t); };
  if (a.selection == SEL_TOURNAMENT) {
    const uint32_t k = a.tour_k;
    uint32_t best[2];
    for (uint32_t p = 0; p < 2; ++p) {
      uint32_t b = word_to_index(w(p * k), S);
      float bs = a.score_cur[b];
      for (uint32_t j = 1; j < k; ++j) {
        uint32_t c = word_to_index(w(p * k + j), S);
        float cs = a.score_cur[c];
        if (bs < cs) { bs = cs; b = c; }
      }
      best[p] = b;
    }
    pa = best[0];
    pb = best[1];
  } else if (a.selection == SEL_ROULETTE) {
    pa = roulette_pick(a.cumfit, S, w(0));
    pb = roulette_pick(a.cumfit, S, w(1));
  } else if (a.selection == SEL_RANK) {
    pa = a.rank_order[rank_pick(w(0), w(1), w(2), S, a.rank_thresh)];
    pb = a.rank_order[rank_pick(w(3), w(4), w(5), S, a.rank_thresh)];
  } else {
    pa = word_to_index(w(0), S);
    pb = word_to_index(w(1), S);
  }
}

// sparse bit-flip: the first K distinct positions of the mutation words
static void sparse_positions(const GenArgs& a, uint64_t child, uint32_t K, std::vector<uint32_t>& out) {
  out.clear();
  for (uint32_t j = 0; out.size() < K; ++j) {
    const uint32_t p = word_to_index(bin_mut_word(a.key, child, j), a.L);
    if (std::find(out.begin(), out.end(), p) == out.end()) out.push_back(p);
  }
}

uint32_t binary_run(int mode, const GenArgs& a, unsigned long long* best_parts) {
  const uint32_t GS = group_size(a.chunks);
  const uint64_t rw = a.row_words;
  const uint32_t* cur = (const uint32_t*)a.cur;
  uint32_t* nxt = (uint32_t*)a.next;
  const uint32_t L = a.L, nchunks = a.chunks;
  const bool gen = mode == MODE_GEN, cross = mode == MODE_CROSS;
  const bool evaluates = a.objective != OBJ_NONE && (mode == MODE_GEN || mode == MODE_INIT || mode == MODE_EVAL);
  const bool bitflip = (gen || mode == MODE_MUTATE) && a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f;
  const bool reset_one = (gen || mode == MODE_MUTATE) && a.mutation == MUT_RESET_ONE;

  uint32_t elite0 = 0;
  if (gen && a.n_elite > 0 && a.elite_idx == nullptr) elite0 = (uint32_t)best_index(reduce_best(a.best_cur, a.n_best_cur));

  std::vector<unsigned long long> bests(cpu_threads(), 0ull);
  parallel_for(a.S, 64, [&](uint64_t c_begin, uint64_t c_end, unsigned slot) {
  unsigned long long best = 0;
  std::vector<uint32_t> seg((size_t)GS * 4), flips;
  for (uint64_t child = c_begin; child < c_end; ++child) {
    float score = 0.f;
    {
      // elitism: child = copy of the elite row, re-evaluated like every child
      const bool elite = gen && child < a.n_elite;
      uint32_t pa = 0, pb = 0;
      bool xo = false;
      uint32_t blo = 0, bhi = 0;
      const u32x4 misc = bin_misc(a.key, child);
      if (elite) {
        pa = pb = a.elite_idx ? a.elite_idx[child] : elite0;
      } else if (gen || cross) {
        bin_select_parents(a, child, pa, pb);
        xo = a.crossover != XO_NONE && do_crossover(a, misc.x);
        if (a.crossover == XO_ONE_POINT) {
          blo = word_to_index(misc.y, L);
          bhi = L;
        } else if (a.crossover == XO_TWO_POINT) {
          uint32_t c1 = word_to_index(misc.y, L);
          uint32_t c2 = word_to_index(misc.z, L);
          blo = std::min(c1, c2);
          bhi = std::max(c1, c2);
        }
      }
      // flipped positions: RESET_ONE (at most one) or the sparse bit-flip sampler
      flips.clear();
      if (reset_one && !elite && misc.w < a.mut_ind_thresh)
        flips.push_back(word_to_index(bin_mut_word(a.key, child, 0), L));
      if (bitflip && !elite && a.mut_sparse) sparse_positions(a, child, binom_count(misc.w, a.mut_thr), flips);

      // per-lane objective accumulators
      uint32_t acc_u[64] = {0};
      uint32_t first0[64];
      float acc_v[64] = {0}, acc_w[64] = {0};
      for (uint32_t q = 0; q < GS; ++q) first0[q] = 0xFFFFFFFFu;

      for (uint32_t c0 = 0; c0 < nchunks; c0 += GS) {
        for (uint32_t q = 0; q < GS; ++q) {
          const uint32_t c = c0 + q;
          uint32_t* v = &seg[q * 4];
          v[0] = v[1] = v[2] = v[3] = 0;
          if (c >= nchunks) continue;
          if (mode == MODE_INIT) {
            u32x4 r = draw(a.key, ST_INIT, child, c);
            v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
          } else if (mode == MODE_EVAL || mode == MODE_MUTATE) {
            std::memcpy(v, cur + child * rw + 4 * c, 16);
          } else {
            const uint32_t* A = cur + (uint64_t)pa * rw + 4 * c;
            if (xo) {
              const uint32_t* B = cur + (uint64_t)pb * rw + 4 * c;
              uint32_t m[4];
              if (a.crossover == XO_UNIFORM) {
                u32x4 r = draw(a.key, ST_XO, child, c);
                m[0] = r.x; m[1] = r.y; m[2] = r.z; m[3] = r.w;
              } else {
                for (int j = 0; j < 4; ++j) m[j] = ~range_mask32(c * 128u + 32u * j, blo, bhi);
              }
              for (int j = 0; j < 4; ++j) v[j] = (A[j] & m[j]) | (B[j] & ~m[j]);
            } else {
              std::memcpy(v, A, 16);
            }
          }
          if (c == nchunks - 1) {
            v[0] &= a.last_mask.x; v[1] &= a.last_mask.y; v[2] &= a.last_mask.z; v[3] &= a.last_mask.w;
          }
        }
        for (uint32_t q = 0; q < GS; ++q) {
          const uint32_t c = c0 + q;
          if (c >= nchunks) continue;
          uint32_t* v = &seg[q * 4];
          if (bitflip && !elite && !a.mut_sparse) {
            const uint32_t clen = std::min(128u, L - c * 128u);
            u32x4 m = chunk_flip_mask(a, child, c, clen, bin_chunk_mut_word(a.key, child, c), a.mut_thr);
            v[0] ^= m.x; v[1] ^= m.y; v[2] ^= m.z; v[3] ^= m.w;
          } else {
            for (uint32_t pos : flips)
              if ((pos >> 7) == c) v[(pos & 127u) >> 5] ^= 1u << (pos & 31u);
          }
        }
        for (uint32_t q = 0; q < GS; ++q) {
          const uint32_t c = c0 + q;
          if (c >= nchunks) continue;
          const uint32_t* v = &seg[q * 4];
          if (mode != MODE_EVAL) std::memcpy(nxt + child * rw + 4 * c, v, 16);
          if (!evaluates) continue;
          if (a.objective == OBJ_ONEMAX) {
            acc_u[q] += popc(v[0]) + popc(v[1]) + popc(v[2]) + popc(v[3]);
          } else if (a.objective == OBJ_KNAPSACK) {
            for (int j = 0; j < 4; ++j) {
              uint32_t bits = v[j];
              const uint32_t base = c * 128u + 32u * j;
              while (bits) {
                uint32_t b = (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1;
                acc_v[q] += a.obj_data[base + b];
                acc_w[q] += a.obj_data[L + base + b];
              }
            }
          } else if (a.objective == OBJ_TRAP) {
            const uint32_t k = (uint32_t)a.obj_i;
            const uint32_t km = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
            for (int j = 0; j < 4; ++j) {
              const uint32_t base = c * 128u + 32u * j;
              for (uint32_t i = 0; i < 32u; i += k) {
                if (base + i + k > L) break;
                uint32_t ones = popc((v[j] >> i) & km);
                acc_u[q] += ones == k ? k : (k - 1 - ones);
              }
            }
          } else if (a.objective == OBJ_LEADING_ONES) {
            for (int j = 0; j < 4; ++j) {
              uint32_t inv = ~v[j];
              if (inv) {
                uint32_t p = c * 128u + 32u * j + (uint32_t)__builtin_ctz(inv);
                first0[q] = std::min(first0[q], p);
                break;
              }
            }
          }
        }
      }
      if (evaluates) {
        if (a.objective == OBJ_ONEMAX || a.objective == OBJ_TRAP) {
          uint32_t s = 0;
          for (uint32_t q = 0; q < GS; ++q) s += acc_u[q];
          score = (float)s;
        } else if (a.objective == OBJ_KNAPSACK) {
          float vv = butterfly_sum(acc_v, GS), ww = butterfly_sum(acc_w, GS);
          score = ww <= a.obj_f0 ? vv : a.obj_f0 - ww;
        } else if (a.objective == OBJ_LEADING_ONES) {
          uint32_t m = 0xFFFFFFFFu;
          for (uint32_t q = 0; q < GS; ++q) m = std::min(m, first0[q]);
          score = (float)std::min(m, L);
        }
      }
    }
    if (evaluates) {
      a.score_next[child] = score;
      best = std::max(best, pack_best(score, child));
    }
  }
  bests[slot] = best;
  });
  const unsigned long long best = *std::max_element(bests.begin(), bests.end());
  if (evaluates && best_parts) best_parts[0] = best;
  return 1;
}

// ------------------------------------------------------------- utilities ---
unsigned long long reduce_best(const unsigned long long* parts, uint32_t n) {
  unsigned long long b = 0;
  for (uint32_t i = 0; i < n; ++i) b = std::max(b, parts[i]);
  return b;
}

unsigned long long best_of_scores(const float* scores, uint64_t S) {
  unsigned long long b = 0;
  for (uint64_t i = 0; i < S; ++i) b = std::max(b, pack_best(scores[i], i));
  return b;
}

void score_stats(const float* s, uint64_t S, float* out) {
  float mn = INFINITY, mx = -INFINITY;
  double sm = 0;
  for (uint64_t i = 0; i < S; ++i) {
    mn = std::fmin(mn, s[i]);
    mx = std::fmax(mx, s[i]);
    sm += s[i];
  }
  out[0] = mn;
  out[1] = mx;
  out[2] = (float)sm;
  out[3] = (float)S;
}

void roulette_prefix(const float* s, uint64_t S, float* cumfit) {
  float st[4];
  score_stats(s, S, st);
  // accumulated in f64 and rounded once per entry: integer weights give the
  // exact prefix the GPU's integer roulette computes (util.hip
  // roulette_fused_kernel) at any population size
  double acc = 0.0;
  for (uint64_t i = 0; i < S; ++i) {
    acc += (double)std::fmax(s[i] - st[0], 0.f);
    cumfit[i] = (float)acc;
  }
}

// ascending (score_key, index): the order a stable LSD radix sort of the
// keys produces on the GPU (util.hip rank_order_launch)
void rank_order(const float* s, uint64_t S, uint32_t* order) {
  std::vector<uint32_t> key(S);
  for (uint64_t i = 0; i < S; ++i) {
    key[i] = score_key(s[i]);
    order[i] = (uint32_t)i;
  }
  std::stable_sort(order, order + S, [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
}

void topk(const float* scores, uint64_t S, uint32_t k, bool largest, uint32_t* idx_out, bool sorted) {
  if (k > S) throw std::runtime_error("topk: k > S");
  if (k == 0) return;
  auto key = [&](uint32_t i) {
    uint32_t kk = score_key(scores[i]);
    return largest ? kk : ~kk;
  };
  std::vector<uint32_t> idx(S);
  std::iota(idx.begin(), idx.end(), 0u);
  if (sorted) {
    std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), [&](uint32_t x, uint32_t y) {
      uint32_t kx = key(x), ky = key(y);
      return kx != ky ? kx > ky : x < y;
    });
    std::memcpy(idx_out, idx.data(), 4ull * k);
    return;
  }
  // selection order (matches the GPU's unsorted mode): keys above the k-th
  // largest key T by index, then the first (k - #above) keys equal to T by index
  std::vector<uint32_t> keys(S);
  for (uint64_t i = 0; i < S; ++i) keys[i] = key((uint32_t)i);
  std::vector<uint32_t> tmp(keys);
  std::nth_element(tmp.begin(), tmp.begin() + (k - 1), tmp.end(), std::greater<uint32_t>());
  const uint32_t T = tmp[k - 1];
  uint32_t n = 0, above = 0;
  for (uint64_t i = 0; i < S; ++i) above += keys[i] > T;
  uint32_t need_eq = k - above;
  for (uint64_t i = 0; i < S; ++i)
    if (keys[i] > T) idx_out[n++] = (uint32_t)i;
  for (uint64_t i = 0; i < S && need_eq; ++i)
    if (keys[i] == T) {
      idx_out[n++] = (uint32_t)i;
      --need_eq;
    }
}

void stripe_emigrate(const float* scores, const void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                     void* out_rows, float* out_scores) {
  for (uint32_t i = 0; i < k; ++i) {
    const uint64_t lo = (uint64_t)i * S / k, hi = (uint64_t)(i + 1) * S / k;
    unsigned long long b = 0;
    for (uint64_t j = lo; j < hi; ++j) b = std::max(b, pack_best(scores[j], j));
    const uint64_t src = best_index(b);
    std::memcpy((uint32_t*)out_rows + (uint64_t)i * row_words, (const uint32_t*)rows + src * row_words,
                4ull * row_words);
    out_scores[i] = scores[src];
  }
}

void stripe_immigrate(float* scores, void* rows, uint32_t row_words, uint64_t S, uint32_t k, const void* in_rows,
                      const float* in_scores) {
  for (uint32_t i = 0; i < k; ++i) {
    const uint64_t lo = (uint64_t)i * S / k, hi = (uint64_t)(i + 1) * S / k;
    unsigned long long w = ~0ull;  // (score key << 32 | index): the minimum is the worst, lowest index
    for (uint64_t j = lo; j < hi; ++j) w = std::min(w, ((unsigned long long)score_key(scores[j]) << 32) | j);
    const uint64_t dst = (uint32_t)w;
    std::memcpy((uint32_t*)rows + dst * row_words, (const uint32_t*)in_rows + (uint64_t)i * row_words,
                4ull * row_words);
    scores[dst] = in_scores[i];
  }
}

void gather_rows(const void* rows, const float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                 void* out_rows, float* out_scores) {
  for (uint32_t r = 0; r < n; ++r) {
    std::memcpy((uint32_t*)out_rows + (uint64_t)r * row_words, (const uint32_t*)rows + (uint64_t)idx[r] * row_words,
                4ull * row_words);
    if (scores && out_scores) out_scores[r] = scores[idx[r]];
  }
}

void scatter_rows(void* rows, float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                  const void* in_rows, const float* in_scores) {
  for (uint32_t r = 0; r < n; ++r) {
    std::memcpy((uint32_t*)rows + (uint64_t)idx[r] * row_words, (const uint32_t*)in_rows + (uint64_t)r * row_words,
                4ull * row_words);
    if (scores && in_scores) scores[idx[r]] = in_scores[r];
  }
}

}  // namespace cpu
}  // namespace pga
