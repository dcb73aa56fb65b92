// cpu.hpp — CPU reference backend.
//
// Same operator semantics as the gfx950 kernels, evaluated one individual at a
// time on host memory.  Because every random draw is addressed by
// (seed, generation, island, individual, purpose, block) and group
// reductions follow the same lane butterfly, generations are bit-identical to
// the GPU: rows of every encoding, scores up to the transcendental objectives
// (REAL Rastrigin / Ackley / Griewank / Schwefel, whose libm calls differ from
// the device's by ulps).  This is the oracle of the test-suite and the
// "CPU reference path" config of BASELINE.json.
#pragma once

#include <functional>

#include "pga/core.hpp"

namespace pga {
namespace cpu {

// worker pool of the CPU backend (parallel.cpp): fn(begin, end, slot) over
// contiguous ranges of [0, n), slot < cpu_threads(); serial when n < 2 grains
// or when another generation holds the pool
unsigned cpu_threads();
void parallel_for(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t, unsigned)>& fn);

// returns number of best parts written (always 1)
uint32_t encoding_run(int mode, const GenArgs& a, unsigned long long* best_parts);
uint32_t binary_run(int mode, const GenArgs& a, unsigned long long* best_parts);
uint32_t real_run(int mode, const GenArgs& a, unsigned long long* best_parts);
uint32_t perm_run(int mode, const GenArgs& a, unsigned long long* best_parts);
// PMX (op = XO_PMX) or OX1 child of A and B keeping A's segment [lo, hi)
void perm_crossover(int op, const uint16_t* A, const uint16_t* B, uint32_t L, uint32_t lo, uint32_t hi, uint16_t* C);

unsigned long long reduce_best(const unsigned long long* parts, uint32_t n);
unsigned long long best_of_scores(const float* scores, uint64_t S);
void score_stats(const float* scores, uint64_t S, float* out4);
void roulette_prefix(const float* scores, uint64_t S, float* cumfit);
void rank_order(const float* scores, uint64_t S, uint32_t* order);
void topk(const float* scores, uint64_t S, uint32_t k, bool largest, uint32_t* idx_out, bool sorted = true);
// MIG_STRIPE migration (see ops.hpp stripe_*_launch)
void stripe_emigrate(const float* scores, const void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                     void* out_rows, float* out_scores);
void stripe_immigrate(float* scores, void* rows, uint32_t row_words, uint64_t S, uint32_t k, const void* in_rows,
                      const float* in_scores);
void gather_rows(const void* rows, const float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                 void* out_rows, float* out_scores);
void scatter_rows(void* rows, float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                  const void* in_rows, const float* in_scores);

// CPU emulation of a GS-lane butterfly sum (lane 0's result)
inline float butterfly_sum(float* v, uint32_t GS) {
  float t[64];
  for (uint32_t o = GS / 2; o > 0; o >>= 1) {
    for (uint32_t q = 0; q < GS; ++q) t[q] = v[q] + v[q ^ o];
    for (uint32_t q = 0; q < GS; ++q) v[q] = t[q];
  }
  return v[0];
}

// child word t (see core.hpp for the layout)
inline uint32_t pool_word(const RngKey& key, uint64_t child, uint32_t t) { return child_word(key, child, t); }

void select_parents(const GenArgs& a, uint64_t child, uint32_t& pa, uint32_t& pb);
// parents from the ST_SEL words (the BINARY and REAL layouts)
void bin_select_parents(const GenArgs& a, uint64_t child, uint32_t& pa, uint32_t& pb);

}  // namespace cpu
}  // namespace pga
