// binary.hip — bit-packed BINARY encoding on gfx950.
//
// One individual = one row of `chunks` 16-byte chunks (128 genes each).  A
// group of GS = group_size(chunks) lanes owns one individual: lane q holds
// chunk q (q+GS, ... for genomes longer than 64 chunks), so every parent-row
// gather is a fully used 16 B/lane dwordx4 load (8 lanes = one 128-B line for
// the 1024-bit headline config) and the fitness reduction is a GS-lane
// butterfly.  ONE launch per generation fuses
//     tournament selection -> crossover -> bit-flip mutation -> fitness
//     -> child store + score store + per-block best
// replacing the reference's RNG-fill + 3 kernels x ceil(S/512) launches + 3
// device syncs per generation (src/pga.cu:376-391, :250-347).  No random
// buffer is materialised: every draw is an in-register Philox4x32-10 (the
// BINARY randomness layout is defined in core.hpp).
//
// Two kernels (binary_dev.hpp):
//   binary_kernel<GS,OBJ,MODE>   every mode / operator / genome length; one
//                                child per group at a time
//   binary_gen_tp<GS,OBJ,XO,KEY> the hot generation path (L <= 8192 bits,
//                                tournament-2, roulette, linear ranking or
//                                random selection)
// This file: the knapsack digit table, the hot-kernel plan and the group-size
// dispatch; the launchers are instantiated per group size in binary_gs.hip
// (one translation unit each, compiled in parallel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <type_traits>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/tp.hpp"
#include "pga/binary_dev.hpp"

namespace pga {

using namespace dev;

bool build_knap_table(const float* values, const float* weights, uint32_t L, uint32_t chunks,
                      std::vector<uint8_t>& tab, uint32_t& digits, uint32_t& cols) {
  tab.clear();
  digits = cols = 0;
  const uint32_t GS = group_size(chunks);
  if (GS < 4 || GS > 32 || chunks > GS) return false;
  double sv = 0, sw = 0;
  int64_t vmax = 0;
  for (uint32_t i = 0; i < L; ++i) {
    for (const float x : {values[i], weights[i]}) {
      if (!(x == std::nearbyint(x)) || std::fabs(x) >= 16777216.f) return false;
      vmax = std::max<int64_t>(vmax, (int64_t)std::fabs(x));
    }
    sv += std::fabs(values[i]);
    sw += std::fabs(weights[i]);
  }
  if (sv >= 16777216.0 || sw >= 16777216.0) return false;
  uint32_t D = 1;  // balanced base-256 digits in [-128, 127]
  for (int64_t lim = 127; vmax > lim && D < 4; ++D) lim = lim * 256 + 127;
  const uint32_t R = GS / 4, NC = 2 * R * D;
  if (NC > kKnapMaxCols) return false;
  tab.assign((size_t)kKnapSlices * 4 * kKnapMaxCols * 16, 0);  // [s][h][16 columns], columns >= NC zero
  for (uint32_t s = 0; s < kKnapSlices; ++s)
    for (uint32_t h = 0; h < 4; ++h)
      for (uint32_t c = 0; c < NC; ++c) {
        const uint32_t r = c / (2 * D), qty = (c / D) & 1u, d = c % D;
        for (uint32_t j = 0; j < 16; ++j) {
          const uint32_t gi = 128u * (4u * r + h) + 16u * s + j;
          int64_t x = gi < L ? (int64_t)(qty ? weights[gi] : values[gi]) : 0;
          int dig = 0;
          for (uint32_t k = 0; k <= d; ++k) {
            dig = (int)(((x + 128) & 255) - 128);
            x = (x - dig) / 256;
          }
          tab[(((size_t)s * 4 + h) * kKnapMaxCols + c) * 16 + j] = (uint8_t)(int8_t)dig;
        }
      }
  digits = D;
  cols = NC;
  return true;
}

bool binary_tp_plan(const GenArgs& a, uint32_t& gs, bool& full, bool& dense) {
  // the conditions launch_mode applies before choosing binary_gen_tp, for an
  // objective that tournaments on f32 scores (a JIT objective)
  gs = group_size(a.chunks);
  const bool fast = ((a.selection == SEL_TOURNAMENT && a.tour_k == 2) || a.selection == SEL_RANDOM ||
                     (a.selection == SEL_RANK && a.rank_order != nullptr) ||
                     (a.selection == SEL_ROULETTE && a.cumfit != nullptr && a.roul_guide != nullptr)) &&
                    !(a.n_elite > 1 && a.elite_idx == nullptr) && !force_generic_kernels();
  const bool o32 = (a.S + kRowPad) * (uint64_t)a.row_words * 4u <= 0xFFFFFFFFull;
  full = a.chunks == gs;
  dense = a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f && !a.mut_sparse;
  return a.chunks <= 64u && fast && o32 && a.n_elite <= kTpMaxElite;
}

bool& binary_hist_written() {
  static thread_local bool w = false;
  return w;
}

bool& binary_rank_counts_written() {
  static thread_local bool w = false;
  return w;
}

TpPartition& binary_tp_partition() {
  static thread_local TpPartition p{0, 0, 0};
  return p;
}

uint32_t binary_launch_multi(const GenArgs& a, const MultiGenArgs& mg, hipStream_t s) {
  if (mg.gens < 2 || force_generic_kernels()) return 0;
  uint32_t grid = 0;
  switch (group_size(a.chunks)) {
    case 1: grid = binary_launch_multi_group<1>(a, mg, s); break;
    case 2: grid = binary_launch_multi_group<2>(a, mg, s); break;
    case 4: grid = binary_launch_multi_group<4>(a, mg, s); break;
    case 8: grid = binary_launch_multi_group<8>(a, mg, s); break;
    case 16: grid = binary_launch_multi_group<16>(a, mg, s); break;
    case 32: grid = binary_launch_multi_group<32>(a, mg, s); break;
    default: grid = binary_launch_multi_group<64>(a, mg, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

uint32_t binary_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  uint32_t grid = 0;
  binary_hist_written() = false;  // go_tp sets it when its kernel takes the histogram
  binary_rank_counts_written() = false;
  binary_tp_partition() = TpPartition{0, 0, 0};
  switch (group_size(a.chunks)) {  // one translation unit per group size (binary_gs.hip)
    case 1: grid = binary_launch_group<1>(mode, a, best_parts, s); break;
    case 2: grid = binary_launch_group<2>(mode, a, best_parts, s); break;
    case 4: grid = binary_launch_group<4>(mode, a, best_parts, s); break;
    case 8: grid = binary_launch_group<8>(mode, a, best_parts, s); break;
    case 16: grid = binary_launch_group<16>(mode, a, best_parts, s); break;
    case 32: grid = binary_launch_group<32>(mode, a, best_parts, s); break;
    default: grid = binary_launch_group<64>(mode, a, best_parts, s); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace pga
