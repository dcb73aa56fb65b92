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
// Two kernels:
//   binary_kernel<GS,OBJ,MODE>   every mode / operator / genome length; one
//                                child per group at a time
//   binary_gen_tp<GS,OBJ,XO,KEY> the hot generation path (L <= 8192 bits,
//                                tournament-2, roulette, linear ranking or
//                                random selection), see below
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
namespace {

using namespace dev;

template <typename K>
uint32_t go(K kernel, const GenArgs& a, unsigned long long* parts, uint32_t gpb, hipStream_t s) {
  const uint32_t grid = launch_grid_occ(a.S, gpb, (const void*)kernel);
  hipLaunchKernelGGL(kernel, grid, kBlock, 0, s, a, parts);
  return grid;
}

template <typename K>
uint32_t go_tp(K kernel, const GenArgs& a0, unsigned long long* parts, hipStream_t s) {
  const TpGeom t = tp_geometry(a0.S, 1, (const void*)kernel, 64 / group_size(a0.chunks));
  GenArgs a = a0;
  a.tp_unit = t.unit;
  hipLaunchKernelGGL(kernel, t.grid, t.block, t.lds, s, a, parts);
  return t.grid;
}

template <int GS, int OBJ>
uint32_t launch_mode(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  constexpr uint32_t gpb = kBlock / GS;
  switch (mode) {
    case MODE_GEN: {
      const bool fast = a.chunks <= (uint32_t)GS &&
                        ((a.selection == SEL_TOURNAMENT && a.tour_k == 2) || a.selection == SEL_RANDOM ||
                         (a.selection == SEL_RANK && a.rank_order != nullptr) ||
                         (a.selection == SEL_ROULETTE && a.cumfit != nullptr && a.roul_guide != nullptr)) &&
                        !(a.n_elite > 1 && a.elite_idx == nullptr) && !force_generic_kernels();
      constexpr bool INT_OBJ = OBJ == OBJ_ONEMAX || OBJ == OBJ_LEADING_ONES || OBJ == OBJ_TRAP;
      // 32-bit offsets: the (S + kRowPad)-row buffers must stay below 4 GiB
      const bool o32 = (a.S + kRowPad) * (uint64_t)a.row_words * 4u <= 0xFFFFFFFFull;
      if (fast && o32 && a.n_elite <= kTpMaxElite && (!INT_OBJ || a.key_cur != nullptr)) {
        if constexpr (OBJ == OBJ_KNAPSACK && GS >= 4 && GS <= 32) {
          if (a.knap_tab != nullptr &&
              (a.knap_cols == 0 || a.knap_cols > kKnapMaxCols || a.knap_dig == 0 || a.knap_dig > 4 ||
               a.knap_cols != (uint32_t)GS / 2u * a.knap_dig))
            throw std::invalid_argument("knapsack digit table does not match the genome geometry");
        }
        const bool dense = a.mutation == MUT_BIT_FLIP && a.mut_rate > 0.f && !a.mut_sparse;
        const bool full = a.chunks == (uint32_t)GS;
        if constexpr (OBJ == OBJ_KNAPSACK && GS >= 4 && GS <= 32) {
          if (a.knap_tab != nullptr) {  // integer-exact instance: the matrix-core evaluation
            if (full) {
              if (dense) return go_tp(binary_gen_tp<GS, kObjKnapMfma, true, true>, a, parts, s);
              return go_tp(binary_gen_tp<GS, kObjKnapMfma, true, false>, a, parts, s);
            }
            if (dense) return go_tp(binary_gen_tp<GS, kObjKnapMfma, false, true>, a, parts, s);
            return go_tp(binary_gen_tp<GS, kObjKnapMfma, false, false>, a, parts, s);
          }
        }
        if (full) {
          if (dense) return go_tp(binary_gen_tp<GS, OBJ, true, true>, a, parts, s);
          return go_tp(binary_gen_tp<GS, OBJ, true, false>, a, parts, s);
        }
        if (dense) return go_tp(binary_gen_tp<GS, OBJ, false, true>, a, parts, s);
        return go_tp(binary_gen_tp<GS, OBJ, false, false>, a, parts, s);
      }
      return go(binary_kernel<GS, OBJ, MODE_GEN>, a, parts, gpb, s);
    }
    case MODE_INIT: return go(binary_kernel<GS, OBJ, MODE_INIT>, a, parts, gpb, s);
    case MODE_EVAL: return go(binary_kernel<GS, OBJ, MODE_EVAL>, a, parts, gpb, s);
    case MODE_CROSS: return go(binary_kernel<GS, OBJ_NONE, MODE_CROSS>, a, parts, gpb, s);
    default: return go(binary_kernel<GS, OBJ_NONE, MODE_MUTATE>, a, parts, gpb, s);
  }
}

template <int GS>
uint32_t launch_obj(int mode, const GenArgs& a, unsigned long long* parts, hipStream_t s) {
  switch (a.objective) {
    case OBJ_ONEMAX: return launch_mode<GS, OBJ_ONEMAX>(mode, a, parts, s);
    case OBJ_KNAPSACK: return launch_mode<GS, OBJ_KNAPSACK>(mode, a, parts, s);
    case OBJ_TRAP: return launch_mode<GS, OBJ_TRAP>(mode, a, parts, s);
    case OBJ_LEADING_ONES: return launch_mode<GS, OBJ_LEADING_ONES>(mode, a, parts, s);
    default: return launch_mode<GS, OBJ_NONE>(mode, a, parts, s);
  }
}

}  // namespace

#ifdef PGA_TP_TIMING
// experiment builds: mean per-wave cycles of the tournament / breed phases of
// the last binary_gen_tp launch (bench/gen_bench.cpp prints it)
extern "C" void pga_tp_timing_dump(uint32_t nwaves) {
  static unsigned long long h[kMaxGrid * 4][8];  // per wave: blockIdx.x * waves + wave
  PGA_HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(pga_tp_clk), sizeof(h)));
  double t = 0, b = 0, tot = 0, n = 0, mx = 0;
  unsigned long long rt_min = ~0ull, rt_max = 0, st_max = 0;
  uint32_t nw = 0;
  for (uint32_t i = 0; i < nwaves && i < kMaxGrid * 4; ++i) {
    if (h[i][2] == 0) continue;
    t += (double)h[i][0];
    b += (double)h[i][1];
    tot += (double)h[i][2];
    mx = std::max(mx, (double)h[i][2]);
    n += 1;
    rt_min = std::min(rt_min, h[i][4]);
    rt_max = std::max(rt_max, h[i][5]);
    st_max = std::max(st_max, h[i][4]);
    nw = i + 1;
  }
  std::printf("{\"tp_timing\": {\"waves\": %.0f, \"tourn_cycles\": %.0f, \"breed_cycles\": %.0f, "
              "\"wave_cycles\": %.0f, \"max_wave_cycles\": %.0f, \"tourn_frac\": %.3f, "
              "\"span_us\": %.2f, \"last_start_us\": %.2f}}\n",
              n, t / n, b / n, tot / n, mx, t / (t + b), (rt_max - rt_min) / 100.0, (st_max - rt_min) / 100.0);
  // wall-clock end time (us after the first start, 100 MHz clock) per XCD and
  // by block order (older blocks first): is the tail an XCD or an age effect?
  double xe[8] = {0}, xm[8] = {0}, xn[8] = {0};
  const uint32_t bins = 8;
  double be[bins] = {0}, bm[bins] = {0}, bn[bins] = {0}, bs[bins] = {0};
  for (uint32_t i = 0; i < nw; ++i) {
    if (h[i][2] == 0) continue;
    const double e = (h[i][5] - rt_min) / 100.0, st = (h[i][4] - rt_min) / 100.0;
    const uint32_t x = (uint32_t)(h[i][6] & 7u), k = i * bins / nw;
    xe[x] += e; xn[x] += 1; xm[x] = std::max(xm[x], e);
    be[k] += e; bn[k] += 1; bm[k] = std::max(bm[k], e); bs[k] += st;
  }
  std::printf("{\"tp_xcd_end_us\": [");
  for (int x = 0; x < 8; ++x) std::printf("%s[%.1f, %.1f]", x ? ", " : "", xn[x] ? xe[x] / xn[x] : 0.0, xm[x]);
  std::printf("], \"tp_order_start_end_max_us\": [");
  for (uint32_t k = 0; k < bins; ++k)
    std::printf("%s[%.1f, %.1f, %.1f]", k ? ", " : "", bn[k] ? bs[k] / bn[k] : 0.0, bn[k] ? be[k] / bn[k] : 0.0, bm[k]);
  std::printf("]}\n");
}
#endif

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

uint32_t binary_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
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
