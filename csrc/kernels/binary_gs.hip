// binary_gs.hip — the BINARY launchers of ONE group size (built once per
// group size by tools/build.py with -DPGA_BIN_GS=<1|2|4|...|64>, so the seven
// sets of kernel instantiations compile in parallel): the generic kernel for
// every mode and the two-phase generation kernel binary_gen_tp for every
// objective / variant of this group size (binary_dev.hpp, binary.hip).
#ifndef PGA_BIN_GS
#error "build with -DPGA_BIN_GS=<group size>"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

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
  a.tp_pool_units = a.tp_pool ? tp_pool_units(t, a.S) : 0u;
  a.tp_skew = tp_skew_units(t, a.S);
  // the fused key histogram's LDS bins follow the round's parents
  // (binary_gen_tp's HISTK: the objectives with exact u16 keys)
  const bool key_obj = a.objective == OBJ_ONEMAX || a.objective == OBJ_LEADING_ONES || a.objective == OBJ_TRAP;
  const bool hist = key_obj && a.key_cur != nullptr && a.key_hist != nullptr && a.hist_bins > 0 &&
                    a.hist_bins <= kHistMaxBins;
  if (!hist) a.key_hist = nullptr;
  // the rank sort's tile counts: only when block b's children are exactly
  // sort tile b (tp_share with a share of kRankTile, a multiple of every
  // unit; no pair pool).  The share skew (PGA_TP_SKEW, worth ~0.5 us at the
  // headline) is dropped for it: the count pass it saves costs ~6 us.
  const bool rk = key_obj && a.key_cur != nullptr && a.rank_counts != nullptr && a.hist_bins > 0 &&
                  a.hist_bins <= kHistMaxBins && a.tp_pool_units == 0 &&
                  (a.S + t.grid - 1) / t.grid == kRankTile && (uint64_t)t.grid == (a.S + kRankTile - 1) / kRankTile;
  if (rk) a.tp_skew = 0;
  else a.rank_counts = nullptr;
  hipLaunchKernelGGL(kernel, t.grid, t.block, t.lds + (hist || rk ? 4u * a.hist_bins : 0u), s, a, parts);
  binary_hist_written() = hist;
  binary_rank_counts_written() = rk;
  if (a.tp_pool_units == 0) binary_tp_partition() = TpPartition{t.grid, tp_unit(a, 64u / group_size(a.chunks)), a.tp_skew};
  return t.grid;
}

// G generations in one persistent launch (binary_dev.hpp binary_gen_tp_multi):
// only the headline geometry (one 16-wave block per CU), else 0 (run them
// one launch each)
template <typename K>
uint32_t go_tp_multi(K kernel, const GenArgs& a0, const MultiGenArgs& mg, hipStream_t s) {
  const TpGeom t = tp_geometry(a0.S, 1, (const void*)kernel, 64 / group_size(a0.chunks));
  if (t.block != kTpMaxWaves * 64 || t.grid > (uint32_t)device_cu_count()) return 0;
  GenMulti m;
  m.a = a0;
  m.a.tp_unit = t.unit;
  m.a.tp_pool = nullptr;
  m.a.tp_pool_units = 0;
  m.a.tp_skew = tp_skew_units(t, a0.S);
  const bool hist = mg.hist[0] && mg.hist[1] && mg.hist[2] && mg.hist_bins > 0 && mg.hist_bins <= kHistMaxBins;
  m.a.key_hist = nullptr;
  m.a.hist_zero = nullptr;
  m.a.rank_counts = nullptr;
  m.a.hist_bins = hist ? mg.hist_bins : 0u;
  m.a.hist_zero_words = hist ? mg.hist_zero_words : 0u;
  for (int j = 0; j < 3; ++j) m.hist[j] = hist ? mg.hist[j] : nullptr;
  m.hist_rot = mg.hist_rot;
  m.parts[0] = mg.parts[0];
  m.parts[1] = mg.parts[1];
  m.stats[0] = mg.stats[0];
  m.stats[1] = mg.stats[1];
  m.gens = mg.gens;
  m.bar = mg.barrier;
  PGA_HIP_CHECK(hipMemsetAsync(mg.barrier, 0, 4, s));
  hipLaunchKernelGGL(kernel, t.grid, t.block, t.lds + (hist ? 4u * mg.hist_bins : 0u), s, m);
  binary_hist_written() = hist;
  return t.grid;
}

template <int GS, int OBJ>
uint32_t launch_multi(const GenArgs& a, const MultiGenArgs& mg, hipStream_t s) {
  if constexpr (OBJ == OBJ_ONEMAX || OBJ == OBJ_LEADING_ONES || OBJ == OBJ_TRAP) {
    uint32_t gs = 0;
    bool full = false, dense = false;
    if (a.chunks > (uint32_t)GS || !binary_tp_plan(a, gs, full, dense) || gs != (uint32_t)GS) return 0;
    if (a.key_cur == nullptr || a.key_next == nullptr || a.n_elite > 1 ||
        !(a.selection == SEL_TOURNAMENT || a.selection == SEL_RANDOM))
      return 0;
    if (full) {
      if (dense) return go_tp_multi(binary_gen_tp_multi<GS, OBJ, true, true>, a, mg, s);
      return go_tp_multi(binary_gen_tp_multi<GS, OBJ, true, false>, a, mg, s);
    }
    if (dense) return go_tp_multi(binary_gen_tp_multi<GS, OBJ, false, true>, a, mg, s);
    return go_tp_multi(binary_gen_tp_multi<GS, OBJ, false, false>, a, mg, s);
  }
  (void)a;
  (void)mg;
  (void)s;
  return 0;
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

template <>
uint32_t binary_launch_group<PGA_BIN_GS>(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  return launch_obj<PGA_BIN_GS>(mode, a, best_parts, s);
}

template <>
uint32_t binary_launch_multi_group<PGA_BIN_GS>(const GenArgs& a, const MultiGenArgs& mg, hipStream_t s) {
  switch (a.objective) {
    case OBJ_ONEMAX: return launch_multi<PGA_BIN_GS, OBJ_ONEMAX>(a, mg, s);
    case OBJ_TRAP: return launch_multi<PGA_BIN_GS, OBJ_TRAP>(a, mg, s);
    case OBJ_LEADING_ONES: return launch_multi<PGA_BIN_GS, OBJ_LEADING_ONES>(a, mg, s);
    default: return 0;
  }
}

#if defined(PGA_TP_TIMING) && PGA_BIN_GS == 8
// (only the headline group size's translation unit defines the dump)
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
  {  // producers (waves that ran tournaments) vs breed-only waves
    double c[2][5] = {{0}};
    for (uint32_t i = 0; i < nwaves && i < kMaxGrid * 4; ++i) {
      if (h[i][2] == 0) continue;
      const int k = h[i][0] > 0 ? 0 : 1;
      c[k][0] += 1; c[k][1] += (double)h[i][0]; c[k][2] += (double)h[i][1]; c[k][3] += (double)h[i][7];
      c[k][4] += (double)h[i][3];
    }
    for (int k = 0; k < 2; ++k)
      if (c[k][0] > 0)
        std::printf("{\"tp_%s\": {\"waves\": %.0f, \"tourn_cycles\": %.0f, \"breed_cycles\": %.0f, \"spin_cycles\": %.0f, "
                    "\"children\": %.0f}}\n", k ? "breeders" : "producers", c[k][0], c[k][1] / c[k][0],
                    c[k][2] / c[k][0], c[k][3] / c[k][0], c[k][4] / c[k][0]);
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

}  // namespace pga
