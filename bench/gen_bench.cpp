// gen_bench.cpp — native (no python) generation benchmark of the Island runtime.
//
//   gen_bench [--pop N] [--length L] [--gens G] [--warmup W] [--xo uniform|one|two]
//             [--elitism E] [--encoding binary|real|perm] [--objective N]
//             [--tsp f32|int|euc] [--pmx 1]
// Prints one JSON line: us per generation measured with hipEvents around G
// back-to-back fused generations on the null stream.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pga/island.hpp"
#include "pga/ops.hpp"

// phase clocks of the headline kernel (experiment builds with -DPGA_TP_TIMING)
extern "C" __attribute__((weak)) void pga_tp_timing_dump(uint32_t nwaves);


int main(int argc, char** argv) {
  pga::Config c;
  c.S = 1u << 20;
  c.L = 1024;
  c.objective = pga::OBJ_ONEMAX;
  c.n_elite = 1;
  c.seed = 1234;
  int gens = 300, warm = 30;
  std::string tsp;  // PERMUTATION: the bench_configs.py TSP-256 instance kinds
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--pop") c.S = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--length") c.L = (uint32_t)std::atoi(v.c_str());
    else if (k == "--gens") gens = std::atoi(v.c_str());
    else if (k == "--warmup") warm = std::atoi(v.c_str());
    else if (k == "--elitism") c.n_elite = (uint32_t)std::atoi(v.c_str());
    else if (k == "--objective") c.objective = std::atoi(v.c_str());
    else if (k == "--mutation") c.mutation = v == "reset_one" ? pga::MUT_RESET_ONE : pga::MUT_GAUSSIAN;
    else if (k == "--xo")
      c.crossover = v == "one" ? pga::XO_ONE_POINT
                    : v == "two" ? pga::XO_TWO_POINT
                    : v == "blend" ? pga::XO_BLEND
                    : v == "arith" ? pga::XO_ARITHMETIC : pga::XO_UNIFORM;
    else if (k == "--encoding") {
      c.encoding = v == "real" ? pga::ENC_REAL : (v == "perm" ? pga::ENC_PERMUTATION : pga::ENC_BINARY);
      if (c.encoding == pga::ENC_REAL) {  // the Rastrigin-30D config of bench_configs.py
        c.mutation = pga::MUT_GAUSSIAN;
        c.lo = -5.12f;
        c.hi = 5.12f;
        c.crossover = pga::XO_BLEND;
        c.blend_alpha = 0.3f;
        c.sigma = 0.512f;  // Rastrigin default_operators: 0.05 (hi - lo)
        c.objective = pga::OBJ_RASTRIGIN;
      }
      if (c.encoding == pga::ENC_PERMUTATION) { c.mutation = pga::MUT_SWAP; c.crossover = pga::XO_OX; }
    }
  }
  for (int i = 1; i + 1 < argc; i += 2) {  // options that override the encoding's defaults
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--objective") c.objective = std::atoi(v.c_str());
    else if (k == "--mutation") c.mutation = v == "reset_one" ? pga::MUT_RESET_ONE : pga::MUT_GAUSSIAN;
    else if (k == "--xo") c.crossover = v == "uniform" ? pga::XO_UNIFORM : c.crossover;
    else if (k == "--lo") c.lo = std::strtof(v.c_str(), nullptr);
    else if (k == "--hi") c.hi = std::strtof(v.c_str(), nullptr);
    else if (k == "--pmx") c.crossover = v == "1" ? pga::XO_PMX : pga::XO_OX;
    else if (k == "--tsp") tsp = v;
  }
  if (!tsp.empty()) c.objective = tsp == "euc" ? pga::OBJ_TSP_EUC : pga::OBJ_TSP;
  pga::Island isl(c, 0);
  if (!tsp.empty()) {  // uniform random cities in the unit square (fixed LCG)
    std::vector<float> xy(2 * c.L), d;
    uint64_t st = 7;
    for (auto& x : xy) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      x = (float)((st >> 40) * (1.0 / 16777216.0));
    }
    if (tsp == "euc") {
      d = xy;
    } else {
      d.resize((size_t)c.L * c.L);
      for (uint32_t i = 0; i < c.L; ++i)
        for (uint32_t j = 0; j < c.L; ++j) {
          const float dx = xy[2 * i] - xy[2 * j], dy = xy[2 * i + 1] - xy[2 * j + 1];
          const float e = std::sqrt(dx * dx + dy * dy);
          d[(size_t)i * c.L + j] = tsp == "int" ? std::nearbyint(1000.f * e) : e;
        }
    }
    isl.set_objective_data(d.data(), d.size(), 0);
  }
  isl.initialize();
  isl.run(warm);
  PGA_HIP_CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  PGA_HIP_CHECK(hipEventCreate(&e0));
  PGA_HIP_CHECK(hipEventCreate(&e1));
  PGA_HIP_CHECK(hipEventRecord(e0, nullptr));
  isl.run(gens);
  PGA_HIP_CHECK(hipEventRecord(e1, nullptr));
  PGA_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  PGA_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1000.0 * ms / gens;
  std::printf("{\"pop\": %llu, \"length\": %u, \"gens\": %d, \"us_per_gen\": %.2f, \"gens_per_sec\": %.1f, "
              "\"evals_per_sec\": %.4e, \"best\": %.1f}\n",
              (unsigned long long)c.S, c.L, gens, us, 1e6 / us, 1e6 / us * (double)c.S, isl.best_score());
  if (pga_tp_timing_dump) pga_tp_timing_dump(8192 * 4);
  return 0;
}
