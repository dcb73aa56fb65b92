// E1 — "continuous OneMax": maximise the sum of 100 float genes in [0, 1].
// The reference's first example (test/test.cu) rewritten against pga.h with a
// user __device__ objective handed over as a device function pointer.
//   e1_onemax_float [generations] [population] [cb]
// "cb" also installs a user mutation callback, which moves generations onto
// the reference-ABI callback kernel (compat.hip); every score is then checked
// to be a real evaluation, so a population beyond one launch's worth of
// threads (e.g. 4M) proves the grid-stride coverage.
// Build: python tools/build.py   ->  build/examples/e1_onemax_float
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pga.h"
#include "pga_ext.h"

#define GENOME_LENGTH 100

__device__ float sum_genes(gene* g, unsigned n) {
  float s = 0.f;
  for (unsigned i = 0; i < n; ++i) s += g[i];
  return s;
}
__device__ obj_f sum_genes_ptr = sum_genes;

// 5% of children get one gene reset to a fresh uniform
__device__ void reset_one(gene* g, float* rand, unsigned n) {
  if (rand[0] <= 0.05f) {
    unsigned i = (unsigned)(rand[1] * (float)n);
    g[i < n ? i : n - 1] = rand[2];
  }
}
__device__ mutate_f reset_one_ptr = reset_one;

int main(int argc, char** argv) {
  const unsigned gens = argc > 1 ? (unsigned)atoi(argv[1]) : 100;
  const unsigned long size = argc > 2 ? strtoul(argv[2], NULL, 10) : 40000;
  const int cb = argc > 3 && strcmp(argv[3], "cb") == 0;
  pga_t* p = pga_init();
  if (!p) return 1;
  population_t* pop = pga_create_population(p, size, GENOME_LENGTH, RANDOM_POPULATION);
  if (!pop) return 1;
  obj_f f;
  if (hipMemcpyFromSymbol(&f, HIP_SYMBOL(sum_genes_ptr), sizeof(f)) != hipSuccess) return 2;
  pga_set_objective_function(p, f);
  if (cb) {
    mutate_f m;
    if (hipMemcpyFromSymbol(&m, HIP_SYMBOL(reset_one_ptr), sizeof(m)) != hipSuccess) return 2;
    pga_set_mutate_function(p, m);
  }
  // a short warm-up run (code objects loaded, clocks up), then the timed run:
  // generations through the user's function pointer, plus pga_run's final
  // evaluation (src/pga.cu:376-391 order)
  pga_run(p, 5);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pga_run(p, gens);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  clock_gettime(CLOCK_MONOTONIC, &t1);
  const double us = ((t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_nsec - t0.tv_nsec) * 1e-3) / (gens ? gens : 1);
  printf("{\"e1_fnptr_us_per_gen\": %.2f, \"gens\": %u, \"population\": %lu, \"user_mutation\": %d}\n", us, gens,
         size, cb);
  gene* best = pga_get_best(p, pop);  // prints the best score
  float s = 0.f;
  for (int i = 0; i < GENOME_LENGTH; ++i) s += best[i];
  printf("E1 best sum %.3f of %d (population %lu%s)\n", s, GENOME_LENGTH, size, cb ? ", user mutation" : "");
  free(best);
  float* scores = (float*)malloc(sizeof(float) * size);
  if (!scores || pga_get_scores(p, pop, scores) != 0) return 4;
  unsigned long bad = 0;
  unsigned long long h = 1469598103934665603ull;  // FNV-1a of the score bytes: equal runs, equal hashes
  for (unsigned long i = 0; i < size; ++i) {
    bad += !(scores[i] > 0.f && scores[i] <= (float)GENOME_LENGTH);
    unsigned int u;
    memcpy(&u, &scores[i], 4);
    for (int b = 0; b < 4; ++b) h = (h ^ ((u >> (8 * b)) & 0xFFu)) * 1099511628211ull;
  }
  printf("E1 scores hash %016llx\n", h);
  free(scores);
  pga_deinit(p);
  if (bad) {
    printf("E1: %lu of %lu scores are not evaluations\n", bad, size);
    return 5;
  }
  return s > 0.9f * GENOME_LENGTH ? 0 : 3;
}
