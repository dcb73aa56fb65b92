// E1 — "continuous OneMax": maximise the sum of 100 float genes in [0, 1].
// The reference's first example (test/test.cu) rewritten against pga.h with a
// user __device__ objective handed over as a device function pointer.
// Build: python tools/build.py   ->  build/examples/e1_onemax_float
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "pga.h"

#define GENOME_LENGTH 100

__device__ float sum_genes(gene* g, unsigned n) {
  float s = 0.f;
  for (unsigned i = 0; i < n; ++i) s += g[i];
  return s;
}
__device__ obj_f sum_genes_ptr = sum_genes;

int main(int argc, char** argv) {
  const unsigned gens = argc > 1 ? (unsigned)atoi(argv[1]) : 100;
  pga_t* p = pga_init();
  if (!p) return 1;
  population_t* pop = pga_create_population(p, 40000, GENOME_LENGTH, RANDOM_POPULATION);
  obj_f f;
  if (hipMemcpyFromSymbol(&f, HIP_SYMBOL(sum_genes_ptr), sizeof(f)) != hipSuccess) return 2;
  pga_set_objective_function(p, f);
  pga_run(p, gens);
  gene* best = pga_get_best(p, pop);  // prints the best score
  float s = 0.f;
  for (int i = 0; i < GENOME_LENGTH; ++i) s += best[i];
  printf("E1 best sum %.3f of %d\n", s, GENOME_LENGTH);
  free(best);
  pga_deinit(p);
  return s > 0.9f * GENOME_LENGTH ? 0 : 3;
}
