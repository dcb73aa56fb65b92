// E2 — bounded knapsack with 6 items (values / weights in __constant__
// memory), each gene encodes an item count (int)(g * 2); capacity 10.
// The reference's second example (test2/test.cu); known optimum 285 = items
// 2 and 3, i.e. counts "0 0 1 1 0 0".
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "pga.h"

#define ITEMS 6
#define MAX_COUNT 2
#define CAPACITY 10.0f
__constant__ float item_value[ITEMS] = {75, 150, 250, 35, 10, 100};
__constant__ float item_weight[ITEMS] = {7, 8, 6, 4, 3, 9};

__device__ float knapsack(gene* g, unsigned n) {
  float v = 0.f, w = 0.f;
  for (unsigned i = 0; i < n; ++i) {
    const int c = (int)(g[i] * MAX_COUNT);
    v += item_value[i] * c;
    w += item_weight[i] * c;
  }
  return w <= CAPACITY ? v : CAPACITY - w;
}
__device__ obj_f knapsack_ptr = knapsack;

int main(int argc, char** argv) {
  const unsigned gens = argc > 1 ? (unsigned)atoi(argv[1]) : 5;
  pga_t* p = pga_init();
  if (!p) return 1;
  population_t* pop = pga_create_population(p, 100, ITEMS, RANDOM_POPULATION);
  obj_f f;
  if (hipMemcpyFromSymbol(&f, HIP_SYMBOL(knapsack_ptr), sizeof(f)) != hipSuccess) return 2;
  pga_set_objective_function(p, f);
  pga_run(p, gens);
  gene* g = pga_get_best(p, pop);
  int ok = 1;
  const int expect[ITEMS] = {0, 0, 1, 1, 0, 0};
  for (int i = 0; i < ITEMS; ++i) {
    const int c = (int)(g[i] * MAX_COUNT);
    printf("%d ", c);
    ok &= c == expect[i];
  }
  printf("\n");
  free(g);
  pga_deinit(p);
  return ok ? 0 : 3;
}
