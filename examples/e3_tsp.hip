// E3 — TSP with float random keys: city_i = (int)(g_i * n).  Objective =
// -(open path length + 10000 per duplicated ordered pair); a user crossover
// repairs duplicates (takes parent 1's city if unused, else parent 2's, else
// the rand value).  The reference's third example (test3/test.cu), with the
// out-of-bounds decode (g = 1.0 -> city n) clamped and the distance matrix
// copied with its real stride.  Input on stdin: n, then n*n distances
// (examples/gen_tsp.c plants the path 0->1->...->n-1 of length 10 (n-1)).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "pga.h"

#define MAX_CITIES 128
__constant__ float dist[MAX_CITIES * MAX_CITIES];

__device__ inline int city(float g, unsigned n) {
  int c = (int)(g * (float)n);
  return c >= (int)n ? (int)n - 1 : c;
}

__device__ float tour(gene* g, unsigned n) {
  float len = 0.f;
  for (unsigned i = 1; i < n; ++i) len += dist[city(g[i - 1], n) * n + city(g[i], n)];
  for (unsigned i = 0; i < n; ++i)
    for (unsigned j = 0; j < n; ++j)
      if (i != j && city(g[i], n) == city(g[j], n)) len += 10000.f;
  return -len;
}

__device__ void repair_crossover(gene* p1, gene* p2, gene* c, float* rand, unsigned n) {
  unsigned long long used[MAX_CITIES / 64] = {0, 0};
  for (unsigned i = 0; i < n; ++i) {
    const int a = city(p1[i], n), b = city(p2[i], n);
    if (!((used[a / 64] >> (a % 64)) & 1ull)) {
      c[i] = p1[i];
      used[a / 64] |= 1ull << (a % 64);
    } else if (!((used[b / 64] >> (b % 64)) & 1ull)) {
      c[i] = p2[i];
      used[b / 64] |= 1ull << (b % 64);
    } else {
      c[i] = rand[i];
    }
  }
}

__device__ obj_f tour_ptr = tour;
__device__ crossover_f repair_ptr = repair_crossover;

int main(int argc, char** argv) {
  const unsigned gens = argc > 1 ? (unsigned)atoi(argv[1]) : 1000;
  int n = 0;
  if (scanf("%d", &n) != 1 || n < 4 || n > MAX_CITIES) {
    fprintf(stderr, "expected a city count in [4, %d] on stdin\n", MAX_CITIES);
    return 1;
  }
  static float h[MAX_CITIES * MAX_CITIES];
  for (int i = 0; i < n * n; ++i)
    if (scanf("%f", &h[i]) != 1) return 1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(dist), h, sizeof(float) * n * n) != hipSuccess) return 2;

  pga_t* p = pga_init();
  if (!p) return 1;
  population_t* pop = pga_create_population(p, 1000, (unsigned)n, RANDOM_POPULATION);
  obj_f f;
  crossover_f x;
  if (hipMemcpyFromSymbol(&f, HIP_SYMBOL(tour_ptr), sizeof(f)) != hipSuccess) return 2;
  if (hipMemcpyFromSymbol(&x, HIP_SYMBOL(repair_ptr), sizeof(x)) != hipSuccess) return 2;
  pga_set_objective_function(p, f);
  pga_set_crossover_function(p, x);
  pga_run(p, gens);
  gene* g = pga_get_best(p, pop);
  int seen[MAX_CITIES] = {0}, dups = 0;
  for (int i = 0; i < n; ++i) {
    int c = (int)(g[i] * n);
    if (c >= n) c = n - 1;
    dups += seen[c]++ > 0;
    printf("%d ", c);
  }
  printf("\nduplicates: %d\n", dups);
  free(g);
  pga_deinit(p);
  return dups == 0 ? 0 : 3;
}
