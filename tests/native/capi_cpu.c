/* C API exercise on the CPU reference backend (device -1): every entry point of
 * pga.h plus the pga_ext.h extensions, with assertions.  Built and run under
 * AddressSanitizer + UBSan (host code) by tools/asan_host.sh; also a plain C
 * consumer check of the headers. */
#include <assert.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pga.h"
#include "pga_ext.h"

static pga_t *solver(unsigned long long seed) {
  pga_t *p = pga_init_device(-1);
  assert(p);
  pga_set_seed(p, seed);
  pga_set_quiet(p, 1);
  pga_set_abort_on_error(p, 0);
  return p;
}

static float sum(const gene *g, unsigned n) {
  float s = 0.f;
  for (unsigned i = 0; i < n; ++i) s += g[i];
  return s;
}

int main(int argc, char **argv) {
  const char *ckpt = argc > 1 ? argv[1] : "/tmp/pga_capi_cpu.ckpt";
  /* limits: L < 4 and MAX_POPULATIONS */
  pga_t *p = solver(1);
  assert(!pga_create_population(p, 100, 3, RANDOM_POPULATION));
  for (int i = 0; i < MAX_POPULATIONS; ++i) assert(pga_create_population(p, 10, 8, RANDOM_POPULATION));
  assert(!pga_create_population(p, 10, 8, RANDOM_POPULATION));
  pga_deinit(p);

  /* E2 knapsack with the built-in objective */
  p = solver(3);
  population_t *pop = pga_create_population(p, 100, 6, RANDOM_POPULATION);
  const float kd[12] = {75, 150, 250, 35, 10, 100, 7, 8, 6, 4, 3, 9};
  assert(pga_set_objective_builtin(p, pop, PGA_OBJ_KNAPSACK_REAL, kd, 12, NULL, 0, 2, 10.f, 0.f) == 0);
  pga_run(p, 5);
  gene *g = pga_get_best(p, pop);
  assert(g && pga_best_score(p, pop) == 285.f);
  free(g);
  pga_deinit(p);

  /* staged API + queries */
  p = solver(5);
  pop = pga_create_population(p, 300, 20, RANDOM_POPULATION);
  pga_set_objective_builtin(p, pop, PGA_OBJ_LINEAR, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  pga_evaluate(p, pop);
  const float s0 = pga_best_score(p, pop);
  for (int i = 0; i < 10; ++i) {
    pga_fill_random_values(p, pop);
    pga_evaluate(p, pop);
    pga_crossover(p, pop, TOURNAMENT);
    pga_mutate(p, pop);
    pga_swap_generations(p, pop);
  }
  pga_evaluate(p, pop);
  assert(pga_generation(pop) == 10 && pga_best_score(p, pop) > s0);
  float *sc = malloc(300 * sizeof(float)), st[4];
  assert(pga_get_scores(p, pop, sc) == 0 && pga_stats(p, pop, st) == 0);
  float mx = -INFINITY;
  for (int i = 0; i < 300; ++i) mx = sc[i] > mx ? sc[i] : mx;
  assert(st[1] == mx && mx == pga_best_score(p, pop));
  gene **top = pga_get_best_top(p, pop, 5);
  for (int i = 1; i < 5; ++i) assert(sum(top[i - 1], 20) >= sum(top[i], 20) - 1e-4f);
  for (int i = 0; i < 5; ++i) free(top[i]);
  free(top);
  free(sc);
  pga_deinit(p);

  /* islands and migration */
  p = solver(7);
  population_t *pops[4];
  for (int i = 0; i < 4; ++i) {
    pops[i] = pga_create_population(p, 200, 16, RANDOM_POPULATION);
    pga_set_objective_builtin(p, pops[i], PGA_OBJ_LINEAR, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  }
  pga_evaluate_all(p);
  pga_crossover_all(p, TOURNAMENT);
  pga_mutate_all(p);
  for (int i = 0; i < 4; ++i) pga_swap_generations(p, pops[i]);
  pga_evaluate_all(p);
  pga_migrate_between(p, pops[0], pops[1], 0.05f);
  pga_run_islands(p, 30, 5, 10.f);
  pga_migrate(p, 0.1f);
  gene *b = pga_get_best_all(p);
  float best = -INFINITY;
  for (int i = 0; i < 4; ++i) best = fmaxf(best, pga_best_score(p, pops[i]));
  assert(fabsf(sum(b, 16) - best) < 1e-3f);
  free(b);
  gene **tops = pga_get_best_top_all(p, 3);
  for (int i = 0; i < 3; ++i) free(tops[i]);
  free(tops);
  pga_deinit(p);

  /* encodings, operators, checkpoint */
  p = solver(11);
  pop = pga_create_population_ext(p, 512, 64, PGA_BINARY);
  pga_set_objective_builtin(p, pop, PGA_OBJ_ONEMAX, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  pga_set_operators(p, pop, PGA_SEL_TOURNAMENT, 2, PGA_XO_TWO_POINT, 1.f, PGA_MUT_BIT_FLIP, -1.f, 0.f, 1);
  pga_run(p, 5);
  assert(pga_save(p, pop, ckpt) == 0);
  pga_run(p, 30);
  assert(pga_best_score(p, pop) == 64.f);
  population_t *perm = pga_create_population_ext(p, 256, 16, PGA_PERMUTATION);
  float d[256];
  for (int i = 0; i < 256; ++i) d[i] = (float)((i * 37) % 17 + 1);
  assert(pga_set_objective_builtin(p, perm, PGA_OBJ_TSP, d, 256, NULL, 0, 0, 0.f, 0.f) == 0);
  pga_set_operators(p, perm, PGA_SEL_TOURNAMENT, 4, PGA_XO_OX, 1.f, PGA_MUT_INVERSION, 0.3f, 0.f, 1);
  pga_run_islands(p, 10, 0, 0.f);
  pga_t *q = solver(11);
  population_t *pop2 = pga_create_population_ext(q, 512, 64, PGA_BINARY);
  pga_set_objective_builtin(q, pop2, PGA_OBJ_ONEMAX, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  assert(pga_load(q, pop2, ckpt) == 0 && pga_generation(pop2) == 5);
  /* errors are recorded, not fatal, with abort off */
  assert(pga_load(q, pop2, "/nonexistent/pga.ckpt") == -1 && strlen(pga_last_error()) > 0);
  pga_deinit(p);
  pga_deinit(q);
  printf("capi_cpu ok\n");
  return 0;
}
