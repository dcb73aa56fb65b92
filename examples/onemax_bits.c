/* onemax_bits.c — plain C (no HIP in user code) through pga_ext.h: the
 * headline configuration, bit-packed OneMax with 1024-bit genomes and a
 * population of 2^20 on one GPU, with a built-in fused objective. */
#include <stdio.h>
#include <stdlib.h>

#include "pga_ext.h"

int main(int argc, char** argv) {
  const unsigned long pop_size = argc > 1 ? strtoul(argv[1], NULL, 10) : (1ul << 20);
  const unsigned gens = argc > 2 ? (unsigned)atoi(argv[2]) : 200;
  pga_t* p = pga_init();
  if (!p) return 1;
  pga_set_seed(p, 42);
  pga_set_quiet(p, 1);
  population_t* pop = pga_create_population_ext(p, pop_size, 1024, PGA_BINARY);
  pga_set_objective_builtin(p, pop, PGA_OBJ_ONEMAX, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  pga_set_operators(p, pop, PGA_SEL_TOURNAMENT, 2, PGA_XO_UNIFORM, 1.f, PGA_MUT_BIT_FLIP, -1.f, 0.f, 1);
  pga_run(p, gens);
  float st[4];
  pga_stats(p, pop, st);
  printf("onemax-1024 pop %lu after %u generations: best %.0f mean %.2f\n", pop_size, gens,
         pga_best_score(p, pop), st[2] / st[3]);
  pga_deinit(p);
  return 0;
}
