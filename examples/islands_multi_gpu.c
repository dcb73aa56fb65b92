/* islands_multi_gpu.c — plain C island model over every visible GPU from ONE
 * process: one solver per GPU (pga_init_device), RCCL communicators from
 * ncclCommInitAll (pga_comm_init_local), migration of the top 1% every 10
 * generations around a ring over xGMI (or all-to-all / random rings).
 *
 *   islands_multi_gpu [pop_per_gpu] [generations] [ring|random|all_to_all]
 *
 * The reference declares pga_run_islands but leaves it empty
 * (src/pga.cu:393-395) and has no multi-GPU code (README.md:4). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pga_ext.h"

int main(int argc, char** argv) {
  const unsigned long pop_size = argc > 1 ? strtoul(argv[1], NULL, 10) : (1ul << 18);
  const unsigned gens = argc > 2 ? (unsigned)atoi(argv[2]) : 100;
  enum pga_topology topo = PGA_TOPO_RING;
  if (argc > 3 && !strcmp(argv[3], "random")) topo = PGA_TOPO_RANDOM;
  if (argc > 3 && !strcmp(argv[3], "all_to_all")) topo = PGA_TOPO_ALL_TO_ALL;
  int n = pga_device_count();
  if (n < 1) {
    fprintf(stderr, "no GPU\n");
    return 1;
  }
  if (n > 8) n = 8;
  pga_t* s[8];
  population_t* pop[8];
  for (int i = 0; i < n; ++i) {
    s[i] = pga_init_device(i);
    if (!s[i]) return 1;
    pga_set_seed(s[i], 1000 + i);
    pga_set_quiet(s[i], 1);
    pop[i] = pga_create_population_ext(s[i], pop_size, 1024, PGA_BINARY);
    pga_set_objective_builtin(s[i], pop[i], PGA_OBJ_ONEMAX, NULL, 0, NULL, 0, 0, 0.f, 0.f);
    pga_set_operators(s[i], pop[i], PGA_SEL_TOURNAMENT, 2, PGA_XO_UNIFORM, 1.f, PGA_MUT_BIT_FLIP, -1.f, 0.f, 1);
  }
  if (pga_comm_init_local(s, n) != 0) {
    fprintf(stderr, "pga_comm_init_local: %s\n", pga_last_error());
    return 1;
  }
  pga_comm_set_topology(s[0], topo);
  pga_comm_set_timeout(s[0], 60.0);
  if (pga_run_islands_multi(s, n, gens, 10, 0.01f) != 0) {
    fprintf(stderr, "pga_run_islands_multi: %s\n", pga_last_error());
    return 1;
  }
  float best = 0.f;
  int owner = 0;
  pga_comm_best(s[0], &best, &owner);
  struct pga_comm_stats st;
  pga_comm_info(s[0], &st);
  printf("%d GPU islands x pop %lu, %u generations: best %.0f (rank %d), %llu migration epochs, %llu bytes sent%s\n",
         n, pop_size, gens, best, owner, (unsigned long long)st.epochs, (unsigned long long)st.bytes_sent,
         st.degraded ? " (degraded)" : "");
  for (int i = 0; i < n; ++i) pga_deinit(s[i]);
  return best > 0.f ? 0 : 1;
}
