/* islands_multiproc.c — plain C island model, ONE PROCESS PER GPU: the
 * MPI-free replacement of the reference's "GPUs+MPI" claim (README.md:4).
 * Rank 0 creates the RCCL unique id and publishes it through a file; every
 * rank reads it, joins with ncclCommInitRank (pga_comm_init) on GPU
 * rank % device_count, and runs pga_run_islands: top 1% every 10
 * generations over xGMI, with a host-side exchange timeout so a dead peer
 * degrades the run instead of hanging it.
 *
 *   islands_multiproc <rank> <nranks> <id_file> [pop] [generations]
 *   (start all ranks, e.g. for r in 0 1 2 3; do islands_multiproc $r 4 /tmp/id & done)
 *
 * Prints one line per rank: rank, generations, best score, migration stats. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "pga_ext.h"

static int publish_id(const char* path, const char id[128]) {
  char tmp[4096];
  snprintf(tmp, sizeof tmp, "%s.tmp", path);
  FILE* f = fopen(tmp, "wb");
  if (!f || fwrite(id, 1, 128, f) != 128) return -1;
  fclose(f);
  return rename(tmp, path); /* atomic: readers never see a partial id */
}

static int read_id(const char* path, char id[128], double timeout_s) {
  const time_t t0 = time(NULL);
  for (;;) {
    FILE* f = fopen(path, "rb");
    if (f) {
      const size_t n = fread(id, 1, 128, f);
      fclose(f);
      if (n == 128) return 0;
    }
    if (difftime(time(NULL), t0) > timeout_s) return -1;
    usleep(10000);
  }
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <rank> <nranks> <id_file> [pop] [generations]\n", argv[0]);
    return 2;
  }
  const int rank = atoi(argv[1]), nranks = atoi(argv[2]);
  const char* id_file = argv[3];
  const unsigned long pop_size = argc > 4 ? strtoul(argv[4], NULL, 10) : (1ul << 18);
  const unsigned gens = argc > 5 ? (unsigned)atoi(argv[5]) : 100;
  const int ndev = pga_device_count();
  if (ndev < 1 || rank < 0 || rank >= nranks) {
    fprintf(stderr, "rank %d: no GPU or bad rank\n", rank);
    return 1;
  }
  char id[128];
  if (rank == 0) {
    if (pga_comm_unique_id(id) != 0 || publish_id(id_file, id) != 0) {
      fprintf(stderr, "rank 0: cannot create / publish the communicator id\n");
      return 1;
    }
  } else if (read_id(id_file, id, 60.0) != 0) {
    fprintf(stderr, "rank %d: no communicator id in %s\n", rank, id_file);
    return 1;
  }
  pga_t* p = pga_init_device(rank % ndev);
  if (!p) return 1;
  pga_set_seed(p, 1000 + (uint64_t)rank);
  pga_set_quiet(p, 1);
  pga_set_abort_on_error(p, 0);
  population_t* pop = pga_create_population_ext(p, pop_size, 1024, PGA_BINARY);
  if (!pop) return 1;
  pga_set_objective_builtin(p, pop, PGA_OBJ_ONEMAX, NULL, 0, NULL, 0, 0, 0.f, 0.f);
  pga_set_operators(p, pop, PGA_SEL_TOURNAMENT, 2, PGA_XO_UNIFORM, 1.f, PGA_MUT_BIT_FLIP, -1.f, 0.f, 1);
  if (pga_comm_init(p, nranks, rank, id) != 0) {
    fprintf(stderr, "rank %d: pga_comm_init: %s\n", rank, pga_last_error());
    return 1;
  }
  pga_comm_set_timeout(p, 30.0);
  pga_run_islands(p, gens, 10, 0.01f);
  struct pga_comm_stats st;
  pga_comm_info(p, &st);
  float best = 0.f;
  int owner = 0;
  if (!st.degraded) pga_comm_best(p, &best, &owner);
  else best = pga_best_score(p, pop);
  printf("rank %d/%d generations %u best %.0f (rank %d) epochs %llu received %llu degraded %d\n", rank, nranks,
         pga_generation(pop), best, owner, (unsigned long long)st.epochs, (unsigned long long)st.migrants_received,
         st.degraded);
  pga_deinit(p);
  return st.degraded ? 3 : 0;
}
