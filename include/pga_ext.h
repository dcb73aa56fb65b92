/*
 * pga_ext.h — extensions of the pga.h C API (not in the original library).
 *
 * Enum values mirror csrc/include/pga/core.hpp exactly.
 */
#ifndef PGA_EXT_H
#define PGA_EXT_H

#include <stddef.h>
#include <stdint.h>

#include "pga.h"

#ifdef __cplusplus
extern "C" {
#endif

enum pga_encoding { PGA_BINARY = 0, PGA_REAL = 1, PGA_PERMUTATION = 2 };
enum pga_selection { PGA_SEL_TOURNAMENT = 0, PGA_SEL_ROULETTE = 1, PGA_SEL_RANDOM = 2, PGA_SEL_RANK = 3 };
enum pga_crossover {
  PGA_XO_UNIFORM = 0, PGA_XO_ONE_POINT = 1, PGA_XO_TWO_POINT = 2, PGA_XO_BLEND = 3,
  PGA_XO_ARITHMETIC = 4, PGA_XO_PMX = 5, PGA_XO_OX = 6, PGA_XO_NONE = 7
};
enum pga_mutation {
  PGA_MUT_BIT_FLIP = 0, PGA_MUT_GAUSSIAN = 1, PGA_MUT_UNIFORM = 2, PGA_MUT_RESET_ONE = 3,
  PGA_MUT_SWAP = 4, PGA_MUT_INVERSION = 5, PGA_MUT_NONE = 6
};
enum pga_objective {
  PGA_OBJ_NONE = 0, PGA_OBJ_ONEMAX = 1, PGA_OBJ_KNAPSACK = 2, PGA_OBJ_TRAP = 3, PGA_OBJ_LEADING_ONES = 4,
  PGA_OBJ_QUBO = 5, /* BINARY, data = L*L integer Q in [-128,127], fparam0 = sign (+1 max x^TQx, -1 min) */
  PGA_OBJ_SPHERE = 16, PGA_OBJ_RASTRIGIN = 17, PGA_OBJ_ROSENBROCK = 18, PGA_OBJ_ACKLEY = 19,
  PGA_OBJ_GRIEWANK = 20, PGA_OBJ_SCHWEFEL = 21, PGA_OBJ_LINEAR = 22, PGA_OBJ_KNAPSACK_REAL = 23,
  PGA_OBJ_TSP_RANDOM_KEY = 24, PGA_OBJ_TSP = 32, PGA_OBJ_TSP_OPEN = 33, PGA_OBJ_TSP_EUC = 34,
  PGA_OBJ_USER_FNPTR = 64
};

/* ---- solver options (call before creating populations) ---- */
pga_t *pga_init_device(int device);            /* device < 0: CPU reference backend */
int pga_device_count(void);                      /* visible GPUs (0 without a GPU) */
void pga_set_seed(pga_t *p, uint64_t seed);      /* default: PGA_SEED env or time(NULL) */
void pga_set_quiet(pga_t *p, int quiet);         /* 1: pga_get_best does not print */
/* 1 (default, reference behaviour): print the error and exit; 0: record it and return */
void pga_set_abort_on_error(pga_t *p, int abort_on_error);
const char *pga_last_error(void);                /* thread-local, "" when none */

/* ---- populations of any encoding ---- */
population_t *pga_create_population_ext(pga_t *p, unsigned long size, unsigned genome_len,
                                        enum pga_encoding encoding);
/* built-in fused objective; data / data2 are host arrays copied to the device */
int pga_set_objective_builtin(pga_t *p, population_t *pop, enum pga_objective objective, const float *data,
                              size_t n, const float *data2, size_t n2, int iparam, float fparam0, float fparam1);
/* objective from HIP source compiled at runtime for gfx950 (hipRTC): `name` is a
 *   __device__ float name(const T *row, unsigned int n, const float *data)
 * with T = unsigned int (BINARY words), float (REAL), unsigned short (PERMUTATION);
 * data: n floats copied to the device (may be NULL).  GPU only.  On a compile
 * error: -1 and the compiler log in pga_last_error() (when abort is off). */
int pga_set_objective_source(pga_t *p, population_t *pop, const char *source, const char *name, const float *data,
                             size_t n);
int pga_set_operators(pga_t *p, population_t *pop, enum pga_selection selection, unsigned tournament_k,
                      enum pga_crossover crossover, float crossover_prob, enum pga_mutation mutation,
                      float mutation_rate /* < 0: default */, float sigma, unsigned elitism);
int pga_set_bounds(pga_t *p, population_t *pop, float lo, float hi);
int pga_set_blend_alpha(pga_t *p, population_t *pop, float alpha);
/* PGA_SEL_RANK: linear ranking pressure sp in [1, 2] (expected copies of the best; default 1.5) */
int pga_set_rank_pressure(pga_t *p, population_t *pop, float sp);

/* ---- queries ---- */
unsigned long pga_population_size(const population_t *pop);
unsigned pga_genome_length(const population_t *pop);
unsigned pga_generation(const population_t *pop);
float pga_best_score(pga_t *p, population_t *pop);
unsigned long pga_best_index(pga_t *p, population_t *pop);
int pga_get_scores(pga_t *p, population_t *pop, float *out);             /* S floats */
int pga_get_genome(pga_t *p, population_t *pop, unsigned long i, void *out); /* raw row (row bytes) */
size_t pga_row_bytes(const population_t *pop);
int pga_stats(pga_t *p, population_t *pop, float out[4]);                /* min, max, sum, count */
/* Per-generation history of {min, max, sum, count}: on != 0 clears and starts
 * recording (each generation appends one row from its kernel's fused
 * partials, stream-ordered); pga_get_stats_history copies up to max_rows rows
 * (4 floats each) and returns the number recorded (-1 on error). */
int pga_set_stats_history(pga_t *p, population_t *pop, int on);
long pga_get_stats_history(pga_t *p, population_t *pop, float *out, unsigned long max_rows);
int pga_synchronize(pga_t *p);

/* ---- checkpoint / resume (exact: the generation counter is the RNG state) ---- */
int pga_save(pga_t *p, population_t *pop, const char *path);
int pga_load(pga_t *p, population_t *pop, const char *path);

/* ---- inter-rank island model ----
 * Population 0 of every rank takes part; every m generations of
 * pga_run_islands each rank exports its top pct% and replaces its worst
 * pct% with what it receives (after re-scoring it with its own objective).
 *
 * Transports:
 *  - RCCL, one process per GPU: rank 0 creates an id (128 bytes) with
 *    pga_comm_unique_id and shares it (file, env, MPI, ...); every rank calls
 *    pga_comm_init and then pga_run_islands.
 *  - RCCL, one process driving n GPUs: pga_comm_init_local(solvers, n) over
 *    solvers created with pga_init_device(0..n-1), then
 *    pga_run_islands_multi(solvers, n, ...).
 *  - loopback: pga_comm_init_loopback(solvers, n), in-process copies between
 *    any solvers (CPU or GPU): tests, and fault injection. */
enum pga_topology {
  PGA_TOPO_RING = 0,       /* rank r -> r+1 (one xGMI link per direction) */
  PGA_TOPO_RANDOM = 1,     /* a fresh random ring per epoch, from the shared seed */
  PGA_TOPO_ALL_TO_ALL = 2  /* k/(n-1) emigrants to every other rank (all links) */
};
struct pga_comm_stats {
  uint64_t epochs, failures, migrants_received, bytes_sent;
  int degraded;
};
int pga_comm_unique_id(char id[128]);
int pga_comm_init(pga_t *p, int nranks, int rank, const char id[128]);
int pga_comm_init_local(pga_t **solvers, int n);
int pga_comm_init_loopback(pga_t **solvers, int n);
int pga_comm_rank(const pga_t *p);
int pga_comm_size(const pga_t *p);
int pga_comm_set_topology(pga_t *p, enum pga_topology t); /* applies to the whole local group */
/* Emigrant / victim choice of every migration of `pop` (pga_migrate*,
 * pga_run_islands*, inter-rank epochs).  TOPK (default, the "top pct%" of
 * the reference's pga_migrate / pga_run_islands, include/pga.h): the exact
 * top-k emigrate and the bottom-k are replaced.  STRIPE (opt-in, cheaper):
 * the population is cut into k contiguous stripes; stripe i's best emigrates
 * and its worst is replaced by immigrant i — one pass over the scores each
 * way, and the global best still always emigrates. */
enum pga_migration_policy { PGA_MIGRATE_TOPK = 0, PGA_MIGRATE_STRIPE = 1 };
int pga_set_migration_policy(pga_t *p, population_t *pop, enum pga_migration_policy policy);
/* > 0: every collective of the island model is bounded by `seconds` on the
 * host (RCCL: event polling + async error check): the migration exchange
 * (polled only after the next generation is queued, so it still overlaps
 * compute), the all-gathers of the global best / target checks and the
 * best-genome broadcast.  A failed or late collective aborts the
 * communicator at once; the islands continue alone (degraded) and queries
 * fall back to the local best.  0 (default): exchanges fully asynchronous
 * (errors are only checked), collectives block until done. */
int pga_comm_set_timeout(pga_t *p, double seconds);
int pga_comm_set_validation(pga_t *p, int on);             /* re-score received migrants (default 1) */
int pga_comm_degraded(const pga_t *p);
int pga_comm_info(const pga_t *p, struct pga_comm_stats *out);
/* tests: every `every`-th exchange is dropped (mode 1, loopback), arrives
 * with forged scores (mode 2, loopback) or has this rank's sends withheld so
 * its receives never complete (mode 3, RCCL: exercises the timeout + abort
 * path); mode 4 (RCCL) stalls every `every`-th all-gather behind a receive
 * that never completes (a peer lost between two check points); mode 0
 * disarms it. */
int pga_comm_set_fault(pga_t *p, int every, int mode);
/* tests: let a 1-rank communicator exchange with itself (normally migration
 * is skipped at one rank), so the real transport runs on one GPU */
int pga_comm_set_self_exchange(pga_t *p, int on);
/* one inter-rank migration epoch now, serially (exchange, wait, immigrate;
 * pga_run_islands overlaps it with the next generation instead), for callers
 * driving their own generation loop; pass every rank of an InitAll /
 * loopback group, or the one solver of an InitRank rank */
int pga_comm_exchange(pga_t **solvers, int count, float pct);
/* global best over ranks: score and owning rank (ties: the lowest rank), an
 * all-gather of (score, index) of every rank's population 0 */
int pga_comm_best(pga_t *p, float *score, int *rank);
/* the same plus the winning genome: its raw row (pga_row_bytes bytes,
 * pga_get_genome layout) is broadcast from the owning rank and copied to
 * row_out on every rank (row_out may be NULL).  Every rank must call it. */
int pga_comm_get_best(pga_t *p, float *score, int *rank, void *row_out);
/* pga_run_islands over every rank of an InitAll / loopback group at once */
int pga_run_islands_multi(pga_t **solvers, int n, unsigned generations, unsigned m, float pct);

/* ---- target-fitness termination ("until n generations or obj(best) ==
 * value", include/pga.h of the reference) ----
 * pga_run_until: pga_run, stopping once population 0's best score >= target;
 * the best is read every check_every generations (0: 10), so there is one
 * stream sync per check, none per generation.  Returns the generations run
 * (-1 on error).
 * pga_run_islands_until: pga_run_islands, checked at every migration point
 * (every m generations; every 10 when m == 0) against the best over all
 * populations and, with a communicator, over all ranks (an all-gather, so
 * every rank stops at the same generation).  Returns the generations run. */
int pga_run_until(pga_t *p, unsigned generations, float target, unsigned check_every);
int pga_run_islands_until(pga_t *p, unsigned generations, unsigned m, float pct, float target);
/* the same over every rank of an InitAll / loopback group at once */
int pga_run_islands_multi_until(pga_t **solvers, int n, unsigned generations, unsigned m, float pct, float target);

/* ---- batched islands ----
 * pga_run_islands / pga_run_islands_until run the populations of one solver
 * as ONE kernel launch per generation (island = grid y) when they qualify:
 * two to ten BINARY populations of the same size and length with a built-in
 * integer objective (OneMax, LeadingOnes, Trap) and the hot kernel's
 * operators; otherwise each population runs on its own stream.  On by
 * default; pga_batched_generations counts the generations run batched. */
int pga_set_batch_islands(pga_t *p, int on);
unsigned long long pga_batched_generations(const pga_t *p);

#ifdef __cplusplus
}
#endif

#endif /* PGA_EXT_H */
