/*
 * pga.h — C API of the MI355X-native parallel genetic-algorithm engine.
 *
 * Source-compatible with the pbalcer/libpga interface (same types, enums,
 * callback signatures and the same 22 entry points), backed
 * by the gfx950 engine (csrc/engine/island.cpp, csrc/kernels/).  Every entry
 * point is implemented — including the ones the original leaves as stubs
 * (pga_get_best_top*, pga_get_best_all, pga_migrate*, pga_run_islands).
 *
 * Semantics worth knowing:
 *   - genes are float, initialised U(0, 1]; a population holds two
 *     generations (current / next) that pga_swap_generations exchanges;
 *   - the objective is MAXIMISED; user callbacks are __device__ function
 *     pointers fetched with hipMemcpyFromSymbol (link with libpga.a and
 *     -fgpu-rdc); NULL mutate/crossover restore the built-in defaults;
 *   - pga_run(p, n) evolves population 0 for n generations (fused
 *     select + crossover + mutate + evaluate kernel); pga_run_islands evolves
 *     every population and migrates between them;
 *   - calls are stream-ordered on one HIP stream per pga_t; only the
 *     pga_get_best* queries synchronise.
 * Extensions (seeds, encodings, operators, built-in objectives, multi-GPU
 * islands over RCCL, checkpoints): pga_ext.h.
 */
#ifndef PGA_H
#define PGA_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pga_solver pga_t;  /* tag differs from the original: "pga" is the C++ namespace */
typedef struct pga_population population_t;

typedef float gene;

enum population_type {
  RANDOM_POPULATION,
  MAX_POPULATION_TYPE
};

/* selection used by pga_crossover (tournament of size 2 unless changed via pga_ext.h) */
enum crossover_selection_type {
  TOURNAMENT,
  MAX_SELECTION_TYPE
};

#define MAX_POPULATIONS 10

/* device callbacks */
typedef float (*obj_f)(gene *genome, unsigned length);
typedef void (*mutate_f)(gene *genome, float *rand, unsigned length);
typedef void (*crossover_f)(gene *parent1, gene *parent2, gene *child, float *rand, unsigned length);

/* solver lifetime */
pga_t *pga_init(void);
void pga_deinit(pga_t *p);

/* NULL when MAX_POPULATIONS already exist or genome_len < 4 */
population_t *pga_create_population(pga_t *p, unsigned long size, unsigned genome_len, enum population_type type);

/* callbacks (device function pointers) */
void pga_set_objective_function(pga_t *p, obj_f f);
void pga_set_mutate_function(pga_t *p, mutate_f f);      /* NULL -> default: 1% single-gene reset */
void pga_set_crossover_function(pga_t *p, crossover_f f); /* NULL -> default: uniform */

/* results: host copies the caller frees with free(); pga_get_best prints the best score */
gene *pga_get_best(pga_t *p, population_t *pop);
gene **pga_get_best_top(pga_t *p, population_t *pop, unsigned length);
gene *pga_get_best_all(pga_t *p);
gene **pga_get_best_top_all(pga_t *p, unsigned length);

/* stages */
void pga_evaluate(pga_t *p, population_t *pop);
void pga_evaluate_all(pga_t *p);
void pga_crossover(pga_t *p, population_t *pop, enum crossover_selection_type type);
void pga_crossover_all(pga_t *p, enum crossover_selection_type type);
void pga_mutate(pga_t *p, population_t *pop);
void pga_mutate_all(pga_t *p);
void pga_swap_generations(pga_t *p, population_t *pop);
void pga_fill_random_values(pga_t *p, population_t *pop);

/* islands: the best pct (fraction or percent) of a population replaces the worst of another */
void pga_migrate(pga_t *p, float pct);
void pga_migrate_between(pga_t *p, population_t *from, population_t *to, float pct);

/* drivers */
void pga_run(pga_t *p, unsigned n);
void pga_run_islands(pga_t *p, unsigned n, unsigned m, float pct);

#ifdef __cplusplus
}
#endif

#endif /* PGA_H */
