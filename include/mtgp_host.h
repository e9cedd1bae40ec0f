/* mtgp_host.h -- C ABI of the native host library (libmtgp_host.so): the evolution step between
 * two evaluations, so a generation's host work stays far below the GPU evaluation's time.
 *
 * Replaces GeneticProgramming.evolve / initialize_population (MultiTreeGP
 * genetic_programming.py:298-308, 475-525 with genetic_operators/{initialization,mutation,
 * crossover,reproduction}.py).  Trees use the reference's [max_nodes, 4] float32 layout
 * [f, a, b, value] (empty rows low, root at row N-1); a population array is
 * [num_pop, pop_size, num_trees, N, 4] contiguous.
 *
 * Draws come from per-(population, pair) xoshiro256** streams derived from `seed`: results are
 * reproducible for a seed and independent of the thread count, and distributed like the
 * reference's (which splits JAX keys per operation), not draw-for-draw equal to it.
 */
#ifndef MTGP_HOST_H
#define MTGP_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTGP_HOST_ABI_VERSION 1

typedef struct MtgpEvolveConfig {
  /* node library (node_library.NodeLibrary / gp.py:123-190) */
  int32_t n_funcs;        /* entries of slots[] (every index a tree row can hold) */
  const int32_t* slots;   /* operand count per index (0 empty, 1 coefficient) */
  int32_t n_ops;          /* operators: op_index[n_ops], sampled with op_prob[n_ops] */
  const int32_t* op_index;
  const double* op_prob;
  int32_t var_start;      /* variables: var_start .. var_start + n_vars - 1 */
  int32_t n_vars;
  const float* var_mask;  /* [num_trees, n_vars]: variables allowed per tree (variable_array) */
  /* strategy (gp.py:61-121) */
  int32_t max_init_depth;
  float coefficient_sd;
  int32_t current_generation;
  int32_t migration_period;
  int32_t migration_size;
  int32_t tournament_size;
  int32_t elite_size;
  const double* tournament_prob;        /* [num_pop, tournament_size] */
  const double* reproduction_type_prob; /* [num_pop, 3]: crossover, mutation, resampling */
  const double* reproduction_prob;      /* [num_pop]: per-tree Bernoulli rate of the operators */
} MtgpEvolveConfig;

int mtgp_host_abi_version(void);

/* One generation (gp.py:475-497): ring migration when num_pop > 1 and
 * (current_generation + 1) % migration_period == 0, then per population the elite_size best
 * (stable sort) followed by (pop_size - elite_size) / 2 pairs of tournament winners reproduced by
 * crossover / mutation / resampling -- first children of every pair, then second children.
 * `out` holds [num_pop, E + 2 * pairs, num_trees, N, 4].  Returns the output population size, or
 * -1 on invalid arguments. */
int mtgp_evolve_populations(const float* populations, const float* fitness, int32_t num_pop, int32_t pop_size,
                            int32_t num_trees, int32_t N, const MtgpEvolveConfig* cfg, uint64_t seed, float* out);

/* initialize_population (gp.py:298-308): [num_pop, pop_size, num_trees, N, 4] fresh trees of
 * max_init_depth.  Returns 0, or -1 on invalid arguments. */
int mtgp_sample_population(int32_t num_pop, int32_t pop_size, int32_t num_trees, int32_t N,
                           const MtgpEvolveConfig* cfg, uint64_t seed, float* out);

#ifdef __cplusplus
}
#endif

#endif /* MTGP_HOST_H */
