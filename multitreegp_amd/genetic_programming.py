"""GeneticProgramming facade: the reference strategy's evaluation half on MI355X.

Keeps the constructor signature, validation and bookkeeping of
MultiTreeGP/genetic_programming.py:GeneticProgramming (gp.py:61-270, 403-433, 527-537) and
replaces ``evaluate_population``'s ``jit(shard_map(vmap(fitness_function)))`` with the flatten
+ fused RK4 / Dopri5 HIP kernels.  ``evolve`` runs the host restatement of genetic_operators/
(multitreegp_amd.genetic_operators), so whole generations run on the GPU box; a maintainer who
keeps the reference's JAX evolution swaps only ``evaluate_population``.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from . import distributed as mdist
from .engine import DeviceEngine
from .coefficients import CoefficientOptimiser, adam
from .genetic_operators import Operators, evolve_populations
from .node_library import NodeLibrary
from .sampling import sample_population


def _seed_of(key) -> int:
    """numpy seed from a JAX-style key (uint32 words) or an int."""
    if isinstance(key, (int, np.integer)):
        return int(key)
    words = np.asarray(key, np.uint64).reshape(-1)
    return int(sum(int(w) << (32 * i) for i, w in enumerate(words[::-1])))


class TreeEvaluator:
    """Counterpart of ``GeneticProgramming.vmap_foriloop`` (gp.py:390-401).

    Passed to the evaluators as ``tree_evaluator`` like in the reference; it carries the node
    library, and calling it evaluates every tree of a candidate on one data vector on the GPU."""

    def __init__(self, library: NodeLibrary, max_nodes: int, device=None):
        self.library = library
        self.max_nodes = max_nodes
        self.device = device
        self._engines = {}
        self._tree_only = {}

    def engine(self, fitness_function, size_parsinomy: float = 0.0) -> DeviceEngine:
        key = (id(fitness_function), float(size_parsinomy))
        if key not in self._engines:
            self._engines[key] = DeviceEngine(fitness_function, self.library, size_parsinomy, self.device)
        return self._engines[key]

    def __call__(self, candidate, data) -> np.ndarray:
        from .evaluators import _TreeOnly
        cand = np.asarray(candidate, dtype=np.float32)
        d = np.asarray(data, dtype=np.float32).reshape(1, -1)
        shape = (cand.shape[0], d.shape[1])
        ff = self._tree_only.get(shape)
        if ff is None:  # one pseudo fitness config (hence one engine) per (trees, data) shape
            ff = self._tree_only[shape] = _TreeOnly(*shape)
        eng = self.engine(ff)
        pop = torch.from_numpy(cand[None]).to(eng.device)
        eng.prepare_data(None)
        fl = eng.flatten(pop)
        eng.check_status(fl)
        out = eng.eval_programs(fl, torch.from_numpy(d).to(eng.device))
        return out[0, :, 0].cpu().numpy()


class GeneticProgramming:
    """Genetic programming strategy (evaluation side).  Parameters as gp.py:61-84."""

    def __init__(self, num_generations: int, population_size: int, fitness_function, operator_list,
                 variable_list, layer_sizes, num_populations: int = 1, max_init_depth: int = 4,
                 max_nodes: int = 30, device_type: str = "gpu", tournament_size: int = 7,
                 size_parsinomy: float = 0.0, coefficient_sd: float = 1.0, migration_period: int = 10,
                 migration_percentage: float = 0.1, elite_percentage: float = 0.1,
                 coefficient_optimisation: bool = False, gradient_steps: int = 10, optimiser=None,
                 selection_pressure_factors=(0.6, 0.9), reproduction_probability_factors=(1.0, 0.5),
                 crossover_probability_factors=(0.9, 0.4), mutation_probability_factors=(0.1, 0.5),
                 sample_probability_factors=(0.0, 0.1), device=None, verbose: bool = True,
                 evolve_backend: str = "native"):
        self.layer_sizes = np.asarray(layer_sizes)
        assert num_populations > 0, "The number of populations should be larger than 0"
        self.num_populations = num_populations
        assert population_size > 0 and population_size % 2 == 0, \
            "The population_size should be larger than 0 and an even number"
        self.population_size = population_size
        assert max_init_depth > 0, "The max initial depth should be larger than 0"
        self.max_init_depth = max_init_depth
        assert max_nodes > 0, "The max number of nodes should be larger than 0"
        self.max_nodes = max_nodes
        self.num_trees = int(np.sum(self.layer_sizes))
        assert self.num_trees > 0, "The number of trees should be larger than 0"
        self.current_generation = 0
        assert num_generations > 0, "The number of generations should be larger than 0"
        self.num_generations = num_generations
        self.best_fitnesses = np.zeros(num_generations, dtype=np.float32)
        self.best_solutions = np.zeros((num_generations, self.num_trees, max_nodes, 4), dtype=np.float32)
        self.size_parsinomy = size_parsinomy
        self.coefficient_sd = coefficient_sd
        assert migration_period > 1, "The migration period should be larger than 1"
        self.migration_period = migration_period
        assert migration_percentage * population_size % 1 == 0, "The migration size should be an integer"
        self.migration_size = int(migration_percentage * population_size)
        assert tournament_size > 1, "The number of gradient steps should be larger than 1"
        self.tournament_size = tournament_size
        # per-population schedules, linearly spaced over the populations (gp.py:113-121)
        self.selection_pressures = np.linspace(*selection_pressure_factors, num_populations)
        self.tournament_probabilities = np.array([sp * (1 - sp) ** np.arange(tournament_size)
                                                  for sp in self.selection_pressures])
        self.reproduction_type_probabilities = np.vstack([np.linspace(*crossover_probability_factors, num_populations),
                                                          np.linspace(*mutation_probability_factors, num_populations),
                                                          np.linspace(*sample_probability_factors, num_populations)]).T
        self.reproduction_probabilities = np.linspace(*reproduction_probability_factors, num_populations)
        self.elite_size = int(elite_percentage * population_size)
        assert self.elite_size % 2 == 0, "The elite size should be a multiple of two"
        self.coefficient_optimisation = bool(coefficient_optimisation)
        if coefficient_optimisation:
            assert gradient_steps > 0, "The number of gradient steps should be larger than 0"
            CoefficientOptimiser.check_evaluator(fitness_function)
        self.gradient_steps = gradient_steps
        self.optimiser = optimiser if optimiser is not None else adam(learning_rate=0.001, b1=0.9, b2=0.999)
        self.fitness_function = fitness_function
        self.library = NodeLibrary(operator_list, variable_list, self.layer_sizes)
        self.node_to_string = self.library.node_to_string
        self.string_to_node = self.library.string_to_node
        self.slots = self.library.slots
        self.variable_array = self.library.variable_array
        if verbose:
            print(f"Input data should be formatted as: {self.library.input_format}.")
        self.vmap_foriloop = TreeEvaluator(self.library, max_nodes, device)
        self.device = device
        self.operators = Operators(self.library, max_nodes, max_init_depth, coefficient_sd)
        if evolve_backend not in ("native", "numpy"):
            raise ValueError(f"evolve_backend must be 'native' or 'numpy', got {evolve_backend!r}")
        self.evolve_backend = evolve_backend
        self._evolver = None

    # ----------------------------------------------------------------- hot path
    def _engine(self) -> DeviceEngine:
        return self.vmap_foriloop.engine(self.fitness_function, self.size_parsinomy)

    def evaluate_population(self, populations, data) -> Tuple[np.ndarray, np.ndarray]:
        """Fitness of every candidate (gp.py:403-433): flatten, shard over ranks, one fused kernel
        launch per rank, parsimony in-kernel, all-gather of fitness, best-so-far bookkeeping.
        With coefficient_optimisation, every 5th generation after generation 10 the 50 best
        candidates (by fitness before parsimony) get `gradient_steps` optimiser steps on their
        coefficients (gp.py:418-422; multitreegp_amd.coefficients), split over the ranks like
        shard_optimise (gp.py:264-267) and all-gathered.  Under Dopri5 + PIDController the
        step sizes carry no tangent, as diffrax's controller stops their gradient
        (multitreegp_amd.coefficients)."""
        pops = np.asarray(populations, dtype=np.float32)
        P = self.num_populations * self.population_size
        flat = pops.reshape(P, *pops.shape[2:])
        g = self.current_generation
        if self.coefficient_optimisation:  # on every rank, before any collective: all raise together
            CoefficientOptimiser.check_data(self.fitness_function.prepare(data))
        if self.coefficient_optimisation and g > 10 and (g + 1) % 5 == 0:
            raw = mdist.sharded_fitness(lambda lo, hi: self._evaluate_shard(flat, lo, hi, data, 0.0), P)
            raw = raw.cpu().numpy()
            best_idx = np.argsort(raw, kind="stable")[:50]
            # shard_optimise (gp.py:264-267): the candidates split over the ranks, one all-gather
            opt_fit, opt_pop = mdist.sharded_rows(
                lambda lo, hi: self._optimise_shard(flat[best_idx[lo:hi]], data), len(best_idx), flat.shape[1:])
            flat = flat.copy()
            flat[best_idx] = opt_pop
            raw[best_idx] = opt_fit
            # gp.py:424: + size_parsinomy * (non-empty rows), in float32 like the kernel's epilogue
            counts = (flat[..., 0] != 0).sum(axis=tuple(range(1, flat.ndim - 1))).astype(np.float32)
            fitness = (raw + np.float32(self.size_parsinomy) * counts).astype(np.float32)
        else:
            fitness = mdist.sharded_fitness(lambda lo, hi: self._evaluate_shard(flat, lo, hi, data), P).cpu().numpy()
        best = int(np.argmin(fitness))
        if g < self.num_generations:
            self.best_solutions[g] = flat[best]
            self.best_fitnesses[g] = fitness[best]
        return fitness.reshape(self.num_populations, self.population_size), \
            flat.reshape(self.num_populations, self.population_size, *flat.shape[1:])

    def _optimise_shard(self, cands: np.ndarray, data):
        """GeneticProgramming.optimise (gp.py:454-473) of this rank's candidates on its GPU."""
        if len(cands) == 0:
            return np.zeros(0, np.float32), cands
        opt = CoefficientOptimiser(self.vmap_foriloop.engine(self.fitness_function, 0.0))
        return opt.optimise(cands, data, self.gradient_steps, self.optimiser)

    def _evaluate_shard(self, flat: np.ndarray, lo: int, hi: int, data, parsimony=None) -> torch.Tensor:
        """Fitness of individuals [lo, hi) of the flattened population on this rank's GPU (one
        flatten + one fused kernel launch; shard_eval, gp.py:259-262)."""
        eng = self._engine() if parsimony is None else self.vmap_foriloop.engine(self.fitness_function, parsimony)
        if hi <= lo:
            return torch.empty((0,), dtype=torch.float32, device=eng.device)
        pop_dev = torch.from_numpy(np.ascontiguousarray(flat[lo:hi])).to(eng.device, non_blocking=True)
        return eng.evaluate(pop_dev, data)["fitness"]

    # --------------------------------------------------------------- host side
    def initialize_population(self, key) -> np.ndarray:
        """gp.py:298-308 with the numpy sampler (multitreegp_amd.sampling)."""
        return sample_population(_seed_of(key), self.library, self.population_size, self.num_populations,
                                 self.max_init_depth, self.max_nodes, self.coefficient_sd)

    def evolve(self, populations, fitness, key):
        """gp.py:475-497: optional ring migration, then per population elitism + tournament
        selection + crossover / mutation / resampling.  evolve_backend "native" (default): the C++
        host library (multitreegp_amd.host, include/mtgp_host.h) seeded with `key`; "numpy": the
        numpy restatement (multitreegp_amd.genetic_operators) on PCG64 seeded with `key` (a JAX
        key's words or an int)."""
        if self.evolve_backend == "native":
            if self._evolver is None:
                from .host import HostEvolver
                self._evolver = HostEvolver.for_strategy(self)
            out = self._evolver.evolve(populations, fitness, _seed_of(key), self.current_generation)
            self.current_generation += 1
            return out
        rng = np.random.default_rng(_seed_of(key))
        out = evolve_populations(self.operators, np.asarray(populations, np.float32), np.asarray(fitness), rng,
                                 self.current_generation, self.migration_period, self.migration_size,
                                 self.reproduction_type_probabilities, self.reproduction_probabilities,
                                 self.tournament_probabilities, self.tournament_size, self.elite_size)
        self.current_generation += 1
        return out

    def mutate_pair(self, parent1, parent2, keys, reproduction_probability: float):
        """gp.py:499-511"""
        return self.operators.mutate_pair(parent1, parent2, np.random.default_rng(_seed_of(keys)),
                                          reproduction_probability)

    def sample_pair(self, parent1, parent2, keys, reproduction_probability: float):
        """gp.py:513-525"""
        return self.operators.sample_pair(parent1, parent2, np.random.default_rng(_seed_of(keys)),
                                          reproduction_probability)

    def get_statistics(self, generation: Optional[int] = None):
        if generation is not None:
            return self.best_fitnesses[generation], self.best_solutions[generation]
        return self.best_fitnesses, self.best_solutions

    def tree_to_string(self, tree) -> str:
        return self.library.tree_to_string(tree)

    def to_string(self, candidate) -> str:
        """gp.py:330-354 (requires sympy)."""
        import sympy
        out = ""
        tree_index = 0
        layer_index = 0
        for tree in candidate:
            if tree_index == 0:
                out += "["
            out += str(sympy.parsing.sympy_parser.parse_expr(self.tree_to_string(tree)))
            if tree_index < (self.layer_sizes[layer_index] - 1):
                out += ", "
                tree_index += 1
            else:
                out += "]"
                if layer_index < (self.layer_sizes.shape[0] - 1):
                    out += ", "
                tree_index = 0
                layer_index += 1
        return out
