"""Genetic operators: numpy restatement of MultiTreeGP/genetic_operators/ (host side).

The evaluation path runs on the GPU; this module restates the reference's evolution so that
whole generations (evaluate_population -> evolve) run where the reference's JAX code cannot
travel.  Every operator keeps the reference's array contract
(SURVEY.md §2.1): a tree is float32 ``[N, 4]`` rows ``[f, a, b, value]``, empty rows packed at
the low indices, root at row N-1, descending rows in preorder, ``a = k-1`` and
``b = k-1-|subtree(a)|``.  Node choices are made on row indices with the reference's
probabilities; the edits themselves are done on the preorder node list and written back,
which is the layout the reference's roll/where formulas maintain.

The random stream is numpy's PCG64 (jax is absent here), so runs are distributed like the
reference's but not draw-for-draw identical.  Where a reference rejection loop could spin
forever (e.g. a single operator in the library for mutate_operator), the restatement gives up
after ``MAX_RETRIES`` draws and leaves the tree unchanged.

References: initialization.py (sample_tree, via multitreegp_amd.sampling), mutation.py:9-579,
crossover.py:8-218, reproduction.py:8-176, genetic_programming.py:475-525.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from .node_library import NodeLibrary
from .sampling import create_map_b_to_d, sample_tree

MAX_RETRIES = 1000
EMPTY_ROW = np.array([0.0, -1.0, -1.0, 0.0], np.float32)

Node = Tuple[int, float]  # (opcode f, value)


# ------------------------------------------------------------------ layout helpers
def find_end_idx(tree: np.ndarray, idx: int) -> int:
    """mutation.py:9-26 / crossover.py:23-40: row just below the subtree rooted at row idx
    (the subtree spans rows end+1 .. idx)."""
    open_slots, counter = 1, idx
    while open_slots > 0:
        _, a, b, _ = tree[counter]
        open_slots -= 1
        open_slots += int(a >= 0) + int(b >= 0)
        counter -= 1
    return int(counter)


def to_preorder(tree: np.ndarray) -> List[Node]:
    """Non-empty rows N-1, N-2, ... (preorder) -> [(f, value)]."""
    N = tree.shape[0]
    out = []
    for k in range(N - 1, -1, -1):
        f = int(tree[k, 0])
        if f == 0:
            break
        out.append((f, float(tree[k, 3])))
    return out


def subtree_sizes(nodes: Sequence[Node], slots: np.ndarray) -> List[int]:
    """Size of the subtree at every preorder position (one backward pass with a stack of the
    sizes of completed subtrees)."""
    sizes = [0] * len(nodes)
    stack: List[int] = []
    for i in range(len(nodes) - 1, -1, -1):
        s = 1
        for _ in range(int(slots[nodes[i][0]])):
            s += stack.pop()
        sizes[i] = s
        stack.append(s)
    return sizes


def from_preorder(nodes: Sequence[Node], slots: np.ndarray, N: int) -> np.ndarray:
    """[(f, value)] in preorder -> reference [N, 4] array (root at N-1, a = k-1,
    b = k-1-|a|, coefficient values only on f == 1 rows, empties packed low)."""
    n = len(nodes)
    if n > N:
        raise ValueError(f"tree of {n} nodes exceeds max_nodes {N}")
    sizes = subtree_sizes(nodes, slots)
    t = np.tile(EMPTY_ROW, (N, 1))
    for i, (f, v) in enumerate(nodes):
        k = N - 1 - i
        ar = int(slots[f])
        a = k - 1 if ar >= 1 else -1
        b = k - 1 - sizes[i + 1] if ar == 2 else -1
        t[k] = (f, a, b, v if f == 1 else 0.0)
    return t


def check_layout(tree: np.ndarray, slots: np.ndarray) -> None:
    """Assert the reference's layout invariants (tests)."""
    N = tree.shape[0]
    nodes = to_preorder(tree)
    n = len(nodes)
    assert np.all(tree[: N - n, 0] == 0) and np.all(tree[: N - n, 1:3] == -1), "empties not packed low"
    assert n >= 1, "empty tree"
    assert np.array_equal(from_preorder(nodes, slots, N), tree), "rows differ from the preorder layout"


# ------------------------------------------------------------------ the operator context
class Operators:
    """The reference's partial-bound operator arguments (gp.py:204-238): node library,
    max_nodes, max_init_depth, coefficient_sd."""

    def __init__(self, lib: NodeLibrary, max_nodes: int, max_init_depth: int, coefficient_sd: float = 1.0):
        self.lib = lib
        self.N = int(max_nodes)
        self.max_init_depth = int(max_init_depth)
        self.coefficient_sd = float(coefficient_sd)
        self.slots = np.asarray(lib.slots)
        self.map_b_to_d = create_map_b_to_d(self.max_init_depth)
        op_p = np.asarray(lib.operator_probabilities, np.float64)
        self.op_p = op_p / op_p.sum()
        self.operator_indices = np.asarray(lib.operator_indices)
        self.variable_indices = np.asarray(lib.variable_indices)

    # -- sampling primitives
    def sample_tree(self, rng, depth: int, var_mask) -> np.ndarray:
        """sample_tree(key, depth, variable_array) (initialization.py:100-124) with the GP's
        table size 2**max_init_depth - 1 and the depth limit `depth`."""
        return sample_tree(rng, self.lib, np.asarray(var_mask), self.max_init_depth, self.N, self.coefficient_sd,
                           self.map_b_to_d, depth_limit=depth)

    def new_leaf(self, rng, var_mask) -> Node:
        """coefficient w.p. 0.5 (N(0, coefficient_sd)) else an allowed variable (mutation.py:60, 188)."""
        coef = np.float32(rng.standard_normal() * self.coefficient_sd)
        if rng.random() < 0.5:
            return (1, float(coef))
        p = np.asarray(var_mask, np.float64)
        return (int(rng.choice(self.variable_indices, p=p / p.sum())), 0.0)

    def new_operator(self, rng) -> int:
        return int(rng.choice(self.operator_indices, p=self.op_p))

    def choose_row(self, rng, weights: np.ndarray) -> int:
        w = np.asarray(weights, np.float64)
        return int(rng.choice(self.N, p=w / w.sum()))

    def is_leaf(self, tree) -> np.ndarray:
        f = tree[:, 0]
        return (f == 1) | np.isin(f, self.variable_indices)

    def is_operator(self, tree) -> np.ndarray:
        return np.isin(tree[:, 0], self.operator_indices)

    # -- edits on the preorder list
    def _replace(self, tree, row: int, new_nodes: Sequence[Node]) -> np.ndarray:
        """Replace the subtree rooted at `row` by `new_nodes` (a preorder list)."""
        nodes = to_preorder(tree)
        p = self.N - 1 - row
        size = subtree_sizes(nodes, self.slots)[p]
        return from_preorder(nodes[:p] + list(new_nodes) + nodes[p + size:], self.slots, self.N)

    def _subtree_nodes(self, tree, row: int) -> List[Node]:
        nodes = to_preorder(tree)
        p = self.N - 1 - row
        return nodes[p:p + subtree_sizes(nodes, self.slots)[p]]

    # ------------------------------------------------------------ mutations (mutation.py)
    def add_subtree(self, tree, rng, var_mask):
        """mutation.py:127-165: a random leaf becomes a random depth-2 subtree."""
        row = self.choose_row(rng, self.is_leaf(tree))
        sub = to_preorder(self.sample_tree(rng, 2, var_mask))
        return self._replace(tree, row, sub)

    def mutate_leaf(self, tree, rng, var_mask):
        """mutation.py:167-198: a random leaf becomes a different leaf (a coefficient may be
        redrawn as a coefficient)."""
        for _ in range(MAX_RETRIES):
            row = self.choose_row(rng, self.is_leaf(tree))
            f, v = self.new_leaf(rng, var_mask)
            if not (tree[row, 0] == f and f != 1):
                child = tree.copy()
                child[row, 0] = f
                child[row, 3] = v if f == 1 else 0.0
                return child
        return tree.copy()

    def mutate_operator(self, tree, rng, var_mask):
        """mutation.py:300-340: a random operator becomes a different one; an arity change
        resamples its operands (2 -> 1: one depth-2 subtree, replace_with_one_subtree; 1 -> 2: two
        depth-1 leaves, replace_with_two_subtrees).  Rejection test check_invalid_operator_node
        (mutation.py:80-102)."""
        empty = int(np.sum(tree[:, 0] == 0))
        for _ in range(MAX_RETRIES):
            row = self.choose_row(rng, self.is_operator(tree))
            op = self.new_operator(rng)
            size = row - find_end_idx(tree, row)
            need = 7 if self.slots[op] == 2 else 8
            if not (tree[row, 0] == op or empty + size < need):
                break
        else:
            return tree.copy()
        cur, new = int(self.slots[int(tree[row, 0])]), int(self.slots[op])
        if cur == new:
            child = tree.copy()
            child[row, 0] = op
            return child
        if new == 1:
            sub = to_preorder(self.sample_tree(rng, 2, var_mask))
            return self._replace(tree, row, [(op, 0.0)] + sub)
        s1 = to_preorder(self.sample_tree(rng, 1, var_mask))
        s2 = to_preorder(self.sample_tree(rng, 1, var_mask))
        return self._replace(tree, row, [(op, 0.0)] + s1 + s2)

    def delete_operator(self, tree, rng, var_mask):
        """mutation.py:342-382: a random non-root operator and its operands become a leaf."""
        w = self.is_operator(tree).copy()
        w[-1] = False
        row = self.choose_row(rng, w)
        return self._replace(tree, row, [self.new_leaf(rng, var_mask)])

    def prepend_operator(self, tree, rng, var_mask):
        """mutation.py:384-427: a new root operator above the tree; with two operands the old
        tree is the first or second one (Bernoulli), the other a depth-2 subtree."""
        op = self.new_operator(rng)
        sub = to_preorder(self.sample_tree(rng, 2, var_mask))
        second = rng.random() < 0.5
        old = to_preorder(tree)
        if self.slots[op] == 2:
            body = (sub + old) if second else (old + sub)
        else:
            body = old
        return from_preorder([(op, 0.0)] + body, self.slots, self.N)

    def insert_operator(self, tree, rng, var_mask):
        """mutation.py:429-486: a new operator above a random non-root operator node; with two
        operands the old subtree is the first or second one, the other a depth-2 subtree."""
        w = self.is_operator(tree).copy()
        w[-1] = False
        row = self.choose_row(rng, w)
        op = self.new_operator(rng)
        sub = to_preorder(self.sample_tree(rng, 2, var_mask))
        second = rng.random() < 0.5
        old = self._subtree_nodes(tree, row)
        if self.slots[op] == 2:
            body = (sub + old) if second else (old + sub)
        else:
            body = old
        return self._replace(tree, row, [(op, 0.0)] + body)

    def replace_tree(self, tree, rng, var_mask):
        """mutation.py:488-503: a fresh tree of max_init_depth."""
        return self.sample_tree(rng, self.max_init_depth, var_mask)

    MUTATIONS = ("add_subtree", "mutate_leaf", "mutate_operator", "delete_operator", "prepend_operator",
                 "insert_operator", "replace_tree")  # MUTATE_FUNCTIONS, mutation.py:542

    def mutation_probabilities(self, tree) -> np.ndarray:
        """get_mutations (mutation.py:523-539)."""
        p = np.ones(7)
        empty, used = int(np.sum(tree[:, 0] == 0)), int(np.sum(tree[:, 0] != 0))
        if empty < 8:
            p = np.array([0., 1., 1., 1., 0., 0., 1.])  # too big to add nodes
        if used <= 3:
            p = np.array([1., 1., 1., 0., 1., 0., 1.])  # no non-root operator
        if used == 1:
            p = np.array([1., 1., 0., 0., 1., 0., 1.])  # no operator
        return p / p.sum()

    def mutate_tree(self, tree, rng, var_mask, which: Optional[int] = None):
        if which is None:
            which = int(rng.choice(7, p=self.mutation_probabilities(tree)))
        return getattr(self, self.MUTATIONS[which])(tree, rng, var_mask)

    def _tree_mask(self, rng, n_trees: int, p: float) -> np.ndarray:
        """sample_indices loop (mutation.py:28-41, 571): Bernoulli(p) per tree, at least one."""
        while True:
            m = rng.random(n_trees) < p
            if m.any():
                return m

    def mutate_trees(self, candidate, rng, reproduction_probability: float):
        """initialize_mutation_functions.mutate_trees (mutation.py:555-577)."""
        T = candidate.shape[0]
        mask = self._tree_mask(rng, T, reproduction_probability)
        out = candidate.copy()
        for t in range(T):
            mutated = self.mutate_tree(candidate[t], rng, self.lib.variable_array[t])
            if mask[t]:
                out[t] = mutated
        return out

    # ------------------------------------------------------------- crossover (crossover.py)
    def _cx_weights(self, tree) -> np.ndarray:
        """operators weight 2, leaves 1, empty rows 0 (crossover.py:110-116)."""
        w = self.is_operator(tree).astype(np.float64)
        return np.where(tree[:, 0] == 0, w, w + 1)

    def _cx_invalid(self, t1, t2, i1, i2) -> bool:
        """check_invalid_cx_nodes (crossover.py:60-91)."""
        s1, s2 = i1 - find_end_idx(t1, i1), i2 - find_end_idx(t2, i2)
        e1, e2 = int(np.sum(t1[:, 0] == 0)), int(np.sum(t2[:, 0] == 0))
        equal = False
        if s1 == s2 and (np.sum(t1[:, 0] != 0) > 1 or np.sum(t2[:, 0] != 0) > 1):
            equal = True
            for k in range(s1):
                a, b = t1[i1 - k], t2[i2 - k]
                same_leaf = a[3] == b[3] and a[0] == 1
                if not ((a[0] == b[0] and a[0] > 1) or same_leaf):
                    equal = False
                    break
        return e1 < s2 - s1 or e2 < s1 - s2 or equal

    def crossover(self, t1, t2, rng):
        """crossover (crossover.py:120-192): swap two random subtrees (rejection sampling for
        fit and difference)."""
        for _ in range(MAX_RETRIES):
            i1 = self.choose_row(rng, self._cx_weights(t1))
            i2 = self.choose_row(rng, self._cx_weights(t2))
            if not self._cx_invalid(t1, t2, i1, i2):
                break
        else:
            return t1.copy(), t2.copy()
        a, b = self._subtree_nodes(t1, i1), self._subtree_nodes(t2, i2)
        return self._replace(t1, i1, b), self._replace(t2, i2, a)

    def crossover_trees(self, parent1, parent2, rng, reproduction_probability: float):
        """crossover_trees (crossover.py:194-218): per tree pair, Bernoulli mask (>= 1 tree)."""
        T = parent1.shape[0]
        mask = self._tree_mask(rng, T, reproduction_probability)
        c1, c2 = parent1.copy(), parent2.copy()
        for t in range(T):
            o1, o2 = self.crossover(parent1[t], parent2[t], rng)
            if mask[t]:
                c1[t], c2[t] = o1, o2
        return c1, c2

    def mutate_pair(self, parent1, parent2, rng, reproduction_probability: float):
        """GeneticProgramming.mutate_pair (gp.py:499-511)."""
        return (self.mutate_trees(parent1, rng, reproduction_probability),
                self.mutate_trees(parent2, rng, reproduction_probability))

    def sample_pair(self, parent1, parent2, rng, reproduction_probability: float):
        """GeneticProgramming.sample_pair (gp.py:513-525): two fresh candidates."""
        T = parent1.shape[0]
        mk = lambda: np.stack([self.sample_tree(rng, self.max_init_depth, self.lib.variable_array[t])  # noqa: E731
                               for t in range(T)])
        return mk(), mk()


# ---------------------------------------------------------------- reproduction.py
def tournament_selection(population, fitness, rng, tournament_probabilities, tournament_size: int):
    """reproduction.py:29-49: tournament of `tournament_size` (with replacement), rank r of
    the fitness-sorted tournament wins with probability ~ sp (1 - sp)^r."""
    idx = rng.integers(0, population.shape[0], size=tournament_size)
    ranked = idx[np.argsort(fitness[idx], kind="stable")]
    p = np.asarray(tournament_probabilities, np.float64)
    return population[int(rng.choice(ranked, p=p / p.sum()))]


def evolve_population(ops: Operators, population, fitness, rng, reproduction_type_probabilities,
                      reproduction_probability: float, tournament_probabilities, tournament_size: int,
                      elite_size: int):
    """reproduction.py:51-108: elite + pairs of tournament winners reproduced by crossover /
    mutation / resampling -> a population of the same size."""
    pop_size = population.shape[0]
    elite = population[np.argsort(fitness, kind="stable")[:elite_size]]
    n_pairs = (pop_size - elite_size) // 2
    left = [tournament_selection(population, fitness, rng, tournament_probabilities, tournament_size)
            for _ in range(n_pairs)]
    right = [tournament_selection(population, fitness, rng, tournament_probabilities, tournament_size)
             for _ in range(n_pairs)]
    tp = np.asarray(reproduction_type_probabilities, np.float64)
    types = rng.choice(3, size=n_pairs, p=tp / tp.sum())
    funcs = (ops.crossover_trees, ops.mutate_pair, ops.sample_pair)
    lc, rc = [], []
    for k in range(n_pairs):
        a, b = funcs[types[k]](left[k], right[k], rng, reproduction_probability)
        lc.append(a)
        rc.append(b)
    parts = [elite] + ([np.stack(lc), np.stack(rc)] if n_pairs else [])
    return np.concatenate(parts, axis=0).astype(np.float32)


def migrate_population(receiver, sender, receiver_fitness, sender_fitness, migration_size: int):
    """reproduction.py:110-131: the receiver sorted worst-first has its first migration_size
    places taken by the sender's best (sender sorted best-first)."""
    r = receiver[np.argsort(-np.asarray(receiver_fitness), kind="stable")]
    s = sender[np.argsort(np.asarray(sender_fitness), kind="stable")]
    out = r.copy()
    out[:migration_size] = s[:migration_size]
    return out


def evolve_populations(ops: Operators, populations, fitness, rng, current_generation: int, migration_period: int,
                       migration_size: int, reproduction_type_probabilities, reproduction_probabilities,
                       tournament_probabilities, tournament_size: int, elite_size: int):
    """reproduction.py:133-176.  As in the reference, migration re-orders each population but the
    fitness handed to evolve_population keeps the pre-migration order."""
    num_pop = populations.shape[0]
    if num_pop > 1 and (current_generation + 1) % migration_period == 0:
        senders, sfit = np.roll(populations, 1, axis=0), np.roll(fitness, 1, axis=0)
        populations = np.stack([migrate_population(populations[i], senders[i], fitness[i], sfit[i], migration_size)
                                for i in range(num_pop)])
    return np.stack([evolve_population(ops, populations[i], fitness[i], rng, reproduction_type_probabilities[i],
                                       float(reproduction_probabilities[i]), tournament_probabilities[i],
                                       tournament_size, elite_size) for i in range(num_pop)])
