"""Population sampler: numpy restatement of genetic_operators/initialization.py.

Host-side, off the hot path.  It produces populations in the reference's exact array layout
(``[num_pop, pop, T, N, 4]`` float32, rows ``[f, a, b, value]``, empty rows packed at low
indices, root at row N-1, descending rows in preorder) with the reference's distribution
(initialization.py:9-54): breadth-first sampling of a full tree of depth ``max_init_depth``
stored depth-first through ``map_b_to_d`` (gp.py:272-296), operator probability 0.7**depth,
leaf = coefficient N(0, coefficient_sd) w.p. 0.5 else an allowed variable, then pruning of
empty rows (initialization.py:56-98).  The random stream is numpy's PCG64, not JAX threefry,
so populations are distributed like the reference's but not bit-identical to them.
"""
from __future__ import annotations

import numpy as np

from .node_library import NodeLibrary


def create_map_b_to_d(depth: int) -> np.ndarray:
    """Breadth-first index -> depth-first row (gp.py:272-296)."""
    max_nodes = 2 ** depth - 1
    current_depth = 0
    m = np.zeros(max_nodes, dtype=np.int64)
    for i in range(max_nodes):
        if i > 0:
            parent = (i + (i % 2) - 2) // 2
            value = m[parent]
            if i % 2 == 0:
                m[i] = value + 2 ** (depth - current_depth + 1)
            else:
                m[i] = value + 1
        current_depth += i == (2 ** current_depth - 1)
    return max_nodes - 1 - m


def _prune(tree: np.ndarray, max_nodes: int) -> np.ndarray:
    """prune_tree (initialization.py:56-98): keep non-empty rows, highest first, at the end."""
    keep = np.nonzero(tree[:, 0] != 0)[0][::-1]  # rows in descending order
    n = keep.size
    assert n <= max_nodes
    out = np.tile(np.array([0.0, -1.0, -1.0, 0.0], dtype=np.float32), (max_nodes, 1))
    new_pos = np.full(tree.shape[0], -1, dtype=np.int64)
    new_pos[keep] = max_nodes - 1 - np.arange(n)
    rows = tree[keep].copy()
    for c in (1, 2):
        m = rows[:, c] > -1
        rows[m, c] = new_pos[rows[m, c].astype(np.int64)]
    out[new_pos[keep]] = rows
    return out


def sample_tree(rng: np.random.Generator, lib: NodeLibrary, var_mask: np.ndarray, max_init_depth: int,
                max_nodes: int, coefficient_sd: float = 1.0, map_b_to_d: np.ndarray = None,
                depth_limit: int = None) -> np.ndarray:
    """sample_tree (initialization.py:100-124) for one tree with allowed-variable mask.

    `max_init_depth` sizes the breadth-first table (2**max_init_depth - 1 rows, map_b_to_d);
    `depth_limit` (default max_init_depth) is the depth argument of the reference's
    sample_tree(key, depth, variable_array): operators only above depth_limit - 1 (the
    mutations sample depth-2 and depth-1 subtrees this way, mutation.py:149, 226, 273).
    The breadth-first sampling visits only the rows it fills, so they are kept sparsely
    (row -> [f, a, b, value]) and pruned directly (prune_tree, initialization.py:56-98):
    non-empty rows, highest first, packed at the end of max_nodes rows."""
    if map_b_to_d is None:
        map_b_to_d = create_map_b_to_d(max_init_depth)
    if depth_limit is None:
        depth_limit = max_init_depth
    tree_size = 2 ** max_init_depth - 1
    slots = lib.slots
    op_p = lib.operator_probabilities.astype(np.float64)
    op_p = op_p / op_p.sum()
    var_p = var_mask.astype(np.float64)
    var_p = var_p / var_p.sum()
    # bulk draws (the reference splits a key per node; only the distribution matters here):
    # one chunk for trees of depth <= 10, chunks of 64 nodes for deeper ones (most deep trees
    # stop after a few dozen nodes, and the chunked stream keeps sampling O(tree) not O(2^depth))
    chunk = tree_size if tree_size <= 1023 else 64

    def draws():
        return ((rng.standard_normal(chunk) * coefficient_sd).astype(np.float32), rng.random(chunk),
                rng.random(chunk), rng.random(chunk), rng.random(chunk))

    var_cdf = np.cumsum(var_p)
    op_cdf = np.cumsum(op_p)
    nv, no = len(var_cdf), len(op_cdf)
    rows = {}
    open_slots = 1
    for i in range(tree_size):
        if open_slots == 0:
            break  # every remaining node is empty and pruned away
        if i % chunk == 0:
            coef, u_leaf, u_var, u_node, u_op = draws()
        j = i % chunk
        depth = (i + 1).bit_length() - 1
        if u_leaf[j] < 0.5:
            leaf = 1
        else:
            leaf = int(lib.variable_indices[min(int(np.searchsorted(var_cdf, u_var[j], side="right")), nv - 1)])
        if (open_slots < max_nodes - i - 1) and (depth + 1 < depth_limit) and u_node[j] < 0.7 ** depth:
            index = int(lib.operator_indices[min(int(np.searchsorted(op_cdf, u_op[j], side="right")), no - 1)])
        else:
            index = leaf
        if i > 0:
            parent = rows.get(int(map_b_to_d[(i + (i % 2) - 2) // 2]))
            if not (slots[max(int(parent[0]) if parent else 0, 0)] + i % 2) > 1:
                index = 0
        if index != 0:
            rows[int(map_b_to_d[i])] = (index,
                                        int(map_b_to_d[2 * i + 1]) if slots[index] > 0 else -1,
                                        int(map_b_to_d[2 * i + 2]) if slots[index] > 1 else -1,
                                        coef[j] if index == 1 else 0.0)
            open_slots = max(0, open_slots + int(slots[index]) - 1)
    keep = sorted(rows, reverse=True)
    assert len(keep) <= max_nodes
    new_pos = {r: max_nodes - 1 - k for k, r in enumerate(keep)}
    out = np.tile(np.array([0.0, -1.0, -1.0, 0.0], dtype=np.float32), (max_nodes, 1))
    for r in keep:
        f, a, b, v = rows[r]
        out[new_pos[r]] = (f, new_pos[a] if a > -1 else -1, new_pos[b] if b > -1 else -1, v)
    return out


def sample_population(seed: int, lib: NodeLibrary, population_size: int, num_populations: int = 1,
                      max_init_depth: int = 4, max_nodes: int = 30,
                      coefficient_sd: float = 1.0) -> np.ndarray:
    """[num_pop, pop, T, N, 4] float32 population (initialize_population, gp.py:298-308)."""
    rng = np.random.default_rng(seed)
    m = create_map_b_to_d(max_init_depth)
    T = lib.num_trees
    out = np.zeros((num_populations, population_size, T, max_nodes, 4), dtype=np.float32)
    for a in range(num_populations):
        for b in range(population_size):
            for t in range(T):
                out[a, b, t] = sample_tree(rng, lib, lib.variable_array[t], max_init_depth, max_nodes,
                                           coefficient_sd, m)
    return out
