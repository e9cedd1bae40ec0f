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


def sample_trees_batch(rng: np.random.Generator, lib: NodeLibrary, var_mask: np.ndarray, B: int,
                       max_init_depth: int, max_nodes: int, coefficient_sd: float = 1.0,
                       map_b_to_d: np.ndarray = None) -> np.ndarray:
    """B independent trees of sample_tree's distribution (initialization.py:9-124), sampled
    together: the breadth-first loop of sample_node runs once over all B trees with numpy
    vector operations.  Only breadth-first indices below 2*max_nodes - 1 can hold a node: an
    operator needs `open_slots < max_nodes - i - 1` (initialization.py:35), so operators sit at
    i <= max_nodes - 2 and their children at i <= 2*max_nodes - 2 -- the loop stops there (or at
    2**max_init_depth - 1, or when every tree has no open slot).  -> float32 [B, max_nodes, 4]"""
    if map_b_to_d is None:
        map_b_to_d = create_map_b_to_d(max_init_depth)
    N = max_nodes
    tree_size = 2 ** max_init_depth - 1
    I = min(tree_size, 2 * N - 1)
    slots = np.asarray(lib.slots, dtype=np.int64)
    op_p = lib.operator_probabilities.astype(np.float64)
    op_cdf = np.cumsum(op_p / op_p.sum())
    var_p = np.asarray(var_mask, dtype=np.float64)
    var_cdf = np.cumsum(var_p / var_p.sum())
    var_idx = np.asarray(lib.variable_indices, dtype=np.int64)
    op_idx = np.asarray(lib.operator_indices, dtype=np.int64)
    f = np.zeros((B, I), dtype=np.int64)
    coef = np.zeros((B, I), dtype=np.float32)
    open_slots = np.ones(B, dtype=np.int64)
    for i in range(I):
        live = open_slots > 0
        if not live.any():
            break
        c = (rng.standard_normal(B) * coefficient_sd).astype(np.float32)
        u = rng.random((4, B))
        depth = (i + 1).bit_length() - 1
        leaf = np.where(u[0] < 0.5, 1,
                        var_idx[np.minimum(np.searchsorted(var_cdf, u[1], side="right"), len(var_idx) - 1)])
        can_op = (open_slots < N - i - 1) & (depth + 1 < max_init_depth) & (u[2] < 0.7 ** depth)
        op = op_idx[np.minimum(np.searchsorted(op_cdf, u[3], side="right"), len(op_idx) - 1)]
        index = np.where(can_op, op, leaf)
        index = np.where(live, index, 0)
        if i > 0:  # the parent's arity must reach this child (initialization.py:43)
            pf = f[:, (i + (i % 2) - 2) // 2]
            index = np.where(slots[pf] + i % 2 > 1, index, 0)
        f[:, i] = index
        coef[:, i] = np.where(index == 1, c, 0.0)
        open_slots = np.where(index == 0, open_slots, np.maximum(0, open_slots + slots[index] - 1))
    # prune (initialization.py:56-98): non-empty rows, highest depth-first row first, packed at the end
    rows = map_b_to_d[:I]
    key = np.where(f != 0, rows[None, :], -1)
    order = np.argsort(-key, axis=1, kind="stable")
    rank = np.empty_like(order)
    np.put_along_axis(rank, order, np.arange(I)[None, :].repeat(B, 0), axis=1)
    n_keep = (f != 0).sum(1)
    assert int(n_keep.max(initial=0)) <= N
    newpos = np.where(f != 0, N - 1 - rank, -1)
    ch_a = np.minimum(2 * np.arange(I) + 1, I - 1)
    ch_b = np.minimum(2 * np.arange(I) + 2, I - 1)
    a_pos = np.where(slots[f] > 0, newpos[:, ch_a], -1)
    b_pos = np.where(slots[f] > 1, newpos[:, ch_b], -1)
    out = np.tile(np.array([0.0, -1.0, -1.0, 0.0], dtype=np.float32), (B, N, 1))
    bb, ii = np.nonzero(f)
    out[bb, newpos[bb, ii]] = np.stack([f[bb, ii], a_pos[bb, ii], b_pos[bb, ii], coef[bb, ii]], axis=1)
    return out


def sample_population(seed: int, lib: NodeLibrary, population_size: int, num_populations: int = 1,
                      max_init_depth: int = 4, max_nodes: int = 30,
                      coefficient_sd: float = 1.0) -> np.ndarray:
    """[num_pop, pop, T, N, 4] float32 population (initialize_population, gp.py:298-308): each
    tree position t sampled for the whole population at once (sample_trees_batch)."""
    rng = np.random.default_rng(seed)
    m = create_map_b_to_d(max_init_depth)
    T = lib.num_trees
    B = num_populations * population_size
    out = np.zeros((B, T, max_nodes, 4), dtype=np.float32)
    chunk = 1 << 15  # bounded temporaries ([chunk, 2N] index tables)
    for t in range(T):
        for lo in range(0, B, chunk):
            hi = min(B, lo + chunk)
            out[lo:hi, t] = sample_trees_batch(rng, lib, lib.variable_array[t], hi - lo, max_init_depth,
                                               max_nodes, coefficient_sd, m)
    return out.reshape(num_populations, population_size, T, max_nodes, 4)
