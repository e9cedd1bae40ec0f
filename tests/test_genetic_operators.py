"""Host restatement of genetic_operators/ (multitreegp_amd.genetic_operators): the layout
invariants of SURVEY.md §2.1 after every operator, the operator semantics the reference
encodes (mutation.py, crossover.py, reproduction.py), and whole generations on the GPU."""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import genetic_operators as go

from helpers import CONTROL_OPS, SR_OPS

DYN_VARS = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]


def _ops(N=30, depth=4, ops=CONTROL_OPS, variables=DYN_VARS, layers=(2, 1)):
    lib = mt.NodeLibrary(ops, variables, list(layers))
    return lib, go.Operators(lib, N, depth)


def _nodes(t):
    return int(np.sum(t[:, 0] != 0))


@pytest.mark.parametrize("which", range(7))
def test_each_mutation_keeps_the_layout(which):
    """Preorder contiguity, a = k-1, b = k-1-|a|, packed empties, coefficient values only on
    coefficient rows -- after every one of the seven mutations (mutation.py:542)."""
    lib, ops = _ops()
    rng = np.random.default_rng(which)
    done = 0
    for _ in range(300):
        t = ops.sample_tree(rng, 4, lib.variable_array[0])
        p = ops.mutation_probabilities(t)
        if p[which] == 0:
            continue
        c = ops.mutate_tree(t, rng, lib.variable_array[0], which)
        go.check_layout(c, lib.slots)
        assert _nodes(c) <= 30
        done += 1
    assert done >= 100


def test_mutation_semantics():
    lib, ops = _ops()
    rng = np.random.default_rng(5)
    vm = lib.variable_array[2]  # readout tree: a1, a2 only
    allowed = set(lib.variable_indices[vm > 0]) | {1} | set(lib.operator_indices)
    for _ in range(200):
        t = ops.sample_tree(rng, 4, vm)
        n = _nodes(t)
        ml = ops.mutate_leaf(t, rng, vm)
        assert _nodes(ml) == n and np.sum(np.any(ml != t, axis=1)) == 1  # exactly one row changes
        if n > 1:
            mo = ops.mutate_operator(t, rng, vm)
            assert set(np.unique(mo[:, 0][mo[:, 0] != 0])) <= allowed
        pre = ops.prepend_operator(t, rng, vm)
        assert int(pre[-1, 0]) in lib.operator_indices and pre[-1, 1] == 28
        old = go.to_preorder(t)
        body = go.to_preorder(pre)[1:]
        assert body[:len(old)] == old or body[-len(old):] == old  # the old tree is one operand
        if n > 3:
            de = ops.delete_operator(t, rng, vm)
            assert _nodes(de) < n
        for c in (ops.add_subtree(t, rng, vm), ops.replace_tree(t, rng, vm)):
            assert set(np.unique(c[:, 0][c[:, 0] != 0])) <= allowed


def test_get_mutations_probabilities():
    """mutation.py:534-539: no growth with < 8 empty rows, no operator edits without operators."""
    lib, ops = _ops(N=12)
    leaf = go.from_preorder([(1, 0.5)], lib.slots, 12)
    assert np.array_equal(ops.mutation_probabilities(leaf) > 0, [1, 1, 0, 0, 1, 0, 1])
    small = go.from_preorder([(lib.string_to_node["sin"], 0), (1, 0.5)], lib.slots, 12)
    assert np.array_equal(ops.mutation_probabilities(small) > 0, [1, 1, 1, 0, 1, 0, 1])
    plus = lib.string_to_node["+"]
    big = go.from_preorder([(plus, 0)] * 2 + [(1, 0.1)] * 3, lib.slots, 12)  # 5 nodes, 7 empty
    assert np.array_equal(ops.mutation_probabilities(big) > 0, [0, 1, 1, 1, 0, 0, 1])


def test_crossover_swaps_subtrees():
    lib, ops = _ops()
    rng = np.random.default_rng(7)
    for _ in range(300):
        t1 = ops.sample_tree(rng, 4, lib.variable_array[0])
        t2 = ops.sample_tree(rng, 4, lib.variable_array[0])
        c1, c2 = ops.crossover(t1, t2, rng)
        go.check_layout(c1, lib.slots)
        go.check_layout(c2, lib.slots)
        assert _nodes(c1) + _nodes(c2) == _nodes(t1) + _nodes(t2)  # a swap conserves nodes
        a = sorted(go.to_preorder(t1) + go.to_preorder(t2))
        b = sorted(go.to_preorder(c1) + go.to_preorder(c2))
        assert a == b


def test_tree_masks_select_at_least_one_tree():
    lib, ops = _ops()
    rng = np.random.default_rng(1)
    for _ in range(200):
        assert ops._tree_mask(rng, 3, 0.05).any()


def test_elitism_tournament_and_migration():
    lib, ops = _ops(N=20, depth=3)
    rng = np.random.default_rng(2)
    pop = np.stack([np.stack([ops.sample_tree(rng, 3, lib.variable_array[t]) for t in range(3)]) for _ in range(20)])
    fit = rng.random(20).astype(np.float32)
    new = go.evolve_population(ops, pop, fit, rng, [0.9, 0.1, 0.0], 1.0, 0.6 * 0.4 ** np.arange(7), 7, 4)
    assert new.shape == pop.shape
    assert np.array_equal(new[:4], pop[np.argsort(fit)[:4]])  # elite first, best first
    # rank-0 probability 0.6 (normalised): the tournament winner is usually the best of 7
    wins = [go.tournament_selection(np.arange(20)[:, None], fit, rng, 0.6 * 0.4 ** np.arange(7), 7)[0]
            for _ in range(2000)]
    assert np.mean(fit[wins]) < np.mean(fit) - 0.15
    recv, send = pop.copy(), pop[::-1].copy()
    rf, sf = fit.copy(), fit[::-1].copy()
    m = go.migrate_population(recv, send, rf, sf, 3)
    assert np.array_equal(m[:3], send[np.argsort(sf)[:3]])  # sender's best replace
    assert np.array_equal(m[3:], recv[np.argsort(-rf)][3:])  # receiver's worst (sorted worst first)


def test_genetic_programming_evolve_schedules_and_migration():
    """gp.py:113-121 schedules and the migration period; shapes and layout over generations."""
    ff = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05, solver=mt.RK4())
    gp = mt.GeneticProgramming(6, 20, ff, CONTROL_OPS, DYN_VARS, [2, 1], num_populations=3, migration_period=2,
                               verbose=False)
    np.testing.assert_allclose(gp.selection_pressures, [0.6, 0.75, 0.9])
    np.testing.assert_allclose(gp.reproduction_type_probabilities[0], [0.9, 0.1, 0.0])
    np.testing.assert_allclose(gp.reproduction_type_probabilities[-1], [0.4, 0.5, 0.1])
    np.testing.assert_allclose(gp.tournament_probabilities[0, :2], [0.6, 0.24])
    assert gp.migration_size == 2 and gp.elite_size == 2
    pops = gp.initialize_population(3)
    rng = np.random.default_rng(0)
    for g in range(4):
        pops = gp.evolve(pops, rng.random((3, 20)).astype(np.float32), g)
        assert pops.shape == (3, 20, 3, 30, 4) and gp.current_generation == g + 1
        for t in pops.reshape(-1, 30, 4):
            go.check_layout(t, gp.library.slots)


# ------------------------------------------------------------------------------ GPU
def _notebook(kind):
    """The three notebooks' strategies at a small population (5 generations)."""
    from multitreegp_amd import prng
    if kind == "sr":
        env = mt.VanDerPolOscillator(0, 0)
        data = mt.environments.jax_sr_data(prng.split(prng.PRNGKey(0))[1], env, 16, 20.0)
        ff = mt.SREvaluator(solver=mt.Dopri5(), dt0=0.01, max_steps=500,
                            stepsize_controller=mt.PIDController(atol=1e-6, rtol=1e-6, dtmin=0.001))
        return mt.GeneticProgramming(5, 20, ff, SR_OPS, [["x0", "x1"]], [2], num_populations=2,
                                     verbose=False), data
    env = mt.Acrobot(0.05, 0.1)
    data = mt.environments.jax_control_data(prng.split(prng.PRNGKey(1))[1], env, 16, 0.2, 50.0)
    pid = dict(solver=mt.Dopri5(), max_steps=1000,
               stepsize_controller=mt.PIDController(atol=1e-4, rtol=1e-4, dtmin=0.001))
    if kind == "static":
        ff = mt.FeedforwardEvaluator(env, 0.05, **pid)
        return mt.GeneticProgramming(5, 20, ff, CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1], num_populations=2,
                                     size_parsinomy=1, verbose=False), data
    ff = mt.DynamicEvaluator(env, 2, 0.05, **pid)
    return mt.GeneticProgramming(5, 20, ff, CONTROL_OPS, DYN_VARS, [2, 1], num_populations=2,
                                 verbose=False), data


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sr", "static", "dynamic"])
def test_gpu_notebook_loops_run_five_generations(kind):
    """The notebooks' driver loop (evaluate_population -> get_statistics -> evolve) for five
    generations on the GPU: finite best fitness, elitism makes it non-increasing."""
    gp, data = _notebook(kind)
    pops = gp.initialize_population(1)
    for g in range(5):
        fitness, pops = gp.evaluate_population(pops, data)
        assert fitness.shape == (2, 20) and np.all(np.isfinite(fitness))
        if g < 4:
            pops = gp.evolve(pops, fitness, g)
    best, _ = gp.get_statistics()
    assert np.all(np.diff(best) <= 1e-6), best  # the elite survives every generation
    assert gp.to_string(gp.best_solutions[-1]).startswith("[")
