"""Native host library (include/mtgp_host.h, csrc/mtgp_evolve.cpp): the evolution step in C++.

Checked against the numpy restatement (multitreegp_amd.genetic_operators), which follows the
reference's genetic_operators/ line by line: the layout invariants after whole generations, the
exact parts (elitism, ring migration), and the distributions of what the random parts produce
(tree sizes of fresh, mutated and crossed-over children; coefficient draws; variable masks).
The two use different random streams, so children are compared as distributions, not draws."""
import os

import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import genetic_operators as go
from multitreegp_amd.host import HostEvolver, load
from multitreegp_amd.sampling import sample_population

from helpers import CONTROL_OPS

VARS = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"], ["y1", "y2"]]
TP = [0.6 * 0.4 ** i for i in range(7)]


def _lib():
    return mt.NodeLibrary(CONTROL_OPS, VARS, [1, 1, 1])


def _evolver(lib, N=40, depth=5, E=0, rtp=(0.9, 0.1, 0.0), num_pop=1, migration_size=0, period=10, rp=1.0):
    return HostEvolver(lib, N, depth, 1.0, period, migration_size, 7, E, np.tile(TP, (num_pop, 1)),
                       np.tile(rtp, (num_pop, 1)), np.full(num_pop, rp), num_pop)


def _sizes(pop):
    return (pop[..., 0] != 0).sum(axis=-1).reshape(-1)


def _same_dist(a, b, N):
    """chi-squared homogeneity p-value of two samples of tree sizes (sparse bins pooled)."""
    from scipy.stats import chi2_contingency
    ha, hb = np.bincount(a, minlength=N + 1), np.bincount(b, minlength=N + 1)
    rows, acc = [], np.zeros(2)
    for x, y in zip(ha, hb):
        acc += (x, y)
        if acc.sum() >= 20:
            rows.append(acc.copy())
            acc[:] = 0
    if acc.sum() and rows:
        rows[-1] += acc
    return chi2_contingency(np.array(rows).T)[1]


def _check_pop(pop, lib):
    slots = np.asarray(lib.slots)
    for c in pop.reshape(-1, *pop.shape[-3:]):
        for t, tree in enumerate(c):
            go.check_layout(tree, slots)
            f = tree[:, 0].astype(int)
            var = f[np.isin(f, lib.variable_indices)]
            assert np.all(lib.variable_array[t][var - lib.variable_indices[0]] > 0), "variable outside its tree's mask"


def test_library_loads_and_exports():
    lib = load()
    for sym in ("mtgp_host_abi_version", "mtgp_evolve_populations", "mtgp_sample_population"):
        assert hasattr(lib, sym)
    assert lib.mtgp_host_abi_version() == 1


def test_sampled_population_matches_numpy_sampler():
    """initialize_population: fresh trees distributed like sampling.sample_population (initialization.py)."""
    lib = _lib()
    ev = _evolver(lib, N=40, depth=5)
    nat = ev.sample_population(3000, seed=1)
    ref = sample_population(2, lib, 3000, 1, max_init_depth=5, max_nodes=40)
    _check_pop(nat, lib)
    for t in range(3):
        a, b = _sizes(nat[:, :, t]), _sizes(ref[:, :, t])
        p = _same_dist(a, b, 40)
        assert p > 1e-4, f"tree {t}: size distributions differ (p {p:.2g})"
    coef = nat[..., 3][nat[..., 0] == 1]
    assert abs(coef.mean()) < 0.05 and abs(coef.std() - 1.0) < 0.05
    frac = lambda p: np.mean(p[..., 0][p[..., 0] != 0] == 1)  # noqa: E731
    assert abs(frac(nat) - frac(ref)) < 0.02


@pytest.mark.parametrize("rtp", [(1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0), (0.9, 0.1, 0.0)],
                         ids=["crossover", "mutation", "resample", "mixed"])
def test_generation_matches_numpy_restatement(rtp):
    """One generation from the same parents and fitness: children sizes distributed like the numpy
    restatement's (tournament selection + the operator), layout kept, elite exact."""
    lib = _lib()
    S, E = 2048, 40
    parents = sample_population(3, lib, S, 1, max_init_depth=5, max_nodes=40)
    fit = np.random.default_rng(4).random((1, S)).astype(np.float32)
    ev = _evolver(lib, E=E, rtp=rtp)
    nat = ev.evolve(parents, fit, seed=11, current_generation=0)
    ops = go.Operators(lib, 40, 5)
    ref = go.evolve_populations(ops, parents, fit, np.random.default_rng(11), 0, 10, 0, np.array([rtp]),
                                np.array([1.0]), np.array([TP]), 7, E)
    assert nat.shape == ref.shape == parents.shape
    _check_pop(nat, lib)
    assert np.array_equal(nat[0, :E], ref[0, :E])  # elitism is deterministic
    for t in range(3):
        p = _same_dist(_sizes(nat[0, E:, t]), _sizes(ref[0, E:, t]), 40)
        assert p > 1e-4, f"tree {t}: child size distributions differ (p {p:.2g})"


def test_elitism_and_migration_exact():
    """With elite_size = pop_size the output is the (migrated) population sorted by the
    pre-migration fitness (reproduction.py:51-176): compare bit-exactly with the restatement."""
    lib = _lib()
    S = 64
    pops = sample_population(7, lib, S, 3, max_init_depth=4, max_nodes=40)
    fit = np.random.default_rng(8).random((3, S)).astype(np.float32)
    ops = go.Operators(lib, 40, 4)
    ev = _evolver(lib, E=S, num_pop=3, migration_size=6, period=5)
    for gen in (3, 4):  # (4 + 1) % 5 == 0 migrates
        nat = ev.evolve(pops, fit, seed=1, current_generation=gen)
        ref = go.evolve_populations(ops, pops, fit, np.random.default_rng(0), gen, 5, 6, np.tile([1.0, 0, 0], (3, 1)),
                                    np.ones(3), np.tile(TP, (3, 1)), 7, S)
        assert np.array_equal(nat, ref), f"generation {gen}"


def test_seeded_and_thread_count_independent():
    lib = _lib()
    parents = sample_population(3, lib, 1024, 2, max_init_depth=5, max_nodes=40)
    fit = np.random.default_rng(4).random((2, 1024)).astype(np.float32)
    ev = _evolver(lib, E=20, num_pop=2, migration_size=10, period=2)
    a = ev.evolve(parents, fit, seed=5, current_generation=1)
    old = os.environ.get("MTGP_HOST_THREADS")
    try:
        os.environ["MTGP_HOST_THREADS"] = "1"
        b = ev.evolve(parents, fit, seed=5, current_generation=1)
        os.environ["MTGP_HOST_THREADS"] = "3"
        c = ev.evolve(parents, fit, seed=5, current_generation=1)
    finally:
        if old is None:
            os.environ.pop("MTGP_HOST_THREADS", None)
        else:
            os.environ["MTGP_HOST_THREADS"] = old
    assert np.array_equal(a, b) and np.array_equal(a, c)
    d = ev.evolve(parents, fit, seed=6, current_generation=1)
    assert not np.array_equal(a, d)


def test_many_generations_keep_the_layout():
    """Twenty generations at max_nodes 20 (size limits hit often): every tree stays valid."""
    lib = _lib()
    ev = _evolver(lib, N=20, depth=4, E=4, rtp=(0.5, 0.4, 0.1), num_pop=2, migration_size=4, period=3)
    pops = ev.sample_population(128, seed=3)
    rng = np.random.default_rng(0)
    for gen in range(20):
        fit = rng.random((2, 128)).astype(np.float32)
        pops = ev.evolve(pops, fit, seed=100 + gen, current_generation=gen)
    _check_pop(pops, lib)
    assert pops.shape == (2, 128, 3, 20, 4)


def test_rejects_bad_shapes():
    lib = _lib()
    ev = _evolver(lib)
    pops = ev.sample_population(8, seed=0)
    with pytest.raises(ValueError):
        ev.evolve(pops, np.zeros((1, 7), np.float32), 0, 0)
    with pytest.raises(ValueError):
        ev.evolve(pops[:, :, :2], np.zeros((1, 8), np.float32), 0, 0)


def test_strategy_uses_the_native_step():
    ops = CONTROL_OPS
    env = mt.Acrobot(0.0, 0.0)
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4())
    for backend in ("native", "numpy"):
        gp = mt.GeneticProgramming(2, 32, ff, ops, VARS[:2], [2, 1], num_populations=2, max_nodes=30,
                                   migration_period=2, migration_percentage=0.125, elite_percentage=0.125,
                                   verbose=False, evolve_backend=backend)
        pops = gp.initialize_population(0)
        fit = np.random.default_rng(1).random((2, 32)).astype(np.float32)
        out = gp.evolve(pops, fit, 3)
        assert out.shape == pops.shape and gp.current_generation == 1
        _check_pop(out, gp.library)
    with pytest.raises(ValueError):
        mt.GeneticProgramming(2, 32, ff, ops, VARS[:2], [1, 1], max_nodes=30, migration_percentage=0.125, elite_percentage=0.125,
                              verbose=False, evolve_backend="jax")


def test_evolve_never_overwrites_a_population_the_caller_holds():
    """HostEvolver reuses a returned population's buffer only once nothing outside references it:
    populations (or views of them) the caller keeps are never overwritten by later generations."""
    from helpers import CONTROL_OPS
    import multitreegp_amd as mt
    env = mt.Acrobot(0, 0)
    lib_vars = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
    ff = mt.DynamicEvaluator(env, 2, 0.05)
    gp = mt.GeneticProgramming(10, 20, ff, CONTROL_OPS, lib_vars, [2, 1], migration_percentage=0.5,
                               elite_percentage=0.0, verbose=False)
    pop = gp.initialize_population(3)
    fit = np.random.default_rng(0).random((1, 20)).astype(np.float32)
    import torch
    kept, snaps = [], []
    cur = pop
    for g in range(10):
        cur = gp.evolve(cur, fit, 100 + g)
        if g % 2 == 0:  # keep every other generation, through the kinds of view a caller makes
            hold = {0: lambda a: a, 2: lambda a: a.reshape(-1), 4: lambda a: np.asarray(a)[:, 1:][0],
                    6: lambda a: torch.from_numpy(a), 8: lambda a: memoryview(a)}[g](cur)
            kept.append(hold)
            snaps.append(cur.copy())
    for k, s in zip(kept, snaps):
        a = k.numpy() if isinstance(k, torch.Tensor) else np.asarray(k)
        assert np.array_equal(a.reshape(-1), (s[:, 1:][0] if a.size != s.size else s).reshape(-1))
    # a released population is reused (no fresh allocation once the loop has warmed up)
    blocks = set()
    cur = None
    for g in range(6):
        cur = gp.evolve(pop, fit, 200 + g)
        blocks.add(cur.ctypes.data)
        cur = None
    assert len(blocks) <= 2


@pytest.mark.parametrize("rtp,digests", [
    ((1.0, 0.0, 0.0), ("cf77ed59b80e2aff", "e2e8ed97af983120", "35a8bb31cd0a003c")),
    ((0.9, 0.1, 0.0), ("f02b338a65b441b4", "993f7c2cb0397115", "4fbf6b2af620dfbe")),
])
def test_evolve_golden_digest(rtp, digests):
    """Pins the native evolution step bit for bit (the crossover's scan / splice_rows /
    choose_prefix path): sha256 prefixes of three generations from fixed seeds -- all crossover,
    and crossover + mutation, with ring migration every generation.  Recorded from the round-4
    library (the crossover rewrite), so any later change to the draws or the splice shows here."""
    import hashlib
    ev = _evolver(_lib(), rtp=rtp, num_pop=2, migration_size=2, period=1)
    pop = ev.sample_population(64, 7)
    fit = np.random.default_rng(3).random((2, 64)).astype(np.float32)
    for g in range(3):
        pop = ev.evolve(pop, fit, 11 + g, g)
        assert hashlib.sha256(np.ascontiguousarray(pop).tobytes()).hexdigest()[:16] == digests[g], g
