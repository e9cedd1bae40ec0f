"""GPU tests of the drop-in API (GeneticProgramming facade, evaluators, tree_evaluator) and of
edge cases through the full fused RK4 kernel, against the CPU oracle."""
import numpy as np
import pytest
import torch

import multitreegp_amd as mt
from multitreegp_amd.engine import DeviceEngine
from multitreegp_amd.sampling import sample_population
from oracle import oracle as orc
from helpers import (CONTROL_OPS, SR_OPS, bits_equal, dynamic_setup, mismatch_report, oracle_model, oracle_rollouts,
                     sr_setup, static_setup)

pytestmark = pytest.mark.gpu


def test_genetic_programming_evaluate_population():
    env = mt.Acrobot(0.0, 0.0)
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4())
    gp = mt.GeneticProgramming(3, 20, ff, CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]],
                               [2, 1], num_populations=3, size_parsinomy=0.5, max_nodes=30, verbose=False)
    pops = gp.initialize_population(4)
    assert pops.shape == (3, 20, 3, 30, 4)
    data = mt.control_data(env, 16, 0.05, None, seed=2, n_steps=60)
    fit, pops_out = gp.evaluate_population(pops, data)
    assert fit.shape == (3, 20) and pops_out.shape == pops.shape
    d = ff.prepare(data)
    ref = orc.evaluate(oracle_model(ff, d, 0.5), pops.reshape(60, 3, 30, 4), gp.library, oracle_rollouts(d))
    assert bits_equal(fit.reshape(-1), ref["fitness"])
    best, sol = gp.get_statistics(0)
    assert best == fit.min() and np.array_equal(sol, pops.reshape(60, 3, 30, 4)[np.argmin(fit)])
    assert isinstance(gp.to_string(sol), str)


def test_evaluate_candidate_and_call():
    env, lib, ff, data, pop = dynamic_setup(P=3, R=8, n_steps=40)
    gp_eval = mt.TreeEvaluator(lib, 40)
    xs, ys, us, acts, fit = ff.evaluate_candidate(pop[1], data, gp_eval)
    d = ff.prepare(data)
    ref = orc.evaluate(oracle_model(ff, d), pop[1:2], lib, oracle_rollouts(d), trajectories=True)
    assert xs.shape == (8, 41, 4) and us.shape == (8, 41, 1) and acts.shape == (8, 41, 2)
    assert bits_equal(xs, ref["xs"][0]) and bits_equal(ys, ref["ys"][0]) and bits_equal(us, ref["us"][0])
    assert bits_equal(acts, ref["acts"][0]) and bits_equal(fit, ref["rollout_fitness"][0])
    f = ff(pop[1][..., 3:], pop[1][..., :3], data, gp_eval)
    assert np.float32(f) == ref["fitness"][0]


def test_tree_evaluator_matches_body_fun():
    env, lib, ff, data, pop = dynamic_setup(P=2)
    te = mt.TreeEvaluator(lib, 40)
    d = np.random.default_rng(0).standard_normal(7).astype(np.float32)
    got = te(pop[0], d)
    want = np.array([orc.eval_tree(pop[0, t], lib.fn_codes, lib.n_funcs, lib.var_start, d) for t in range(3)])
    assert bits_equal(got, want)


def test_garbage_population_through_rk4():
    """Arbitrary row arrays (bad opcodes, wrapped indices, forward references) in the full
    dynamic evaluator: every flattenable individual must match the oracle bit-for-bit."""
    env, lib, ff, data, _ = dynamic_setup(P=2, R=8, n_steps=30)
    rng = np.random.default_rng(3)
    P, N = 64, 16
    pop = np.empty((P, 3, N, 4), np.float32)
    pop[..., 0] = rng.integers(-1, lib.n_funcs + 2, (P, 3, N))
    pop[..., 1] = rng.integers(-N - 2, N + 2, (P, 3, N))
    pop[..., 2] = rng.integers(-N - 2, N + 2, (P, 3, N))
    pop[..., 3] = rng.standard_normal((P, 3, N))
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, rollout_fitness=True, check=False)
    ok = (res["_flat"].status.cpu().numpy() == 0).all(axis=1)
    assert ok.sum() > 40
    d = ff.prepare(data)
    ref = orc.evaluate(oracle_model(ff, d), pop[ok], lib, oracle_rollouts(d))
    assert bits_equal(res["fitness"].cpu().numpy()[ok], ref["fitness"])


def test_deep_sr_trees_and_wide_state():
    """4-dim SR, max_nodes 128, depth up to 9 (stack > 1, long programs)."""
    env, lib, ff, data, pop = sr_setup(P=24, R=8, n_save=11, save_every=2, depth=9, N=128, n_var=4)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True)
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    assert bits_equal(res["fitness"].cpu().numpy(), ref["fitness"])
    assert bits_equal(res["rollout_fitness"].cpu().numpy(), ref["rollout_fitness"])


def test_population_not_multiple_of_pack():
    """P = 13 with R = 16 (4 individuals per wave): last wave partially filled."""
    env, lib, ff, data, pop = static_setup(P=13, R=16, n_steps=30)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", lanes=0)
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, rollout_fitness=True)
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert bits_equal(res["fitness"].cpu().numpy(), ref["fitness"])


def test_kernel_timing_history():
    """mtgp_kernel_ms_history: the durations of the last n timed evaluator launches, oldest first,
    read with one synchronisation after the run (bench.py's timed loop never stalls the queue)."""
    import ctypes
    env, lib, ff, data, pop = dynamic_setup(P=16, R=8, n_steps=40)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    nat_lib = eng.native
    nat_lib.mtgp_set_timing(1)
    try:
        pd = torch.from_numpy(pop).cuda()
        for _ in range(3):
            eng.evaluate(pd, data, check=False)
        out = (ctypes.c_float * 5)()
        assert nat_lib.mtgp_kernel_ms_history(out, 3) == 3
        ms = list(out)[:3]
        assert all(m > 0 for m in ms)
        assert ms[-1] == nat_lib.mtgp_last_kernel_ms()
        assert 3 <= nat_lib.mtgp_kernel_ms_history(out, 5) <= 5
    finally:
        nat_lib.mtgp_set_timing(0)
