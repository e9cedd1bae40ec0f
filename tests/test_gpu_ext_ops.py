"""The round-3 unary operators (exp, log, sqrt, tanh, abs; node_library.SUPPORTED_OPERATORS) on
the GPU.  Since round 4 the program JIT translates them (exp / log / tanh / sqrt as shared
machine-code subroutines, abs inline; scripts/gen_jit_templates.py), so populations that use
them run JIT code: fitness, per-rollout fitness, trajectories and coefficient gradients must
equal the oracle bit for bit (shared f32 specs in include/mtgp_f32math.h, tangent rules in
include/mtgp_dual.h), and the JIT must equal the evaluators' interpreter (MTGP_JIT=0 path)."""
import numpy as np
import pytest
import torch

import multitreegp_amd as mt
from multitreegp_amd import coefficients as co
from multitreegp_amd.engine import DeviceEngine, to_reference_layout
from multitreegp_amd.sampling import sample_population
from oracle import oracle as orc
from helpers import (CONTROL_OPS, SR_OPS, bits_equal, dynamic_setup, mismatch_report, oracle_model, oracle_rollouts,
                     sr_setup, static_setup, tree_from_expr)

pytestmark = pytest.mark.gpu

EXT = [("exp", None, 1, 0.15), ("log", None, 1, 0.15), ("sqrt", None, 1, 0.15), ("tanh", None, 1, 0.15),
       ("abs", None, 1, 0.15)]


def _ext_lib(lib, ops):
    return mt.NodeLibrary(ops + EXT, lib.variable_list, lib.layer_sizes)


def _run(ff, lib, data, pop, traj=True, jit=True):
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=jit)
    pt = torch.from_numpy(np.ascontiguousarray(pop)).cuda()
    eng.prepare_data(data)  # (the SR evaluator learns n_var from the data)
    fl = eng.flatten(pt)
    res = eng.evaluate(pt, data, flattened=fl, trajectories=traj, rollout_fitness=True)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(fl) == jit  # the JIT code ran (round 4: no opcode declines)
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=traj)
    return res, ref, d


def _check(res, ref, P, R, names):
    for k in ("fitness", "rollout_fitness"):
        got = res[k].cpu().numpy()
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)
    for k in names:
        got = to_reference_layout(res[k], P, R)
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)


def _uses_ext(lib, pop):
    codes = [lib.string_to_node[n] for n, *_ in EXT]
    return bool(np.isin(pop[..., 0], codes).any())


@pytest.mark.parametrize("kind", ["dynamic", "static_noise", "dynamic_dopri5"])
def test_gpu_control_with_extended_operators(kind):
    solver = (1e-4, 1e-4, 0.001, 300) if kind == "dynamic_dopri5" else None
    if kind.startswith("dynamic"):
        env, lib0, ff, data, _ = dynamic_setup(P=32, R=8, n_steps=40, solver=solver)
        names = ("xs", "ys", "us", "acts")
    else:
        env, lib0, ff, data, _ = static_setup(P=32, R=8, n_steps=40, obs_noise=0.1)
        names = ("xs", "ys", "us")
    lib = _ext_lib(lib0, CONTROL_OPS)
    pop = sample_population(21, lib, 32, 1, max_init_depth=6, max_nodes=40)[0]
    assert _uses_ext(lib, pop)
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, 32, d["R"], names)


@pytest.mark.parametrize("n_var", [2, 6])
def test_gpu_sr_with_extended_operators(n_var):
    env, lib0, ff, data, _ = sr_setup(P=24, R=8, n_var=n_var)
    lib = _ext_lib(lib0, SR_OPS)
    pop = sample_population(22, lib, 24, 1, max_init_depth=5, max_nodes=30)[0]
    assert _uses_ext(lib, pop)
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, 24, d["R"], ("xs",))


def test_gpu_tree_evaluator_with_extended_operators():
    """the tree_evaluator plugin (gp.py:390-401 vmap_foriloop) on trees using the new operators"""
    lib = mt.NodeLibrary(SR_OPS + EXT, [["x0", "x1", "x2"]], [2])
    pop = sample_population(23, lib, 40, 1, max_init_depth=6, max_nodes=30)[0]
    assert _uses_ext(lib, pop)
    te = mt.genetic_programming.TreeEvaluator(lib, 30, "cuda:0")
    rng = np.random.default_rng(3)
    for p in range(0, 40, 5):
        x = (rng.standard_normal(3) * 2).astype(np.float32)
        got = np.asarray(te(pop[p], x), np.float32).reshape(-1)
        want = np.array([orc.eval_tree(pop[p, t], lib.fn_codes, lib.n_funcs, lib.var_start, x) for t in range(2)],
                        np.float32)
        assert bits_equal(got, want), (p, got, want)


def test_gpu_sr_grad_with_extended_operators():
    env, lib0, ff, data, _ = sr_setup(P=20, R=4, n_save=9, save_every=2, h=0.05, depth=4, N=20, seed=4)
    lib = _ext_lib(lib0, SR_OPS)
    pop = sample_population(24, lib, 20, 1, max_init_depth=4, max_nodes=20)[0]
    assert _uses_ext(lib, pop)
    d = ff.prepare(data)
    d["h"] = ff.dt0
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    loss, grads = co.CoefficientOptimiser(eng).loss_and_grad(pop, data)
    rl, rg, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert bits_equal(loss, rl), mismatch_report(loss, rl, "loss")
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), p


# Edge cases of every template: zeros of both signs, subnormals, the exp limits (88.7228394,
# -103.972084) and their neighbours, tanh's 0.625 branch point, 2|x| past the exp overflow,
# infinities and NaN, large magnitudes, ordinary values.
EDGE = np.array([0.0, -0.0, 1e-40, -1e-40, 1.17549435e-38, 3e-39, 1e-30, 0.5, 0.625, -0.625, 0.62499994, 1.0, -1.0,
                 88.7228394, 88.72284, -103.972084, -103.97209, 44.4, -44.4, 1e10, -1e10, 3.4e38, np.inf, -np.inf,
                 np.nan, 2.0, 7.5, -0.3, 1e-7, 123.25, -2.5, 0.1], np.float32)


def _edge_population(lib, n_var, N=20):
    x = [f"x{i}" for i in range(n_var)]
    exprs = [("exp", x[0]), ("log", x[0]), ("sqrt", x[0]), ("tanh", x[0]), ("abs", x[0]),
             ("tanh", ("*", x[0], 0.5)), ("log", ("abs", x[0])), ("sqrt", ("abs", x[0])), ("exp", ("-", 0.0, x[0])),
             ("tanh", ("exp", x[0])), ("+", ("log", ("sqrt", ("abs", x[0]))), ("tanh", x[0])),
             ("*", ("exp", ("tanh", x[0])), ("abs", ("log", x[0]))), ("/", ("sqrt", x[0]), ("exp", x[0]))]
    def on(e, v):  # the expression with x0 replaced by variable v
        if isinstance(e, tuple):
            return (e[0],) + tuple(on(c, v) for c in e[1:])
        return v if e == x[0] else e

    pop = np.zeros((len(exprs), n_var, N, 4), np.float32)
    for i, e in enumerate(exprs):
        for t in range(n_var):  # tree t: the expression on x_t (same ops, another state component)
            pop[i, t] = tree_from_expr(on(e, x[t]), lib, N)
    return pop


@pytest.mark.parametrize("n_var", [2, 6])
def test_gpu_jit_templates_edge_values_match_interpreter_and_oracle(n_var):
    """exp / log / sqrt / tanh / abs JIT subroutines = the interpreter = the oracle, bit for bit, on
    the edge values of their specs (first RK4 stage of every rollout evaluates them at x0 = EDGE;
    the trajectory carries the results on)."""
    R = len(EDGE)
    env, lib0, ff, data, _ = sr_setup(P=4, R=R, n_var=n_var, n_save=3, save_every=1, h=0.01)
    lib = _ext_lib(lib0, SR_OPS)
    x0 = np.stack([np.roll(EDGE, k) for k in range(n_var)], axis=1).astype(np.float32)
    data = (x0,) + tuple(data[1:])
    pop = _edge_population(lib, n_var)
    P = pop.shape[0]
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, P, d["R"], ("xs",))
    res_i, _, _ = _run(ff, lib, data, pop, jit=False)
    for k in ("fitness", "rollout_fitness"):
        a, b = res[k].cpu().numpy(), res_i[k].cpu().numpy()
        assert bits_equal(a, b), mismatch_report(a, b, k + " (JIT vs interpreter)")
    a, b = to_reference_layout(res["xs"], P, d["R"]), to_reference_layout(res_i["xs"], P, d["R"])
    assert bits_equal(a, b), mismatch_report(a, b, "xs (JIT vs interpreter)")
