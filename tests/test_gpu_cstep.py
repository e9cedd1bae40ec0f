"""GPU parity of the fixed-step solve under diffrax.ConstantStepSize semantics (ABI v18,
include/mtgp_cstep.h): accumulated f32 step ends, per-step dt, and SaveAt(ts) for ANY non-decreasing
ts through the solver's dense output.  Every kernel family (the JIT-only dynamic / static loops,
their interpreter fallbacks, the runtime state-size kernel, the Acrobot cost-mask kernels, the
register and wide-state SR kernels, the coefficient-optimisation sensitivities) is compared bit for
bit with the oracle on save grids that are not step ends: the notebooks' grid arange(0, T, 0.2) with
dt0 0.05 (DynamicPolicy.ipynb:55), ts not a multiple of dt0, non-uniform ts, an offset start, a
tiny last step, repeated save times, and a max_steps cut."""
import numpy as np
import pytest
import torch

import multitreegp_amd as mt
from multitreegp_amd.engine import DeviceEngine, to_reference_layout
from oracle import oracle as orc
from helpers import (bits_equal, dynamic_setup, mismatch_report, oracle_model, oracle_rollouts, sr_setup,
                     static_setup)

pytestmark = pytest.mark.gpu

GRIDS = {
    "notebook": (lambda: np.arange(0, 50, 0.2).astype(np.float32), 0.05),
    "off_multiple": (lambda: np.arange(0, 6, 0.03).astype(np.float32), 0.05),
    "nonuniform": (lambda: np.concatenate([[0.0], np.sort(np.random.default_rng(1).uniform(0, 4, 30))]).astype(np.float32),
                   0.07),
    "offset": (lambda: (np.float32(1.0) + np.arange(30, dtype=np.float32) * np.float32(0.1)).astype(np.float32), 0.04),
    "tiny_last": (lambda: (np.arange(201, dtype=np.float32) * np.float32(0.01)).astype(np.float32), 0.01),
    "repeats": (lambda: np.array([0, 0, 0.5, 0.5, 0.5, 1.3, 2.0, 2.0, 2.45], np.float32), 0.25),
}


def _with_ts(data, ts):
    return (data[0], ts) + tuple(data[2:])


def _run(ff, lib, data, pop, jit=True, traj=True, parsimony=0.25):
    eng = DeviceEngine(ff, lib, parsimony, "cuda:0", jit=jit)
    res = eng.evaluate(torch.from_numpy(np.ascontiguousarray(pop)).cuda(), data, trajectories=traj,
                       rollout_fitness=True)
    torch.cuda.synchronize()
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d, parsimony), pop, lib, oracle_rollouts(d), trajectories=traj)
    return res, ref, d


def _check(res, ref, P, R, names):
    for k in ("fitness", "rollout_fitness"):
        got = res[k].cpu().numpy()
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)
    for k in names:
        got = to_reference_layout(res[k], P, R)
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)


CONTROL_CASES = ["dynamic", "dynamic_interp", "dynamic_euler", "dynamic_noise", "dynamic_ss5", "static",
                 "static_noise", "harmonic_dynamic", "reactor_static"]


def _control(case, grid):
    make_ts, dt0 = GRIDS[grid]
    ts = make_ts()
    kw = dict(P=20, R=8, n_steps=10, seed=21, h=dt0)
    solver_euler = None
    if case in ("dynamic", "dynamic_interp", "dynamic_euler"):
        env, lib, ff, data, pop = dynamic_setup(depth=8, N=48, **kw)
        if case == "dynamic_euler":
            ff = mt.DynamicEvaluator(env, 2, dt0, solver=mt.Euler())
            solver_euler = True
        names = ["xs", "ys", "us", "acts"]
    elif case == "dynamic_noise":
        env, lib, ff, data, pop = dynamic_setup(depth=8, N=48, obs_noise=0.1, **kw)
        names = ["xs", "ys", "us", "acts"]
    elif case == "dynamic_ss5":
        env, lib, ff, data, pop = dynamic_setup(depth=5, N=30, state_size=5, **kw)
        names = ["xs", "us", "acts"]
    elif case == "static":
        env, lib, ff, data, pop = static_setup(**kw)
        names = ["xs", "ys", "us"]
    elif case == "static_noise":
        env, lib, ff, data, pop = static_setup(obs_noise=0.1, **kw)
        names = ["xs", "ys", "us"]
    elif case == "harmonic_dynamic":
        env, lib, ff, data, pop = dynamic_setup(env="harmonic", state_size=1, **kw)
        names = ["xs", "ys", "us", "acts"]
    else:
        env, lib, ff, data, pop = static_setup(env="reactor", **kw)
        names = ["xs", "ys", "us"]
    del solver_euler
    return ff, lib, _with_ts(data, ts), pop, names


@pytest.mark.parametrize("grid", sorted(GRIDS))
@pytest.mark.parametrize("case", CONTROL_CASES)
def test_control_constant_step_bitexact(case, grid):
    # "repeats" (ts[1] == ts[0]) on Acrobot: acrobot.py:82's 0 / 0 ratio keeps the costs at ts_k = 0,
    # +inf masks the rest -- the general mask table (evaluators.acrobot_mask), no skip
    ff, lib, data, pop, names = _control(case, grid)
    res, ref, d = _run(ff, lib, data, pop, jit=case != "dynamic_interp")
    assert d["n_steps"] == orc.cs_steps(d["ts"], ff.dt0)
    _check(res, ref, pop.shape[0], 8, names)


@pytest.mark.parametrize("grid", ["notebook", "nonuniform", "offset"])
@pytest.mark.parametrize("case", ["dynamic", "static", "harmonic_dynamic"])
def test_control_fitness_only_matches_trajectories(case, grid):
    """The fitness-only kernels (early exit once every lane is settled) equal the trajectory ones."""
    ff, lib, data, pop, _ = _control(case, grid)
    eng = DeviceEngine(ff, lib, 0.25, "cuda:0")
    pt = torch.from_numpy(pop).cuda()
    a = eng.evaluate(pt, data, trajectories=True, rollout_fitness=True)
    b = eng.evaluate(pt, data, trajectories=False, rollout_fitness=True)
    assert bits_equal(a["fitness"].cpu().numpy(), b["fitness"].cpu().numpy())


@pytest.mark.parametrize("solver", ["rk4", "euler"])
@pytest.mark.parametrize("grid", sorted(GRIDS))
@pytest.mark.parametrize("n_var", [2, 12])
def test_sr_constant_step_bitexact(n_var, grid, solver):
    make_ts, dt0 = GRIDS[grid]
    ts = make_ts()
    if grid == "notebook":
        ts = ts[:60]  # (t1 = 11.8: the SR trees diverge long before 50)
    env, lib, ff, data, pop = sr_setup(P=18, R=4, n_var=n_var, depth=6, N=48 if n_var > 4 else 30, seed=23, h=dt0)
    x0 = data[0]
    ys = mt.ground_truth(env, x0, ts)
    ff = mt.SREvaluator(solver=mt.Euler() if solver == "euler" else mt.RK4(), dt0=dt0)
    res, ref, d = _run(ff, lib, (x0, ts, ys, data[3]), pop)
    _check(res, ref, pop.shape[0], 4, ["xs"])


@pytest.mark.parametrize("case", ["dynamic", "static", "sr", "sr_wide"])
def test_max_steps_cut_bitexact(case):
    """max_steps bounds the ConstantStepSize solve too: the points after the cut are +inf."""
    if case in ("dynamic", "static"):
        setup = dynamic_setup if case == "dynamic" else static_setup
        env, lib, ff, data, pop = setup(P=20, R=8, n_steps=60, seed=24)
        ff = (mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4(), max_steps=37) if case == "dynamic"
              else mt.FeedforwardEvaluator(env, 0.05, solver=mt.RK4(), max_steps=37))
        names = ["xs", "us"]
    else:
        env, lib, ff, data, pop = sr_setup(P=18, R=4, n_var=2 if case == "sr" else 9, seed=24, n_save=21, save_every=4)
        ff = mt.SREvaluator(solver=mt.RK4(), dt0=0.05, max_steps=37)
        names = ["xs"]
    res, ref, d = _run(ff, lib, data, pop)
    assert d["max_steps"] == 37 and d["n_steps"] == 37
    _check(res, ref, pop.shape[0], data[0].shape[0], names)
    xs = ref["xs"]
    assert np.isposinf(xs[:, :, -1]).all()


@pytest.mark.parametrize("kind", ["sr", "dynamic", "static"])
def test_gradients_constant_step_bitexact(kind):
    """Coefficient-optimisation sensitivities (mtgp_sr_grad / mtgp_ctl_grad) on a non-uniform save
    grid: loss and gradient equal the oracle's dual-number restatement of the same solve."""
    from multitreegp_amd import coefficients as co
    make_ts, dt0 = GRIDS["nonuniform"]
    ts = make_ts()[:16]
    if kind == "sr":
        env, lib, ff, data, pop = sr_setup(P=12, R=4, depth=4, N=20, seed=25, h=dt0)
        data = (data[0], ts, mt.ground_truth(env, data[0], ts), data[3])
        ff = mt.SREvaluator(solver=mt.RK4(), dt0=dt0)
    else:
        setup = dynamic_setup if kind == "dynamic" else static_setup
        env, lib, ff, data, pop = setup(P=12, R=3, n_steps=10, seed=25, h=dt0, env="harmonic")
        data = _with_ts(data, ts)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    d = eng.prepare_data(data)
    loss, grads = co.CoefficientOptimiser(eng).loss_and_grad(pop, data)
    fn = orc.sr_grad if kind == "sr" else orc.ctl_grad
    rl, rg, rows = fn(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert sum(len(r) for r in rows) > 5
    assert bits_equal(loss, rl), mismatch_report(loss, rl, "loss")
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), mismatch_report(g, rg[p, : len(g)], f"grad {p}")
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit), mismatch_report(loss, fit, "fitness")


@pytest.mark.parametrize("solver", ["rk4", "dopri5"])
def test_nonfinite_stage_zero_tableau_entries(solver):
    """A stage derivative that is +inf only at one stage (dx0 = 1 / (x1 - 0.25) from x1 = 0.25): the
    zero tableau entries multiply it into the later stage inputs as NaN (mtgp_cstep.h /
    mtgp_dopri5.h, diffrax's padded-row dot product) -- GPU bit-exact vs the oracle, trajectories
    included; RK4: x1's save at the event step is NaN."""
    from test_oracle import _nonfinite_stage_candidate
    lib, cand = _nonfinite_stage_candidate()
    pop = np.repeat(cand, 4, axis=0)
    R = 4
    x0 = np.tile(np.array([[1.0, 0.25]], np.float32), (R, 1))
    x0[1:, 0] += np.float32(0.5)  # (the singularity sits in x1: every rollout meets it)
    ts = (np.arange(10, dtype=np.float32) * np.float32(0.1)).astype(np.float32)
    data = (x0, ts, np.zeros((10, 2, R), np.float32).transpose(2, 0, 1).copy(), np.zeros((R, 2), np.uint32))
    if solver == "rk4":
        ff = mt.SREvaluator(solver=mt.RK4(), dt0=0.1)
    else:
        ff = mt.SREvaluator(solver=mt.Dopri5(), dt0=0.1, max_steps=200,
                            stepsize_controller=mt.PIDController(rtol=1e-4, atol=1e-4, dtmin=0.001))
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, pop.shape[0], R, ["xs"])
    if solver == "rk4":
        xs = to_reference_layout(res["xs"], pop.shape[0], R)
        assert np.isnan(xs[0, 0, 1, 1])
