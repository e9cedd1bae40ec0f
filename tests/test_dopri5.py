"""Adaptive Dopri5 + PIDController (spec include/mtgp_dopri5.h).

diffrax is not importable here and the reference holds no solver fixtures, so the restatement is
pinned by known answers (the harmonic oscillator's closed form), by scipy's independent
Dormand-Prince RK45 (same tableau and error estimate, its own controller and interpolant) and by
the controller's documented edge behaviour; the GPU kernel must then match the oracle bit for bit
(parity vs diffrax itself: unpinned)."""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd.evaluators import _check_solver
from oracle import oracle as orc

from helpers import SR_OPS, oracle_model, oracle_rollouts, sr_setup


def _oscillator(N=4):
    """trees [x1, 0 - x0]: dx0 = x1, dx1 = -x0 (tests/test_oracle.py's RK4 known answer)."""
    lib = mt.NodeLibrary(SR_OPS, [["x0", "x1"]], [2])
    cand = np.zeros((1, 2, N, 4), np.float32)
    cand[..., 1:3] = -1
    cand[0, 0, N - 1] = [lib.string_to_node["x1"], -1, -1, 0]
    cand[0, 1, N - 3] = [lib.string_to_node["x0"], -1, -1, 0]
    cand[0, 1, N - 2] = [1, -1, -1, 0.0]
    cand[0, 1, N - 1] = [lib.string_to_node["-"], N - 2, N - 3, 0]
    return lib, cand


def _model(S, rtol, atol, dtmin=0.0, max_steps=1000, h=0.01, dtmax=0.0):
    return dict(model=3, n_var=2, state_size=0, n_obs=0, n_control=0, n_targets=0, n_steps=0, save_every=1,
                n_save=S, h=h, max_fitness=1e5, parsimony=0.0, solver=1, max_steps=max_steps, rtol=rtol,
                atol=atol, dtmin=dtmin, dtmax=dtmax)


X0 = np.array([[1.0, 0.0], [0.3, -0.7], [-2.0, 1.5]], np.float32)
TS = (np.arange(101) * np.float32(0.2)).astype(np.float32)  # SymbolicRegression.ipynb:51 save grid


def _exact(x0, t):
    t = t.astype(np.float64)
    return np.stack([x0[:, :1] * np.cos(t) + x0[:, 1:] * np.sin(t),
                     -x0[:, :1] * np.sin(t) + x0[:, 1:] * np.cos(t)], -1)


@pytest.mark.parametrize("tol,atol_err", [(1e-6, 2e-5), (1e-4, 4e-3)])
def test_dopri5_oscillator_known_answer(tol, atol_err):
    lib, cand = _oscillator()
    out = orc.evaluate(_model(len(TS), tol, tol, dtmin=0.001), cand, lib,
                       dict(x0=X0, ts=TS, ys_true=np.zeros((3, len(TS), 2), np.float32)), trajectories=True)
    xs = out["xs"][0]
    assert np.all(xs[:, 0] == X0)  # SaveAt ts[0] = y0 exactly
    np.testing.assert_allclose(xs, _exact(X0, TS), atol=atol_err)


def _pid_model(S, tol, pid, dtmin=0.0, max_steps=4000):
    m = _model(S, tol, tol, dtmin=dtmin, max_steps=max_steps)
    m.update(pid.model_fields())
    return m


@pytest.mark.parametrize("coeffs", [dict(pcoeff=0.3, icoeff=0.4), dict(pcoeff=0.2, icoeff=0.5, dcoeff=0.1),
                                    dict(icoeff=1.0, safety=0.8, factormin=0.3, factormax=5.0)])
def test_dopri5_general_pid_known_answer(coeffs):
    """PI / PID controllers (diffrax.PIDController coefficients) on the closed-form oscillator:
    accurate to the tolerance scale, and (PI) a different step sequence from the integral default."""
    lib, cand = _oscillator()
    ro = dict(x0=X0, ts=TS, ys_true=np.zeros((3, len(TS), 2), np.float32))
    pid = mt.PIDController(rtol=1e-6, atol=1e-6, dtmin=0.001, **coeffs)
    out = orc.evaluate(_pid_model(len(TS), 1e-6, pid, dtmin=0.001), cand, lib, ro, trajectories=True)
    np.testing.assert_allclose(out["xs"][0], _exact(X0, TS), atol=5e-5)
    base = orc.evaluate(_model(len(TS), 1e-6, 1e-6, dtmin=0.001), cand, lib, ro, trajectories=True)
    assert not np.array_equal(out["xs"], base["xs"])  # the controller changed the steps


def test_dopri5_default_pid_fields_are_the_default_controller():
    """Explicit default coefficients map to pid_custom = 0: the round-1 controller bit for bit."""
    lib, cand = _oscillator()
    ro = dict(x0=X0, ts=TS, ys_true=np.zeros((3, len(TS), 2), np.float32))
    pid = mt.PIDController(rtol=1e-4, atol=1e-4, pcoeff=0.0, icoeff=1.0, dcoeff=0.0, dtmin=0.001)
    a = orc.evaluate(_pid_model(len(TS), 1e-4, pid, dtmin=0.001), cand, lib, ro, trajectories=True)
    b = orc.evaluate(_model(len(TS), 1e-4, 1e-4, dtmin=0.001), cand, lib, ro, trajectories=True)
    assert np.array_equal(a["xs"].view(np.uint32), b["xs"].view(np.uint32))


def test_dopri5_force_dtmin_false_ends_the_solve():
    """force_dtmin=False: once the controller asks for a step below dtmin the solve stops
    (diffrax RESULTS.dt_min_reached; with throw=False the remaining save points are +inf), while
    force_dtmin=True keeps stepping at dtmin.  dx = x * x blows up at t = 1 for x0 = 1."""
    lib = mt.NodeLibrary(SR_OPS, [["x0"]], [1])
    N = 3
    cand = np.zeros((1, 1, N, 4), np.float32)
    cand[..., 1:3] = -1
    cand[0, 0, N - 2] = [lib.string_to_node["x0"], -1, -1, 0]
    cand[0, 0, N - 1] = [lib.string_to_node["*"], N - 2, N - 2, 0]
    x0 = np.array([[1.0], [0.1]], np.float32)
    ts = (np.arange(21) * np.float32(0.1)).astype(np.float32)
    ro = dict(x0=x0, ts=ts, ys_true=np.zeros((2, len(ts), 1), np.float32))
    outs = {}
    for force in (True, False):
        pid = mt.PIDController(rtol=1e-6, atol=1e-6, dtmin=0.01, force_dtmin=force)
        m = _pid_model(len(ts), 1e-6, pid, dtmin=0.01, max_steps=4000)
        m["n_var"] = 1
        outs[force] = orc.evaluate(m, cand, lib, ro, trajectories=True)["xs"][0, :, :, 0]
    soft, hard = outs[False], outs[True]
    np.testing.assert_allclose(soft[1], hard[1])  # the smooth rollout never needs dtmin
    stop = int(np.argmax(np.isinf(soft[0])))
    assert 0 < stop < len(ts) - 1 and np.isinf(soft[0, stop:]).all() and np.isfinite(soft[0, :stop]).all()
    assert np.isfinite(hard[0, :stop + 1]).all()  # forced steps go on past the point where the soft solve gave up


def test_dopri5_vs_scipy_rk45():
    """scipy's RK45 is the same Dormand-Prince pair with an integral controller of the same
    exponent (-1/5), safety and clip range; step sequences and interpolants differ in detail, so
    the saved trajectories agree to the tolerance scale, not bit for bit."""
    from scipy.integrate import solve_ivp
    lib, cand = _oscillator()
    tol = 1e-6
    out = orc.evaluate(_model(len(TS), tol, tol, dtmin=0.001), cand, lib,
                       dict(x0=X0, ts=TS, ys_true=np.zeros((3, len(TS), 2), np.float32)), trajectories=True)
    for r in range(3):
        sol = solve_ivp(lambda t, x: [x[1], -x[0]], (0.0, float(TS[-1])), X0[r].astype(np.float64), method="RK45",
                        t_eval=TS.astype(np.float64), rtol=tol, atol=tol, first_step=0.01)
        np.testing.assert_allclose(out["xs"][0, r], sol.y.T, atol=5e-5)


def test_dopri5_max_steps_leaves_inf_and_max_fitness():
    lib, cand = _oscillator()
    out = orc.evaluate(_model(len(TS), 1e-9, 1e-9, max_steps=20), cand, lib,
                       dict(x0=X0, ts=TS, ys_true=np.zeros((3, len(TS), 2), np.float32)), trajectories=True)
    xs = out["xs"][0]
    assert np.isinf(xs[:, -1]).all()  # t_end never reached within 20 attempts
    assert np.isfinite(xs[:, :2]).all()
    assert np.isinf(out["rollout_fitness"][0]).all()
    assert out["fitness"][0] == np.float32(1e5)


def test_dopri5_force_dtmin_equals_fixed_dtmin_steps():
    """With an unreachable tolerance every attempt is rejected down to dtmin, then force_dtmin
    accepts: the solve is fixed-step Dopri5 at dtmin after the first shrinking attempts, so it is
    still close to the exact solution and uses far fewer attempts than the tolerance would."""
    lib, cand = _oscillator()
    ts = (np.arange(11) * np.float32(0.2)).astype(np.float32)
    out = orc.evaluate(_model(len(ts), 0.0, 1e-30, dtmin=0.01, max_steps=400), cand, lib,
                       dict(x0=X0, ts=ts, ys_true=np.zeros((3, len(ts), 2), np.float32)), trajectories=True)
    xs = out["xs"][0]
    assert np.isfinite(xs).all()
    np.testing.assert_allclose(xs, _exact(X0, ts), atol=1e-5)


def test_dopri5_event_terminates_on_blow_up():
    """dx = x * x blows up in finite time 1/x0: Event(cond_fn_nan) (SR_evaluator.py:93-94) stops
    the solve after the first accepted non-finite state; later save points are +inf."""
    lib = mt.NodeLibrary(SR_OPS, [["x0"]], [1])
    N = 3
    cand = np.zeros((1, 1, N, 4), np.float32)
    cand[..., 1:3] = -1
    cand[0, 0, N - 2] = [lib.string_to_node["x0"], -1, -1, 0]
    cand[0, 0, N - 1] = [lib.string_to_node["*"], N - 2, N - 2, 0]
    x0 = np.array([[1.0], [0.1]], np.float32)
    ts = (np.arange(21) * np.float32(0.1)).astype(np.float32)
    m = _model(len(ts), 1e-4, 1e-4, dtmin=0.001, max_steps=2000)
    m["n_var"] = 1
    out = orc.evaluate(m, cand, lib, dict(x0=x0, ts=ts, ys_true=np.zeros((2, len(ts), 1), np.float32)),
                       trajectories=True)
    xs = out["xs"][0, :, :, 0]
    np.testing.assert_allclose(xs[1, :], 0.1 / (1 - 0.1 * ts), rtol=1e-3)  # no blow-up before t = 10
    assert np.isfinite(xs[0, :10]).all()  # 1 / (1 - t), t < 1
    np.testing.assert_allclose(xs[0, :10], 1.0 / (1.0 - ts[:10]), rtol=2e-3)
    assert np.isinf(xs[0, -1])
    assert out["fitness"][0] == np.float32((1e5 + out["rollout_fitness"][0, 1]) / 2)


def test_solver_selection_api():
    assert _check_solver(mt.RK4(), None) == "rk4"
    assert _check_solver("rk4", mt.ConstantStepSize()) == "rk4"
    pid = mt.PIDController(rtol=1e-6, atol=1e-6, dtmin=0.001)
    assert _check_solver(mt.Dopri5(), pid, adaptive_ok=True) == "dopri5"
    with pytest.raises(NotImplementedError):
        _check_solver(mt.Dopri5(), pid)  # callers that do not opt in
    with pytest.raises(NotImplementedError):
        _check_solver(mt.Dopri5(), None, adaptive_ok=True)
    pid2 = mt.PIDController(rtol=1e-3, atol=1e-3, pcoeff=0.3, icoeff=0.4)  # PI controllers run too (ABI v15)
    f = pid2.model_fields()
    assert f["pid_custom"] == 1 and f["pid_c1"] == np.float32(0.7 / 5) and f["pid_c2"] == np.float32(-0.3 / 5)
    assert mt.PIDController(rtol=1e-3, atol=1e-3).model_fields() == dict(no_force_dtmin=0, pid_custom=0)
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05, solver=mt.Dopri5(), stepsize_controller=mt.ConstantStepSize())
    env, lib, ff, data, pop = sr_setup(P=2, R=4, solver=(1e-6, 1e-6, 0.001, 500))
    d = ff.prepare(data)
    assert d["solver"] == 1 and d["max_steps"] == 500 and d["dtmin"] == np.float32(0.001)
    assert d["n_save"] == len(data[1])


def test_dopri5_sr_population_oracle_is_deterministic():
    """random reference-distribution trees (blow-ups, stiff candidates, early events): the
    population path runs and the per-lane controller gives finite or max fitness everywhere."""
    env, lib, ff, data, pop = sr_setup(P=16, R=4, seed=3, solver=(1e-6, 1e-6, 0.001, 500))
    d = ff.prepare(data)
    a = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    b = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    assert np.array_equal(a["fitness"].view(np.uint32), b["fitness"].view(np.uint32))
    assert np.all((a["fitness"] >= 0) & (a["fitness"] <= 1e5))


# ------------------------------------------------------------------ GPU parity (k_sr_dopri5)
def _gpu_run(ff, lib, data, pop, jit, traj=True, dp_budget=None, steps=False):
    import torch
    from multitreegp_amd.engine import DeviceEngine
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=jit, dp_budget=dp_budget)
    res = eng.evaluate(torch.from_numpy(np.ascontiguousarray(pop)).cuda(), data, trajectories=traj,
                       rollout_fitness=True, step_counts=steps)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(res["_flat"]) == jit
    return {k: v.cpu().numpy() for k, v in res.items() if isinstance(v, torch.Tensor)}, eng.prepare_data(data)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
@pytest.mark.parametrize("n_var,tol,R", [(2, 1e-6, 16), (2, 1e-4, 5), (1, 1e-5, 8), (3, 1e-6, 4), (4, 1e-5, 33)])
def test_gpu_dopri5_sr_bitexact(jit, n_var, tol, R):
    """Per-lane adaptive steps, rejections, forced dtmin steps, events and max_steps exits on
    reference-distribution random trees: fitness, per-rollout fitness and the SaveAt(ts)
    trajectories are bit-identical to the oracle."""
    from helpers import bits_equal, mismatch_report
    env, lib, ff, data, pop = sr_setup(P=37, R=R, n_save=26, save_every=4, h=0.01, seed=11 + n_var, n_var=n_var,
                                       solver=(tol, tol, 0.001, 300))
    res, d = _gpu_run(ff, lib, data, pop, jit)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, S = pop.shape[0], d["n_save"]
    xs = res["xs"].reshape(S, n_var, P, R).transpose(2, 3, 0, 1)  # time-major -> [P, R, S, n_var]
    assert bits_equal(xs, ref["xs"]), mismatch_report(xs, ref["xs"], "xs")


def test_dopri5_wide_sr_oracle_vs_fine_rk4():
    """The checker of the wide-state Dopri5 kernel: the oracle's adaptive solve of 12-variable SR
    candidates at a tight tolerance agrees with a fine fixed-step RK4 solve of the same trees
    wherever that solve is resolved (fp32 RK4 at h and h/2 agree to 2e-4: no near-singular division, no
    blow-up), and starts every trajectory at x0."""
    env, lib, ff, data, pop = sr_setup(P=16, R=3, n_save=11, save_every=4, h=0.01, depth=4, N=30, seed=2, n_var=12,
                                       solver=(1e-6, 1e-6, 0.0001, 2000))
    pop = pop.copy()
    pop[..., 0][pop[..., 0] == lib.string_to_node["/"]] = lib.string_to_node["*"]  # polynomial fields only:
    d = ff.prepare(data)                                  # a division by a vanishing state is unresolvable
    dp = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)["xs"]
    x0, ts, ys, keys = data

    def rk4(h):
        fine = mt.SREvaluator(solver=mt.RK4(), dt0=h)
        d2 = fine.prepare(data)
        return orc.evaluate(oracle_model(fine, d2), pop, lib, oracle_rollouts(d2), trajectories=True)["xs"]

    rk, rk2 = rk4(0.0005), rk4(0.00025)
    assert np.array_equal(dp[:, :, 0, :], np.broadcast_to(x0, dp[:, :, 0, :].shape))
    with np.errstate(all="ignore"):
        resolved = (np.isfinite(rk).all(axis=(1, 2, 3)) & (np.abs(rk).max(axis=(1, 2, 3)) < 1e3) &
                    (np.abs(rk - rk2) / (1e-3 + np.abs(rk2))).reshape(rk.shape[0], -1).max(axis=1).__lt__(2e-4))
        err = (np.abs(dp - rk) / (1e-3 + np.abs(rk))).reshape(dp.shape[0], -1).max(axis=1)
    assert resolved.sum() >= 3, resolved
    assert np.all(err[resolved] < 1e-3), (err, resolved)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
@pytest.mark.parametrize("n_var,tol,R,max_steps", [(5, 1e-5, 8, 300), (12, 1e-4, 4, 200), (64, 1e-4, 8, 150)])
def test_gpu_dopri5_wide_sr_bitexact(jit, n_var, tol, R, max_steps):
    """Wide-state SR (n_var > 4: the workgroup kernel, components spread over waves) with
    Dopri5 + PIDController: per-lane adaptive steps whose error norm, event and save points are
    reduced over all components -- fitness, per-rollout fitness, step counts and SaveAt(ts)
    trajectories bit-identical to the oracle, with the JIT (LDS-data code) and the interpreter."""
    import torch
    from helpers import bits_equal, mismatch_report
    from multitreegp_amd.engine import DeviceEngine
    env, lib, ff, data, pop = sr_setup(P=21, R=R, n_save=26, save_every=4, h=0.01, depth=8, N=64,
                                       seed=40 + n_var, n_var=n_var, solver=(tol, tol, 0.001, max_steps))
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=jit)
    r = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True, step_counts=True)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(r["_flat"]) == jit
    res = {k: v.cpu().numpy() for k, v in r.items() if isinstance(v, torch.Tensor)}
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, S = pop.shape[0], d["n_save"]
    xs = res["xs"].reshape(S, n_var, P, R).transpose(2, 3, 0, 1)
    assert bits_equal(xs, ref["xs"]), mismatch_report(xs, ref["xs"], "xs")
    if "steps" in ref:
        assert np.array_equal(res["steps"], ref["steps"])
    assert (res["steps"] >= 1).all() and (res["steps"] <= max_steps).all()
    # the workload exercises more than one accept/reject pattern
    assert len(np.unique(res["steps"])) > 3


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sr2", "sr12", "dynamic"])
def test_gpu_dopri5_general_pid_bitexact(kind):
    """A PID controller (pcoeff 0.3, icoeff 0.4, dcoeff 0.1, safety 0.85) and force_dtmin=False
    through every Dopri5 kernel (register SR, wide SR, dynamic control): fitness, step counts and
    trajectories bit-identical to the oracle."""
    import torch
    from helpers import bits_equal, dynamic_setup, mismatch_report
    from multitreegp_amd.engine import DeviceEngine
    pid = mt.PIDController(rtol=1e-5, atol=1e-5, pcoeff=0.3, icoeff=0.4, dcoeff=0.1, safety=0.85, dtmin=0.002,
                           force_dtmin=False)
    if kind == "dynamic":
        env, lib, ff, data, pop = dynamic_setup(P=21, R=8, n_steps=30, seed=4, solver=(1e-5, 1e-5, 0.002, 600))
    else:
        nv = 2 if kind == "sr2" else 12
        env, lib, ff, data, pop = sr_setup(P=21, R=8, n_save=26, save_every=4, h=0.01, depth=6, N=40,
                                           seed=70 + nv, n_var=nv, solver=(1e-5, 1e-5, 0.002, 600))
    ff.stepsize_controller = pid
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    r = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True, step_counts=True)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in r.items() if isinstance(v, torch.Tensor)}
    d = eng.prepare_data(data)
    assert d["pid_custom"] == 1 and d["no_force_dtmin"] == 1
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, S, R = pop.shape[0], d["n_save"], d["R"]
    nv = res["xs"].shape[1]
    xs = res["xs"].reshape(S, nv, P, R).transpose(2, 3, 0, 1)
    assert bits_equal(xs, ref["xs"]), mismatch_report(xs, ref["xs"], "xs")


@pytest.mark.gpu
def test_gpu_dopri5_fitness_only_matches_trajectory_mode():
    from helpers import bits_equal
    env, lib, ff, data, pop = sr_setup(P=64, R=16, n_save=101, save_every=4, h=0.01, seed=5,
                                       solver=(1e-6, 1e-6, 0.001, 500))
    a, _ = _gpu_run(ff, lib, data, pop, True, traj=True)
    b, _ = _gpu_run(ff, lib, data, pop, True, traj=False)
    assert bits_equal(a["fitness"], b["fitness"]) and bits_equal(a["rollout_fitness"], b["rollout_fitness"])


# ------------------------------------------------------------------ control evaluators
def test_dopri5_acrobot_oracle_vs_fixed_rk4():
    """Dynamic Acrobot policy (DynamicPolicy.ipynb:105 solver settings): at a tight tolerance the
    adaptive trajectories agree with fine fixed-step RK4 up to the chaos of the dynamics (short
    horizon), and the oracle is deterministic."""
    from helpers import dynamic_setup
    env, lib, ff, data, pop = dynamic_setup(P=6, R=4, n_steps=20, seed=2, solver=(1e-7, 1e-7, 0.0001, 4000))
    d = ff.prepare(data)
    dp = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    env2, lib2, ff2, data2, pop2 = dynamic_setup(P=6, R=4, n_steps=20, seed=2)
    d2 = ff2.prepare(data2)
    rk = orc.evaluate(oracle_model(ff2, d2), pop2, lib2, oracle_rollouts(d2), trajectories=True)
    fin = np.isfinite(rk["xs"]).all(axis=(2, 3)) & np.isfinite(dp["xs"]).all(axis=(2, 3))
    assert fin.sum() >= 12
    np.testing.assert_allclose(dp["xs"][fin][:, :8], rk["xs"][fin][:, :8], atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
@pytest.mark.parametrize("kind,env,obs_noise,state_size", [
    ("dynamic", "acrobot", 0.0, 2), ("dynamic", "acrobot", 0.1, 1), ("static", "acrobot", 0.0, 0),
    ("static", "acrobot", 0.1, 0), ("dynamic", "harmonic", 0.1, 2), ("dynamic", "reactor", 0.0, 3),
    ("static", "harmonic", 0.0, 0), ("static", "reactor", 0.1, 0)])
def test_gpu_dopri5_control_bitexact(jit, kind, env, obs_noise, state_size):
    """The notebooks' Dopri5 + PIDController(1e-4, 1e-4, dtmin=0.001) on every environment, with
    and without observation noise: fitness, per-rollout fitness and xs/ys/us/acts bit-identical to
    the oracle (interpolated save points, save-time readout, event and +inf fill)."""
    from helpers import bits_equal, dynamic_setup, mismatch_report, static_setup
    solver = (1e-4, 1e-4, 0.001, 300)
    if kind == "dynamic":
        e, lib, ff, data, pop = dynamic_setup(P=29, R=6, n_steps=40, seed=3, state_size=state_size,
                                              obs_noise=obs_noise, env=env, solver=solver)
    else:
        e, lib, ff, data, pop = static_setup(P=29, R=6, n_steps=40, seed=3, obs_noise=obs_noise, env=env,
                                             solver=solver)
    res, d = _gpu_run(ff, lib, data, pop, jit)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, R, S = pop.shape[0], d["R"], d["n_save"]
    for k in ("xs", "ys", "us", "acts"):
        if k not in ref:
            continue
        c = ref[k].shape[-1]
        got = res[k].reshape(S, c, P, R).transpose(2, 3, 0, 1)
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)


@pytest.mark.gpu
def test_gpu_dopri5_step_counts():
    """MtgpOutputs.steps: attempts per (individual, rollout), within [1, max_steps]; asking for
    them changes no result."""
    import torch
    from helpers import bits_equal, dynamic_setup
    from multitreegp_amd.engine import DeviceEngine
    e, lib, ff, data, pop = dynamic_setup(P=40, R=8, n_steps=40, seed=5, solver=(1e-4, 1e-4, 0.001, 250))
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    pd = torch.from_numpy(pop).cuda()
    a = eng.evaluate(pd, data, trajectories=True, rollout_fitness=True, step_counts=True)
    b = eng.evaluate(pd, data, trajectories=True, rollout_fitness=True)
    torch.cuda.synchronize()
    st = a["steps"].cpu().numpy()
    assert st.shape == (40, 8) and st.min() >= 1 and st.max() <= 250
    assert bits_equal(a["rollout_fitness"].cpu().numpy(), b["rollout_fitness"].cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
@pytest.mark.parametrize("budget", [0, 1, 7, 40])
@pytest.mark.parametrize("kind", ["dynamic", "static_noise"])
def test_gpu_dopri5_two_launches_bitexact(kind, budget, jit):
    """MtgpModel.dp_budget: launch 1 parks every wave still integrating after `budget` attempts
    (t, controller history, FSAL derivative, save index, fitness accumulator ...), launch 2 resumes
    only those -- fitness, per-rollout fitness, step counts and trajectories identical to one
    launch (budget 0) and to the oracle, including waves parked mid-way through their save points
    and waves whose lanes all finished in launch 1."""
    from helpers import bits_equal, dynamic_setup, mismatch_report, static_setup
    solver = (1e-4, 1e-4, 0.001, 200)
    if kind == "dynamic":
        e, lib, ff, data, pop = dynamic_setup(P=37, R=12, n_steps=40, seed=8, solver=solver)
    else:
        e, lib, ff, data, pop = static_setup(P=37, R=12, n_steps=40, seed=8, obs_noise=0.1, solver=solver)
    res, d = _gpu_run(ff, lib, data, pop, jit, dp_budget=budget, steps=True)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, R, S = pop.shape[0], d["R"], d["n_save"]
    for k in ("xs", "ys", "us", "acts"):
        if k in ref:
            got = res[k].reshape(S, ref[k].shape[-1], P, R).transpose(2, 3, 0, 1)
            assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)
    one, _ = _gpu_run(ff, lib, data, pop, jit, dp_budget=0, steps=True)
    assert np.array_equal(res["steps"], one["steps"])
    if budget in (1, 7):  # these budgets split the solves (some waves were parked)
        assert (one["steps"] > budget).any()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["dynamic", "static_noise", "sr", "sr_wide"])
def test_gpu_dopri5_traj_layouts_identical(kind, monkeypatch):
    """MtgpOutputs.traj_layout (ABI v20): the adaptive kernels' lane-major rows (the engine's
    default for Dopri5) hold exactly the time-major rows' values, element for element, in every
    kernel family (control k_ctl_dopri5, register SR k_sr_dopri5, wide SR k_sr_wide_dopri5);
    fixed-step solves keep time-major rows."""
    from helpers import bits_equal, dynamic_setup, static_setup
    solver = (1e-4, 1e-4, 0.001, 200)
    if kind == "dynamic":
        e, lib, ff, data, pop = dynamic_setup(P=21, R=12, n_steps=40, seed=4, solver=solver)
    elif kind == "static_noise":
        e, lib, ff, data, pop = static_setup(P=21, R=12, n_steps=40, seed=4, obs_noise=0.1, solver=solver)
    else:
        e, lib, ff, data, pop = sr_setup(P=19, R=8, n_save=21, save_every=4, h=0.01, seed=5,
                                         n_var=2 if kind == "sr" else 6, solver=(1e-5, 1e-5, 0.001, 300))
    monkeypatch.setenv("MTGP_TRAJ_LAYOUT", "time")
    tm, _ = _gpu_run(ff, lib, data, pop, True)
    monkeypatch.setenv("MTGP_TRAJ_LAYOUT", "auto")
    lm, _ = _gpu_run(ff, lib, data, pop, True)
    assert bits_equal(tm["fitness"], lm["fitness"])
    names = [k for k in ("xs", "ys", "us", "acts") if k in tm]
    assert names and all(k in lm for k in names)
    for k in names:
        assert tm[k].shape == lm[k].shape
        assert bits_equal(tm[k], lm[k]), k


def test_dp_budget_auto_choice():
    """DeviceEngine's automatic Dopri5 budget (no GPU needed): two launches until a two-launch
    evaluation has reported its parked fraction, one launch while that fraction is below
    kDpOneLaunchFrac, and a two-launch re-probe every kDpProbeEvery evaluations."""
    from multitreegp_amd.engine import DeviceEngine
    eng = object.__new__(DeviceEngine)
    eng._dp_probe, eng._dp_frac, eng._dp_evals = None, None, 0
    assert eng._dp_choose(1000) == 500  # nothing measured yet
    eng._dp_frac = 288 / 4096  # C3 noise-free (profiles/r05/v27_dpab_clean.log)
    picks = [eng._dp_choose(1000) for _ in range(2 * DeviceEngine.kDpProbeEvery)]
    assert picks.count(500) == 2 and picks.count(0) == len(picks) - 2
    assert all(picks[i] == 500 for i in range(len(picks)) if (i + 2) % DeviceEngine.kDpProbeEvery == 0)
    eng._dp_frac = 1587 / 4096  # C3 with obs_noise 0.1 (v27_dpab_noise.log)
    assert {eng._dp_choose(1000) for _ in range(20)} == {500}
