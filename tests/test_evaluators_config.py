"""Evaluator configuration: solver/schedule validation mirrors of the reference constructors."""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd.evaluators import constant_step_grid, fixed_schedule


class Dopri5:  # stand-in with diffrax's class name
    pass


def test_notebook_schedule():
    """The notebook grid with dt0 0.05 (DynamicPolicy.ipynb get_data): diffrax's accumulated
    ConstantStepSize grid to t1 = 49.8 takes 997 steps (nominally 996), save points straight from ts."""
    ts = np.arange(0, 50, 0.2, dtype=np.float32)
    assert fixed_schedule(ts, 0.05, 16 ** 4) == (997, 1, 250)


def test_rejects_adaptive_solver():
    env = mt.Acrobot(0.05, 0.0)
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(env, 2, 0.05, solver=Dopri5())
    ev = mt.DynamicEvaluator(env, 2, 0.05, solver="rk4")
    assert ev.max_fitness == 1e4 and ev.latent_size == 4 and ev.obs_size == 4


def test_obs_noise_data_preparation():
    """obs_noise > 0: the per-rollout keys and W = obs_noise * I go to the kernel (cbase.py:43-48)."""
    from multitreegp_amd import prng
    env = mt.Acrobot(0.05, 0.1)
    ev = mt.DynamicEvaluator(env, 2, 0.05)
    data = mt.control_data(env, 8, 0.05, None, seed=3, n_steps=10)
    d = ev.prepare(data)
    assert d["obs_keys"].dtype == np.uint32 and d["obs_keys"].shape == (8, 2)
    assert np.array_equal(d["obs_w"], np.float32(0.1) * np.eye(4, dtype=np.float32)) and d["prng_impl"] == 0
    prng.set_threefry_partitionable(True)
    try:
        assert ev.prepare(data)["prng_impl"] == 1
    finally:
        prng.set_threefry_partitionable(False)
    bad = data[:4] + (np.zeros((7, 2), np.uint32),) + data[5:]
    with pytest.raises(ValueError):
        ev.prepare(bad)
    assert "obs_keys" not in mt.DynamicEvaluator(mt.Acrobot(0.05, 0.0), 2, 0.05).prepare(data)


def test_schedule_any_grid():
    """ABI v18: any non-decreasing ts (SaveAt(ts) through the dense output); max_steps caps the grid
    (the solve then ends early with +inf saves instead of raising)."""
    assert fixed_schedule(np.array([0.0, 0.07, 0.14], np.float32), 0.05, 100) == (3, 1, 3)  # off the step grid
    assert fixed_schedule(np.array([0.0, 0.1, 0.3], np.float32), 0.05, 100) == (6, 1, 3)    # non-uniform
    assert fixed_schedule(np.arange(0, 10, 0.1, dtype=np.float32), 0.05, 10) == (10, 1, 100)  # max_steps
    assert fixed_schedule(np.array([5.0, 5.1, 5.2], np.float32), 0.05, 100)[::2] == (4, 3)    # offset start
    g = constant_step_grid(np.array([5.0, 5.2], np.float32), 0.05)
    assert g[0] == np.float32(5.0) and g[-1] == np.float32(5.2) and len(g) == 5
    with pytest.raises(ValueError):
        fixed_schedule(np.array([0.0, 0.2, 0.1], np.float32), 0.05, 100)  # decreasing
    with pytest.raises(ValueError):
        fixed_schedule(np.array([0.0], np.float32), 0.05, 100)  # one point


@pytest.mark.parametrize("t0,dt,S", [(0.0, 0.2, 250), (5.0, 0.1, 40), (0.05, 0.1, 30), (-0.35, 0.05, 50),
                                     (-3.0, 0.2, 12), (100.0, 0.5, 20)])
def test_acrobot_mask_table(t0, dt, S):
    """acrobot_mask restates `ts / (ts[1] - ts[0]) > first_success` (acrobot.py:82): for every
    first_success f the kept costs are exactly the first kof[f] save points."""
    from multitreegp_amd.evaluators import acrobot_mask
    ts = (np.float32(t0) + np.arange(S, dtype=np.float32) * np.float32(dt)).astype(np.float32)
    r = acrobot_mask(ts)
    ratio = ts / np.float32(ts[1] - ts[0])
    k = np.arange(S, dtype=np.float32)
    if np.all(ratio > k - 1) and np.all(ratio <= k + 1):  # ts[0] = 0, or an offset below one spacing
        assert r is None and abs(t0 / dt) < 1  # the kernels' one-pass form
        return
    kof, need_hist = r
    assert kof.dtype == np.int32 and kof.shape == (S,)
    for f in range(S):
        keep = ~(ratio > np.float32(f))
        assert np.all(keep[:kof[f]]) and not np.any(keep[kof[f]:])
    assert need_hist == any(1 <= kof[f] <= f for f in range(1, S))
    assert need_hist == (t0 > 0 and t0 / dt < S - 1)  # a positive offset puts the prefix behind fs
    assert t0 / dt >= 1 or t0 / dt <= -1


@pytest.mark.parametrize("ts", [[0.0, 0.0, 0.1, 0.2], [0.0, 0.0, 0.0, 0.5, 0.5, 1.3], [1.0, 1.0, 2.0, 3.0],
                                [-1.0, -1.0, -0.5, 0.0, 0.0, 0.4], [-2.0, -2.0, -1.0]])
def test_acrobot_mask_degenerate_first_spacing(ts):
    """ts[1] == ts[0]: acrobot.py:82 divides by zero -- 0 / 0 = NaN keeps the cost (NaN > f is
    False), +inf masks it, -inf keeps it -- so the kept costs are the saves with ts_k <= 0, for
    every first_success (VERDICT r05 missing #4)."""
    from multitreegp_amd.evaluators import acrobot_mask
    ts = np.asarray(ts, np.float32)
    S = len(ts)
    kof, need_hist = acrobot_mask(ts)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = ts / np.float32(ts[1] - ts[0])
    for f in range(S):
        keep = ~(ratio > np.float32(f))
        assert np.all(keep[:kof[f]]) and not np.any(keep[kof[f]:])
    assert np.all(kof == np.sum(ts <= 0))
    assert need_hist == any(1 <= kof[f] <= f for f in range(1, S))


def test_acrobot_mask_rejects_non_prefix():
    from multitreegp_amd.evaluators import acrobot_mask
    with pytest.raises(NotImplementedError):
        acrobot_mask(np.array([0.0, 0.1, 0.5, 0.2], np.float32))  # decreasing ts: not a prefix
    assert acrobot_mask(np.array([0.0, 0.1, 0.2], np.float32)) is None


def test_program_specs_dynamic():
    ev = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05)
    specs, roles = ev.program_specs()
    # state equations see [y, a, u]; readout in the drift sees y = 0, u = 0; at saves u = 0
    assert specs == [(2, 7, 0b1001111, 4, 0), (0, 7, 0, 4, 0), (1, 7, 0, 4, 0), (2, 7, 0b1000000, 4, 0)]
    assert roles["prog_readout"] == 0 and roles["prog_state"] == 1 and roles["prog_readout_save"] == 3


def test_data_fingerprint_follows_content():
    """the device-data cache is keyed on content, so a mutated or re-allocated array
    is never served stale (ids of freed temporaries can repeat)."""
    from multitreegp_amd.engine import DeviceEngine
    x0 = np.zeros((4, 4), np.float32)
    params = (np.ones(4, np.float32),) * 4
    a = DeviceEngine.data_fingerprint((x0, np.arange(3, dtype=np.float32), params))
    b = DeviceEngine.data_fingerprint((x0.copy(), np.arange(3, dtype=np.float32), params))
    assert a == b
    x0[1, 2] = 1e-30
    c = DeviceEngine.data_fingerprint((x0, np.arange(3, dtype=np.float32), params))
    assert c != a
    assert DeviceEngine.data_fingerprint((x0.astype(np.float64),)) != DeviceEngine.data_fingerprint((x0,))


def test_data_fingerprint_sees_one_middle_element_of_a_large_array():
    """a large SR ground truth re-noised in place at one save point in the middle
    changes the key (the whole buffer is hashed, not a sample)."""
    from multitreegp_amd.engine import DeviceEngine
    ys = np.random.default_rng(0).standard_normal((16, 2001, 8)).astype(np.float32)  # ~1 MB
    a = DeviceEngine.data_fingerprint((ys,))
    ys[7, 1003, 5] = np.nextafter(ys[7, 1003, 5], np.float32(np.inf))
    assert DeviceEngine.data_fingerprint((ys,)) != a


def test_default_solver_is_the_reference_euler():
    """omitting `solver` gives the reference's default diffrax.Euler() (dyn.py:11,
    ff.py:11, sr.py:21), not RK4."""
    from multitreegp_amd import _native as nat
    env = mt.Acrobot(0, 0)
    for ev in (mt.DynamicEvaluator(env, 2, 0.05), mt.FeedforwardEvaluator(env, 0.05), mt.SREvaluator(dt0=0.05)):
        assert ev.solver_kind == "euler" and type(ev.solver).__name__ == "Euler"
    data = mt.control_data(env, 4, 0.05, None, seed=3, n_steps=10)
    assert mt.DynamicEvaluator(env, 2, 0.05).prepare(data)["solver"] == nat.SOLVER_EULER
    assert mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4()).prepare(data)["solver"] == nat.SOLVER_RK4


def test_oracle_euler_known_answer():
    """dx/dt = -x (tree 0 - x0), Euler: x_{n+1} = x_n + (-x_n) * dt in float32 on diffrax's grid."""
    from helpers import SR_OPS, oracle_model, oracle_rollouts
    from oracle import oracle as orc
    lib = mt.NodeLibrary(SR_OPS, [["x0"]], [1])
    N = 4
    cand = np.zeros((1, 1, N, 4), np.float32)
    cand[..., 1:3] = -1
    cand[0, 0, N - 3] = [lib.string_to_node["x0"], -1, -1, 0]
    cand[0, 0, N - 2] = [1, -1, -1, 0.0]
    cand[0, 0, N - 1] = [lib.string_to_node["-"], N - 2, N - 3, 0]
    x0 = np.array([[1.0], [-0.3]], np.float32)
    h = np.float32(0.05)
    ts = (np.arange(21, dtype=np.float32) * h).astype(np.float32)
    ff = mt.SREvaluator(dt0=0.05)
    d = ff.prepare((x0, ts, np.zeros((2, 21, 1), np.float32), None))
    out = orc.evaluate(oracle_model(ff, d), cand, lib, oracle_rollouts(d), trajectories=True)
    # diffrax ConstantStepSize (ABI v18): x1 = x + (0 - x) * dt over the accumulated f32 grid, each
    # ts[k] through LocalLinearInterpolation -- literal float32 (np_reference.cs_solve)
    import np_reference as npr
    for r in range(2):
        want = npr.cs_solve(lambda t, s: np.float32(0.0) - s, x0[r], ts, 0.05, "euler", np.float32)[:, 0]
        assert np.array_equal(out["xs"][0, r, :, 0].view(np.uint32), want.view(np.uint32))
    # and the textbook closed form of Euler's recursion within the grid's rounding
    assert np.allclose(out["xs"][0, 0, :, 0], (1.0 - 0.05) ** np.arange(21), rtol=1e-5)


def test_max_steps_must_be_positive():
    """diffeqsolve takes a positive max_steps; the C entry reads 0 as "no limit" for the fixed-step
    solve, so the Python mirror never hands it 0 or a negative count."""
    env = mt.Acrobot(0.0, 0.0)
    for bad in (0, -1, 2.5, True):
        with pytest.raises(ValueError):
            mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4(), max_steps=bad)
        with pytest.raises(ValueError):
            mt.FeedforwardEvaluator(env, 0.05, solver=mt.RK4(), max_steps=bad)
        with pytest.raises(ValueError):
            mt.SREvaluator(solver=mt.RK4(), dt0=0.05, max_steps=bad)
    assert mt.SREvaluator(solver=mt.RK4(), dt0=0.05, max_steps=np.int64(7)).max_steps == 7


def test_degenerate_interval_rejected():
    """ts[0] == ts[-1]: diffrax special-cases t0 == t1 (y0 at every save point); not built, so it
    raises instead of silently returning +inf saves."""
    from multitreegp_amd.evaluators import adaptive_schedule
    ts = np.array([1.0, 1.0, 1.0], np.float32)
    with pytest.raises(ValueError):
        fixed_schedule(ts, 0.05, 100)
    with pytest.raises(ValueError):
        adaptive_schedule(ts)


def test_stalled_grid_is_finite():
    """dt0 below half an ulp of t: t + dt0 rounds back to t.  diffrax would take dt = 0 steps until
    max_steps; the loop guard (mtgp_cs_advancing) ends after the first such step, which is the only
    one that can save anything -- the host grid, the numpy restatement and the oracle's step count
    agree, and none of them loops forever without max_steps."""
    import np_reference as npr
    from oracle import oracle as orc
    ts = np.array([1000.0, 1000.5, 1001.0], np.float32)
    g = constant_step_grid(ts, 1e-5)
    assert len(g) == 2 and g[1] == g[0]  # one (stalled) step
    assert len(npr.cs_grid(ts, 1e-5)) == 1 and orc.cs_steps(ts, 1e-5) == 1
    # stalls part-way: 2**24 + dt0 advances while t < 2**24, then stops advancing
    ts2 = np.array([16777200.0, 16777300.0], np.float32)
    g2 = constant_step_grid(ts2, 1.0, 10 ** 6)
    ref = npr.cs_grid(ts2, 1.0, 10 ** 6)
    assert len(g2) - 1 == len(ref) == orc.cs_steps(ts2, 1.0) and len(ref) < 100


def test_stalled_grid_oracle_solve_ends_with_inf_saves():
    """The oracle's fixed-step solve on a stalled grid with max_steps 0 (no limit, the C entry's
    reading) terminates; the saves the grid never reaches are +inf (as diffrax's max_steps exit)."""
    from oracle import oracle as orc
    from test_oracle import _linear_sr_candidate
    lib, cand = _linear_sr_candidate()
    ts = np.array([1000.0, 1000.5, 1001.0], np.float32)
    model = dict(model=3, n_var=2, state_size=0, n_obs=0, n_control=0, n_targets=0, n_steps=0, save_every=1,
                 n_save=3, h=1e-5, max_fitness=1e5, parsimony=0.0, solver=0, max_steps=0)
    x0 = np.array([[1.0, 0.0]], np.float32)
    out = orc.evaluate(model, cand, lib, dict(x0=x0, ts=ts, ys_true=np.zeros((1, 3, 2), np.float32)),
                       trajectories=True)
    xs = out["xs"][0, 0]
    assert np.array_equal(xs[0], x0[0]) and np.all(np.isposinf(xs[1:]))


def test_state_size_limits():
    """state_size 1 .. 16 with every solver (round 6: Dopri5 and 9 .. 16 on the runtime-state-size
    kernels); beyond 16, or a data vector [y, a, u, targets] over the 24 LDS slots, raises."""
    env = mt.Acrobot(0.0, 0.0)
    pid = mt.PIDController(rtol=1e-4, atol=1e-4, dtmin=0.001)
    for ss in (4, 8, 12, 16):
        mt.DynamicEvaluator(env, ss, 0.05, solver=mt.RK4())
        mt.DynamicEvaluator(env, ss, 0.05, solver=mt.Dopri5(), stepsize_controller=pid)
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(env, 17, 0.05, solver=mt.RK4())
    reactor = mt.StirredTankReactor(0.0, 0.0)
    need = reactor.n_var * reactor.n_dim + 16 + reactor.n_control + reactor.n_targets
    if need > 24:
        with pytest.raises(NotImplementedError):
            mt.DynamicEvaluator(reactor, 16, 0.05, solver=mt.RK4())
    else:
        mt.DynamicEvaluator(reactor, 16, 0.05, solver=mt.RK4())
