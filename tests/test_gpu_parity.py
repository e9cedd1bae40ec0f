"""GPU parity: the HIP path through the C ABI vs the CPU oracle, bit-for-bit.

Every comparison is exact (uint32 equality, NaN == NaN): kernel and oracle share the fp32
arithmetic spec (include/mtgp_f32math.h), evaluate identical operations in identical order,
and the oracle interprets trees row by row like gp.py:356-388 while the kernel runs the
flattened programs -- so any flattener/interpreter/integrator/fitness bug shows up."""
import numpy as np
import pytest
import torch

import multitreegp_amd as mt
from multitreegp_amd.engine import DeviceEngine, to_reference_layout
from oracle import oracle as orc
from helpers import (bits_equal, dynamic_setup, mismatch_report, oracle_model, oracle_rollouts, sr_setup,
                     static_setup)

pytestmark = pytest.mark.gpu


def _run(ff, lib, data, pop, parsimony=0.0, traj=True, lanes=None):
    eng = DeviceEngine(ff, lib, parsimony, "cuda:0", lanes=lanes)
    res = eng.evaluate(torch.from_numpy(np.ascontiguousarray(pop)).cuda(), data, trajectories=traj,
                       rollout_fitness=True)
    torch.cuda.synchronize()
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d, parsimony), pop, lib, oracle_rollouts(d), trajectories=traj)
    return res, ref, d


def _check(res, ref, P, R, names):
    assert bits_equal(res["fitness"].cpu().numpy(), ref["fitness"]), \
        mismatch_report(res["fitness"].cpu().numpy(), ref["fitness"], "fitness")
    assert bits_equal(res["rollout_fitness"].cpu().numpy(), ref["rollout_fitness"]), \
        mismatch_report(res["rollout_fitness"].cpu().numpy(), ref["rollout_fitness"], "rollout_fitness")
    for k in names:
        got = to_reference_layout(res[k], P, R)
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)


def test_eval_programs_vs_row_order_oracle():
    env, lib, ff, data, pop = dynamic_setup(P=64)
    eng = DeviceEngine(mt.evaluators._TreeOnly(3, 7), lib, 0.0, "cuda:0")
    eng.prepare_data(None)
    fl = eng.flatten(torch.from_numpy(pop).cuda())
    eng.check_status(fl)
    rng = np.random.default_rng(5)
    dv = rng.standard_normal((100, 7)).astype(np.float32) * 3
    out = eng.eval_programs(fl, torch.from_numpy(dv).cuda()).cpu().numpy()
    ref = np.array([[[orc.eval_tree(pop[p, t], lib.fn_codes, lib.n_funcs, lib.var_start, dv[m])
                      for m in range(dv.shape[0])] for t in range(3)] for p in range(pop.shape[0])], np.float32)
    assert bits_equal(out, ref), mismatch_report(out, ref, "eval_programs")


def test_eval_programs_garbage_arrays():
    """Arbitrary arrays (bad opcodes, wrapped/clamped indices, forward refs) follow body_fun."""
    env, lib, ff, data, _ = dynamic_setup(P=4)
    rng = np.random.default_rng(11)
    P, N = 200, 20
    pop = np.empty((P, 3, N, 4), np.float32)
    pop[..., 0] = rng.integers(-2, lib.n_funcs + 3, (P, 3, N)) + (rng.random((P, 3, N)) < 0.1) * 0.5
    pop[..., 1] = rng.integers(-N - 3, N + 3, (P, 3, N))
    pop[..., 2] = rng.integers(-N - 3, N + 3, (P, 3, N))
    pop[..., 3] = rng.standard_normal((P, 3, N)) * 3
    eng = DeviceEngine(mt.evaluators._TreeOnly(3, 7), lib, 0.0, "cuda:0")
    eng.prepare_data(None)
    fl = eng.flatten(torch.from_numpy(pop).cuda())
    status = fl.status.cpu().numpy()
    dv = rng.standard_normal((17, 7)).astype(np.float32)
    out = eng.eval_programs(fl, torch.from_numpy(dv).cuda()).cpu().numpy()
    checked = 0
    for p in range(P):
        for t in range(3):
            if status[p, t] != 0:
                continue
            ref = np.array([orc.eval_tree(pop[p, t], lib.fn_codes, lib.n_funcs, lib.var_start, dv[m])
                            for m in range(dv.shape[0])], np.float32)
            assert bits_equal(out[p, t], ref), mismatch_report(out[p, t], ref, f"tree {p},{t}")
            checked += 1
    assert checked > 400


# lanes: None = the engine's occupancy policy (small P: one individual per wave), 0 = the densest
# packing (64 / R individuals per wave), 32 = an intermediate lane set
LANES = [None, 0, 32]


@pytest.mark.parametrize("lanes", LANES)
@pytest.mark.parametrize("R", [8, 32])
def test_dynamic_acrobot_bitexact(R, lanes):
    env, lib, ff, data, pop = dynamic_setup(P=40, R=R, n_steps=80)
    res, ref, d = _run(ff, lib, data, pop, lanes=lanes)
    _check(res, ref, pop.shape[0], R, ["xs", "ys", "us", "acts"])


def test_dynamic_fitness_only_matches_trajectory_mode():
    env, lib, ff, data, pop = dynamic_setup(P=64, R=16, n_steps=100, seed=3)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    pt = torch.from_numpy(pop).cuda()
    a = eng.evaluate(pt, data, trajectories=True)["fitness"].cpu().numpy()
    b = eng.evaluate(pt, data, trajectories=False)["fitness"].cpu().numpy()
    assert bits_equal(a, b)


@pytest.mark.parametrize("lanes", LANES)
def test_static_acrobot_bitexact(lanes):
    env, lib, ff, data, pop = static_setup(P=40, R=16, n_steps=80)
    res, ref, d = _run(ff, lib, data, pop, parsimony=1.0, lanes=lanes)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us"])


@pytest.mark.parametrize("lanes", LANES)
def test_sr_vanderpol_bitexact(lanes):
    env, lib, ff, data, pop = sr_setup(P=40, R=16)
    res, ref, d = _run(ff, lib, data, pop, lanes=lanes)
    _check(res, ref, pop.shape[0], 16, ["xs"])


@pytest.mark.parametrize("lanes", [None, 0])
@pytest.mark.parametrize("R", [1, 33, 64])
def test_rollout_counts(R, lanes):
    env, lib, ff, data, pop = dynamic_setup(P=9, R=R, n_steps=30, seed=7)
    res, ref, d = _run(ff, lib, data, pop, lanes=lanes)
    _check(res, ref, pop.shape[0], R, ["xs", "us"])


@pytest.mark.parametrize("R", [65, 128, 200])
@pytest.mark.parametrize("kind", ["dynamic", "static", "sr", "sr_wide", "dynamic_dopri5"])
def test_more_than_64_rollouts(kind, R):
    """R > 64 (dyn.py:63 vmaps any batch): an individual's lane set spans ceil(R/64) rounded up
    to a power of two waves, the mean over rollouts is formed by k_rollout_mean in the
    kernel's pairwise order -- fitness, per-rollout fitness and trajectories bit-exact."""
    if kind == "dynamic":
        env, lib, ff, data, pop = dynamic_setup(P=11, R=R, n_steps=24, seed=9)
        names = ["xs", "ys", "us", "acts"]
    elif kind == "dynamic_dopri5":
        env, lib, ff, data, pop = dynamic_setup(P=7, R=R, n_steps=20, seed=9, solver=(1e-3, 1e-3, 0.001, 60))
        names = ["xs", "us"]
    elif kind == "static":
        env, lib, ff, data, pop = static_setup(P=11, R=R, n_steps=24, seed=9)
        names = ["xs", "ys", "us"]
    elif kind == "sr":
        env, lib, ff, data, pop = sr_setup(P=11, R=R, n_save=9, seed=9)
        names = ["xs"]
    else:
        env, lib, ff, data, pop = sr_setup(P=5, R=R, n_save=7, seed=9, n_var=6)
        names = ["xs"]
    res, ref, d = _run(ff, lib, data, pop, parsimony=0.5)
    _check(res, ref, pop.shape[0], R, names)


@pytest.mark.parametrize("n_var,R,N,depth", [(5, 8, 30, 5), (12, 3, 64, 8), (64, 8, 128, 16)])
def test_sr_wide_state_bitexact(n_var, R, N, depth):
    """n_var > 4: the workgroup-per-lane-set SR kernel (BASELINE C5 shape at n_var = 64,
    max_nodes 128, depth <= 16), trajectories and fitness bit-exact vs the oracle."""
    env, lib, ff, data, pop = sr_setup(P=19, R=R, n_save=9, save_every=3, h=0.01, depth=depth, N=N,
                                       n_var=n_var, seed=2)
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, pop.shape[0], R, ["xs"])


def test_sr_wide_fitness_only_matches_trajectory_mode():
    env, lib, ff, data, pop = sr_setup(P=21, R=8, n_save=9, save_every=3, h=0.05, depth=8, N=64, n_var=16,
                                       seed=4)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    pd = torch.from_numpy(pop).cuda()
    a = eng.evaluate(pd, data, trajectories=True, rollout_fitness=True)
    b = eng.evaluate(pd, data, trajectories=False, rollout_fitness=True)
    assert bits_equal(a["fitness"].cpu().numpy(), b["fitness"].cpu().numpy())
    assert bits_equal(a["rollout_fitness"].cpu().numpy(), b["rollout_fitness"].cpu().numpy())


@pytest.mark.parametrize("impl", [0, 1])
def test_dynamic_obs_noise_bitexact(impl):
    """Observation noise (threefry fold_in + normal, control_environment_base.py:43-48) drawn
    in-kernel at every stage time and save time, bit-exact vs the oracle."""
    from multitreegp_amd import prng
    prng.set_threefry_partitionable(bool(impl))
    try:
        env, lib, ff, data, pop = dynamic_setup(P=40, R=32, n_steps=60, obs_noise=0.1, seed=2)
        res, ref, d = _run(ff, lib, data, pop)
        assert d["prng_impl"] == impl
        _check(res, ref, pop.shape[0], 32, ["xs", "ys", "us", "acts"])
    finally:
        prng.set_threefry_partitionable(False)


def test_static_obs_noise_bitexact():
    env, lib, ff, data, pop = static_setup(P=40, R=16, n_steps=60, obs_noise=0.1, seed=4)
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us"])


@pytest.mark.parametrize("kind", ["dynamic", "static"])
def test_obs_noise_save_time_differs_from_step_time(kind):
    """dt0 = 0.1, save spacing f32(0.3): the save times are not step ends of the accumulated grid, so
    the save state comes from the dense output and its observation is drawn at ts[k] (dyn.py:99 /
    ff.py:96)."""
    if kind == "dynamic":
        env = mt.Acrobot(0.0, 0.1)
        from helpers import CONTROL_OPS
        vl = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
        lib = mt.NodeLibrary(CONTROL_OPS, vl, [2, 1])
        ff = mt.DynamicEvaluator(env, 2, 0.1, solver=mt.RK4())
        names = ["xs", "ys", "us", "acts"]
    else:
        env = mt.Acrobot(0.0, 0.1)
        from helpers import CONTROL_OPS
        lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1])
        ff = mt.FeedforwardEvaluator(env, 0.1, solver=mt.RK4())
        names = ["xs", "ys", "us"]
    from multitreegp_amd.sampling import sample_population
    data = mt.control_data(env, 16, 0.3, None, seed=5, n_steps=40)
    ts = data[1]
    tk = np.array([np.float32(ts[0]) + np.float32(3 * k) * np.float32(0.1) for k in range(len(ts))], np.float32)
    assert (ts.view(np.uint32) != tk.view(np.uint32)).sum() > 5
    pop = sample_population(3, lib, 30, 1, max_init_depth=5, max_nodes=30)[0]
    res, ref, d = _run(ff, lib, data, pop)
    assert d["n_steps"] == orc.cs_steps(ts, 0.1) > 3 * (len(ts) - 1) - 2
    _check(res, ref, pop.shape[0], 16, names)


def _run_engine(ff, lib, data, pop, jit):
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=jit)
    res = eng.evaluate(torch.from_numpy(np.ascontiguousarray(pop)).cuda(), data, trajectories=True,
                       rollout_fitness=True)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(res["_flat"]) == jit
    return {k: v.cpu().numpy() for k, v in res.items() if isinstance(v, torch.Tensor)}


@pytest.mark.parametrize("kind", ["dynamic_noise", "static", "sr"])
def test_jit_matches_interpreter(kind):
    """The program JIT (csrc/mtgp_jit.h) and the interpreter give bit-identical results."""
    if kind == "dynamic_noise":
        env, lib, ff, data, pop = dynamic_setup(P=48, R=32, n_steps=60, obs_noise=0.1, seed=6)
    elif kind == "static":
        env, lib, ff, data, pop = static_setup(P=48, R=16, n_steps=60, seed=6)
    else:
        env, lib, ff, data, pop = sr_setup(P=48, R=16, seed=6)
    a = _run_engine(ff, lib, data, pop, True)
    b = _run_engine(ff, lib, data, pop, False)
    for k in a:
        assert bits_equal(a[k], b[k]), mismatch_report(a[k], b[k], k)


def test_jit_slow_sin_cos_lanes_fall_back_to_interpreter():
    """Coefficients scaled by 1e6: sin/cos arguments beyond 2^17 take the spec's slow
    reduction, which the JIT code reports and the evaluator re-runs with the interpreter."""
    env, lib, ff, data, pop = dynamic_setup(P=40, R=16, n_steps=30, seed=9)
    coef = pop[..., 0] == 1.0
    pop = pop.copy()
    pop[..., 3] = np.where(coef, pop[..., 3] * 1e6, pop[..., 3])
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=True)
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(res["_flat"])
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us", "acts"])


def test_jit_code_that_does_not_fit_is_interpreted():
    """The host never waits for the JIT plan: when the code is larger than the buffer the
    evaluator sees it on the device and interprets (results unchanged)."""
    env, lib, ff, data, pop = dynamic_setup(P=24, R=16, n_steps=30, seed=12)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=True)
    real_arena = eng._arena
    eng._arena = lambda nbytes: (real_arena(nbytes)[0], 16)  # claim a 16-byte buffer: every launch falls back
    pd = torch.from_numpy(pop).cuda()
    res = eng.evaluate(pd, data, trajectories=True, rollout_fitness=True)
    assert res["_flat"].jit is not None and not DeviceEngine.jit_ok(res["_flat"])
    torch.cuda.synchronize()
    d = eng.prepare_data(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us", "acts"])


def test_obs_noise_dense_w_bitexact():
    """A general (non-diagonal) noise matrix W: noise = normal @ W summed in index order."""
    env, lib, ff, data, pop = dynamic_setup(P=24, R=16, n_steps=40, obs_noise=0.1, seed=8)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    d = eng.prepare_data(data)
    W = (np.random.default_rng(4).standard_normal((4, 4)) * 0.05).astype(np.float32)
    d["obs_w"] = W
    d["obs_w_dev"] = torch.from_numpy(W).cuda()
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True)
    torch.cuda.synchronize()
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us", "acts"])


# ---------------------------------------------------------------- other environments
_H = {"harmonic": 0.05, "reactor": 0.002}  # reactor: a mix of finite and NaN (terminated) rollouts

@pytest.mark.parametrize("env", ["harmonic", "reactor"])
@pytest.mark.parametrize("state_size", [1, 3])
def test_dynamic_other_envs_bitexact(env, state_size):
    """HarmonicOscillator / StirredTankReactor with the dynamic evaluator: trajectories,
    per-rollout quadratic costs and fitness bit-exact vs the oracle ('Different' parameters)."""
    _, lib, ff, data, pop = dynamic_setup(P=40, R=16, n_steps=80, env=env, state_size=state_size, seed=3,
                                          h=_H[env])
    res, ref, d = _run(ff, lib, data, pop, parsimony=0.5)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us", "acts"])


@pytest.mark.parametrize("env", ["harmonic", "reactor"])
def test_static_other_envs_bitexact(env):
    _, lib, ff, data, pop = static_setup(P=40, R=16, n_steps=80, env=env, seed=4, h=_H[env])
    res, ref, d = _run(ff, lib, data, pop)
    _check(res, ref, pop.shape[0], 16, ["xs", "ys", "us"])


@pytest.mark.parametrize("env", ["harmonic", "reactor"])
@pytest.mark.parametrize("kind", ["dynamic", "static"])
def test_other_envs_obs_noise_bitexact(env, kind):
    """Observation noise with W = obs_noise*I (oscillator) and obs_noise*I*[15, 15, 0.1] (reactor)."""
    setup = dynamic_setup if kind == "dynamic" else static_setup
    _, lib, ff, data, pop = setup(P=32, R=16, n_steps=50, env=env, obs_noise=0.1, seed=5, h=_H[env])
    res, ref, d = _run(ff, lib, data, pop)
    names = ["xs", "ys", "us", "acts"] if kind == "dynamic" else ["xs", "ys", "us"]
    _check(res, ref, pop.shape[0], 16, names)


@pytest.mark.parametrize("env", ["harmonic", "reactor"])
def test_other_envs_fitness_only_and_interpreter(env):
    """Fitness-only mode (early exit once every lane has terminated) and the interpreter path
    agree bit-for-bit with the JIT trajectory run; terminated rollouts give NaN costs -> max_fitness."""
    _, lib, ff, data, pop = dynamic_setup(P=48, R=16, n_steps=100, env=env, seed=6, h=0.2)
    a = _run_engine(ff, lib, data, pop, True)
    b = _run_engine(ff, lib, data, pop, False)
    for k in a:
        assert bits_equal(a[k], b[k]), mismatch_report(a[k], b[k], k)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    c = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=False, rollout_fitness=True)
    assert bits_equal(c["rollout_fitness"].cpu().numpy(), a["rollout_fitness"])
    assert bits_equal(c["fitness"].cpu().numpy(), a["fitness"])


def test_jit_code_of_a_reused_flattened_population_is_rebuilt():
    """a Flattened keeps a pointer into the engine's two-buffer code ring.  Evaluate A,
    B, C (C reuses A's buffer), then A again through its old Flattened: the engine sees that the
    slot was rewritten and translates A again -- results equal the interpreter's."""
    env, lib, ff, data, _ = dynamic_setup(P=8, R=16, n_steps=20, seed=21)
    pops = [dynamic_setup(P=24, R=16, n_steps=20, seed=s)[4] for s in (22, 23, 24)]
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0", jit=True)
    flats = []
    for p in pops:
        res = eng.evaluate(torch.from_numpy(p).cuda(), data)
        flats.append(res["_flat"])
    pa = torch.from_numpy(pops[0]).cuda()
    again = eng.evaluate(pa, data, flattened=flats[0], rollout_fitness=True)
    torch.cuda.synchronize()
    assert DeviceEngine.jit_ok(again["_flat"])
    ref = _run_engine(ff, lib, data, pops[0], False)
    assert bits_equal(again["fitness"].cpu().numpy(), ref["fitness"])
    assert bits_equal(again["rollout_fitness"].cpu().numpy(), ref["rollout_fitness"])


@pytest.mark.parametrize("kind", ["dynamic", "static_noise", "sr", "sr_wide"])
@pytest.mark.parametrize("jit", [True, False])
def test_euler_bitexact(kind, jit):
    """diffrax.Euler (the reference default solver) in every fixed-step kernel: bit-exact with
    the oracle's Euler (trajectories and fitness)."""
    import multitreegp_amd as mt
    if kind == "dynamic":
        env, lib, ff, data, pop = dynamic_setup(P=20, R=16, n_steps=40, seed=31)
        ff = mt.DynamicEvaluator(ff.env, 2, 0.05, solver=mt.Euler())
        keys = ["xs", "ys", "us", "acts"]
    elif kind == "static_noise":
        env, lib, ff, data, pop = static_setup(P=20, R=16, n_steps=40, seed=32, obs_noise=0.1)
        ff = mt.FeedforwardEvaluator(ff.env, 0.05, solver=mt.Euler())
        keys = ["xs", "ys", "us"]
    else:
        env, lib, ff, data, pop = sr_setup(P=20, R=16, seed=33, n_var=2 if kind == "sr" else 9)
        ff = mt.SREvaluator(solver=mt.Euler(), dt0=0.05)
        keys = ["xs"]
    res = _run_engine(ff, lib, data, pop, jit and kind != "sr_wide")
    d = DeviceEngine(ff, lib, 0.0, "cuda:0").prepare_data(data)
    assert d["solver"] == 2
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    for k in ("fitness", "rollout_fitness"):
        assert bits_equal(res[k], ref[k]), mismatch_report(res[k], ref[k], k)
    P, R, S = pop.shape[0], d["R"], d["n_save"]
    for k in keys:
        c = ref[k].shape[-1]
        got = res[k].reshape(S, c, P, R).transpose(2, 3, 0, 1)
        assert bits_equal(got, ref[k]), mismatch_report(got, ref[k], k)


@pytest.mark.parametrize("case", ["acrobot_dyn_2", "acrobot_dyn_1_noise", "acrobot_static_3_noise", "harmonic_dyn_1",
                                  "reactor_static_2_noise", "acrobot_dyn_2_dopri5"])
def test_fewer_observations_than_states(case):
    """n_obs < n_var: C = eye(n_var)[:n_obs] (control_environment_base.py:47, acrobot.py:48), noise
    normal(key, (n_obs,)) @ W with W = obs_noise * eye(n_obs) -- the data vector [y(n_obs), a, u,
    tg] of the reference reaches the kernel's n_var-slot layout through MtgpProgramSpec.gap."""
    env_name, kind, no = case.split("_")[:3]
    noise = 0.1 if case.endswith("noise") else 0.0
    solver = (1e-3, 1e-3, 0.001, 80) if case.endswith("dopri5") else None
    cls = {"acrobot": mt.Acrobot, "harmonic": mt.HarmonicOscillator, "reactor": mt.StirredTankReactor}[env_name]
    env = cls(0.0, noise, n_obs=int(no))
    from helpers import CONTROL_OPS, _ctl_solver, _mode
    from multitreegp_amd.sampling import sample_population
    ys = [f"y{i + 1}" for i in range(env.n_obs)]
    tg = [f"tar{i + 1}" for i in range(env.n_targets)]
    if kind == "dyn":
        vl = [ys + ["a1", "a2", "u"] + tg, ["a1", "a2"] + tg]
        lib = mt.NodeLibrary(CONTROL_OPS, vl, [2, 1])
        ff = mt.DynamicEvaluator(env, 2, 0.05, **_ctl_solver(solver))
        names = ["xs", "ys", "us", "acts"]
    else:
        lib = mt.NodeLibrary(CONTROL_OPS, [ys + tg], [1])
        ff = mt.FeedforwardEvaluator(env, 0.05, **_ctl_solver(solver))
        names = ["xs", "ys", "us"]
    data = mt.control_data(env, 8, 0.05, None, seed=3, n_steps=40, mode=_mode(env_name))
    pop = sample_population(4, lib, 24, 1, max_init_depth=5, max_nodes=30)[0]
    res, ref, d = _run(ff, lib, data, pop)
    assert res["ys"].shape[1] == env.n_obs
    _check(res, ref, pop.shape[0], 8, names)


DP_RT = (1e-4, 1e-4, 0.001, 600)  # Dopri5 + PID (rtol, atol, dtmin, max_steps)


@pytest.mark.parametrize("case", [("acrobot", 4, None, 0.0), ("acrobot", 6, "euler", 0.1), ("harmonic", 5, None, 0.0),
                                  ("reactor", 8, None, 0.1), ("acrobot", 8, None, 0.0), ("acrobot", 12, None, 0.0),
                                  ("acrobot", 12, "euler", 0.1), ("harmonic", 16, None, 0.1), ("reactor", 9, None, 0.0),
                                  ("acrobot", 4, "dopri5", 0.0), ("acrobot", 8, "dopri5", 0.1),
                                  ("acrobot", 12, "dopri5", 0.0), ("harmonic", 16, "dopri5", 0.0),
                                  ("reactor", 6, "dopri5", 0.1)])
def test_state_size_above_three(case):
    """state_size 4 .. 16 (dyn.py:83 takes any): the data vector [y, a, u, tg] no longer fits the
    JIT's eight data registers, so the wide interpreter kernels run it (k_ctl_dynamic /
    k_ctl_dopri5<Env, kNaRuntime | kNaWide>: runtime state size, 16 / 24 LDS data columns; round 6:
    Dopri5 and state_size 9 .. 16) -- bit-exact vs the oracle, trajectories included."""
    env_name, ss, solver, noise = case
    from helpers import dynamic_setup
    env, lib, ff, data, pop = dynamic_setup(P=21, R=8, n_steps=30, depth=5, N=30, seed=11, state_size=ss,
                                            obs_noise=noise, env=env_name,
                                            solver=DP_RT if solver == "dopri5" else None)
    if solver == "euler":
        ff = mt.DynamicEvaluator(env, ss, ff.dt0, solver=mt.Euler())
    res, ref, d = _run(ff, lib, data, pop, parsimony=0.25)
    # fixed-step solvers: LDS-data JIT code (round 6); Dopri5: the interpreter
    assert DeviceEngine.jit_ok(res["_flat"]) == (solver != "dopri5")
    _check(res, ref, pop.shape[0], 8, ["xs", "ys", "us", "acts"])
    assert res["acts"].shape[1] == ss
    if solver != "dopri5":  # the interpreter on the same population: the same bits
        eng = DeviceEngine(ff, lib, 0.25, "cuda:0", jit=False)
        r2 = eng.evaluate(torch.from_numpy(np.ascontiguousarray(pop)).cuda(), data, trajectories=True,
                          rollout_fitness=True)
        assert not DeviceEngine.jit_ok(r2["_flat"])
        for k in ("fitness", "rollout_fitness", "xs", "acts"):
            assert bits_equal(res[k].cpu().numpy(), r2[k].cpu().numpy()), k
