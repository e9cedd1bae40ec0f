"""HarmonicOscillator and StirredTankReactor: the fp32 spec's exp, the
oracle's drifts/costs against the float64 restatement in tests/np_reference.py, the evaluator
semantics over a short horizon, and the host-side configuration checks (CPU only)."""
import mpmath
import numpy as np
import pytest

import multitreegp_amd as mt
import np_reference as npr
from helpers import dynamic_setup, oracle_model, oracle_rollouts, static_setup
from multitreegp_amd import _native as nat
from oracle import oracle as orc

ENV_ID = {"harmonic": nat.ENV_HARMONIC_OSCILLATOR, "reactor": nat.ENV_STIRRED_TANK_REACTOR}


def test_expf_within_1ulp_and_edges():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-103, 88.7, 4000), rng.uniform(-1, 1, 1000), [-87.3, -100.0, 88.72]])
    x = x.astype(np.float32)
    got = orc.expf(x).astype(np.float64)
    ref = np.array([float(mpmath.exp(mpmath.mpf(float(v)))) for v in x])
    tiny = np.float32(np.finfo(np.float32).smallest_subnormal)
    sp = np.maximum(np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64), float(tiny))
    assert np.max(np.abs(got - ref) / sp) <= 1.0
    e = orc.expf(np.array([np.nan, np.inf, -np.inf, 89.0, -104.0, 0.0, -0.0], np.float32))
    assert np.isnan(e[0]) and e[1] == np.inf and e[2] == 0 and e[3] == np.inf and e[4] == 0
    assert e[5] == 1.0 and e[6] == 1.0


@pytest.mark.parametrize("name", ["harmonic", "reactor"])
def test_env_drift_vs_float64(name):
    env = npr_env = None
    env = mt.HarmonicOscillator(0, 0) if name == "harmonic" else mt.StirredTankReactor(0, 0)
    rng = np.random.default_rng(1)
    for i in range(200):
        params = np.array(env.sample_params(1, "Different", None, rng), np.float32).reshape(-1)
        x0, _ = env.sample_init_states(1, rng)
        x = x0[0]
        u = np.float32(rng.normal() * (100 if name == "reactor" else 2))
        got = orc.env_drift(ENV_ID[name], params, x, u)
        want = npr.env_drift(name, x.astype(np.float64), float(u), params.astype(np.float64))
        assert np.allclose(got, want, rtol=2e-5, atol=1e-5 * np.max(np.abs(want))), (got, want)
    del npr_env


@pytest.mark.parametrize("name", ["harmonic", "reactor"])
def test_env_fitness_vs_float64(name):
    env = mt.HarmonicOscillator(0, 0) if name == "harmonic" else mt.StirredTankReactor(0, 0)
    rng = np.random.default_rng(2)
    S = 51
    for i in range(20):
        params = np.array(env.sample_params(1, "Different", None, rng), np.float32).reshape(-1)
        x0, tg = env.sample_init_states(S, rng)
        us = rng.normal(size=S).astype(np.float32) * 3
        ts = np.arange(S, dtype=np.float32) * np.float32(0.1)
        got = orc.env_fitness(ENV_ID[name], x0, us, ts, params, tg[0, 0])
        want = npr.env_fitness(name, x0, us, params.astype(np.float64), float(tg[0, 0]))
        assert abs(float(got) - want) <= 1e-5 * abs(want), (got, want)
    # the +inf fill after termination makes the cost NaN (0 * inf in the quadratic form)
    x0[10:] = np.inf
    assert np.isnan(orc.env_fitness(ENV_ID[name], x0, us, ts, params, tg[0, 0]))


@pytest.mark.parametrize("name", ["harmonic", "reactor"])
@pytest.mark.parametrize("kind", ["dynamic", "static"])
def test_oracle_other_envs_vs_float64_short_horizon(name, kind):
    """Evaluator semantics for the new environments: data layout [y, a, u, target], target
    slots, parameter columns, RK4, saves, per-rollout quadratic cost."""
    n = 20
    h = 0.05 if name == "harmonic" else 0.002  # random policies drive the reactor to NaN within ~0.1 min
    if kind == "dynamic":
        env, lib, ff, data, pop = dynamic_setup(P=12, R=3, n_steps=n, env=name, state_size=2, h=h)
    else:
        env, lib, ff, data, pop = static_setup(P=12, R=3, n_steps=n, env=name, h=h)
    d = ff.prepare(data)
    assert d["env"] == ENV_ID[name] and d["params"].shape == (3, 2 if name == "harmonic" else 8)
    out = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d), trajectories=True)
    nv = env.n_var
    compared = tight = fit_ok = 0
    for p in range(pop.shape[0]):
        for r in range(d["R"]):
            x0 = d["x0"][r].astype(np.float64)
            prm = d["params"][r].astype(np.float64)
            tg = float(d["targets"][r, 0])
            if kind == "dynamic":
                traj = npr.rk4(lambda s: npr.dyn_rhs_env(name, pop[p], lib, s, 2, prm, tg, nv),
                               np.concatenate([x0, [0, 0]]), h, n)
                got = np.concatenate([out["xs"][p, r], out["acts"][p, r]], -1)
            else:
                traj = npr.rk4(lambda s: npr.ff_rhs_env(name, pop[p], lib, s, prm, tg), x0, h, n)
                got = out["xs"][p, r]
            scale = np.maximum(np.abs(traj), 1.0)
            if not (np.all(np.isfinite(traj)) and np.all(np.isfinite(got)) and np.all(np.abs(traj) < 1e4)):
                continue
            compared += 1
            if np.all(np.abs(got - traj) <= 2e-3 * scale):
                tight += 1
                f = npr.env_fitness(name, out["xs"][p, r], out["us"][p, r], prm, tg)
                fit_ok += abs(float(out["rollout_fitness"][p, r]) - f) <= 1e-4 * max(abs(f), 1.0)
    # fp32 vs fp64: sin/cos of products of reactor-scale inputs (~400^2) amplify argument rounding,
    # so a minority of candidates may separate; those that agree must agree on the cost too
    assert compared >= 8 and tight >= 0.8 * compared and fit_ok == tight


def test_other_env_termination_gives_max_fitness():
    """A state equation that blows up (da = 1 + a^2) terminates the rollout: the saved +inf fill
    makes the quadratic cost NaN, which the evaluator maps to max_fitness (dyn.py:49-52)."""
    env, lib, ff, data, _ = dynamic_setup(P=1, R=2, n_steps=60, env="harmonic", state_size=1)
    N = 8
    cand = np.zeros((1, 2, N, 4), np.float32)
    cand[..., 1:3] = -1
    a1 = lib.string_to_node["a1"]
    cand[0, 0, 3] = [a1, -1, -1, 0]
    cand[0, 0, 4] = [a1, -1, -1, 0]
    cand[0, 0, 5] = [lib.string_to_node["*"], 4, 3, 0]
    cand[0, 0, 6] = [1, -1, -1, 1.0]
    cand[0, 0, 7] = [lib.string_to_node["+"], 6, 5, 0]
    cand[0, 1, 7] = [1, -1, -1, 0.3]
    d = ff.prepare(data)
    out = orc.evaluate(oracle_model(ff, d), cand, lib, oracle_rollouts(d), trajectories=True)
    assert np.all(np.isnan(out["rollout_fitness"]))
    assert out["fitness"][0] == np.float32(1e4)


def test_environment_configuration_checks():
    with pytest.raises(ValueError):  # C = eye(n_var)[:n_obs] needs 1 <= n_obs <= n_var
        mt.DynamicEvaluator(mt.HarmonicOscillator(0, 0, n_obs=3), 1, 0.05, solver=mt.RK4())
    with pytest.raises(ValueError):
        mt.FeedforwardEvaluator(mt.StirredTankReactor(0, 0, n_obs=0), 0.05, solver=mt.RK4())
    # state_size > 3: every solver (round 6), up to 16
    mt.DynamicEvaluator(mt.Acrobot(0, 0), 4, 0.05, solver=mt.Dopri5(), stepsize_controller=mt.PIDController(1e-4, 1e-4))
    mt.DynamicEvaluator(mt.Acrobot(0, 0), 9, 0.05, solver=mt.RK4())
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(mt.Acrobot(0, 0), 17, 0.05, solver=mt.RK4())
    mt.DynamicEvaluator(mt.Acrobot(0, 0), 8, 0.05, solver=mt.RK4())
    # fewer observations than states: the data slots after y move up in the kernel's layout
    ev = mt.DynamicEvaluator(mt.Acrobot(0, 0, n_obs=2), 2, 0.05, solver=mt.RK4())
    assert ev.n_data() == 2 + 2 + 1 and ev.obs_gap() == (2, 2)
    assert all(sp[3:] == (2, 2) for sp in ev.program_specs()[0])

    class CartPole:  # no cond_fn_nan in the reference: not runnable by its evaluators
        n_obs = n_var = 4
        n_control = 1
        n_targets = 0
        n_dim = 1
    with pytest.raises(NotImplementedError):
        mt.DynamicEvaluator(CartPole(), 1, 0.05, solver=mt.RK4())
    env = mt.HarmonicOscillator(0, 0)
    ff = mt.DynamicEvaluator(env, 1, 0.05, solver=mt.RK4())
    data = list(mt.control_data(env, 4, 0.05, None, n_steps=10))
    data[5] = (np.ones((4, 11), np.float32), np.zeros((4, 11), np.float32))  # 'Switch'-style [R, S]
    with pytest.raises(NotImplementedError):
        ff.prepare(tuple(data))
    W = mt.StirredTankReactor(0, 0.1).obs_matrix()
    assert W.dtype == np.float32 and np.array_equal(W, np.diag(np.float32(0.1) * np.array([15, 15, 0.1], np.float32)))
