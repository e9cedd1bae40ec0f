"""Shared test fixtures: reference-style node libraries, populations and data."""
import numpy as np

import multitreegp_amd as mt
from multitreegp_amd.sampling import sample_population

CONTROL_OPS = [("+", None, 2, 0.5), ("-", None, 2, 0.1), ("*", None, 2, 0.5), ("sin", None, 1, 0.1),
               ("cos", None, 1, 0.1)]  # DynamicPolicy.ipynb
SR_OPS = [("+", None, 2, 0.5), ("-", None, 2, 0.1), ("*", None, 2, 0.5), ("/", None, 2, 0.1)]  # SymbolicRegression.ipynb


ENVS = {"acrobot": mt.Acrobot, "harmonic": mt.HarmonicOscillator, "reactor": mt.StirredTankReactor}


def make_env(name, obs_noise):
    return ENVS[name](0.0, obs_noise)


def _mode(name):
    return "Constant" if name == "acrobot" else "Different"


def _ctl_solver(solver):
    """None: fixed-step RK4; (rtol, atol, dtmin, max_steps): Dopri5 + PIDController."""
    if solver is None:
        return dict(solver=mt.RK4())
    rtol, atol, dtmin, max_steps = solver
    return dict(solver=mt.Dopri5(), max_steps=max_steps,
                stepsize_controller=mt.PIDController(rtol=rtol, atol=atol, dtmin=dtmin))


def dynamic_setup(P=24, R=8, n_steps=60, depth=6, N=40, seed=0, state_size=2, obs_noise=0.0, env="acrobot",
                  h=0.05, solver=None):
    name = env
    env = make_env(name, obs_noise)
    ys = [f"y{i + 1}" for i in range(env.n_obs)]
    acts = [f"a{i + 1}" for i in range(state_size)]
    tg = [f"tar{i + 1}" for i in range(env.n_targets)]
    vl = [ys + acts + ["u"] + tg, acts + tg]
    lib = mt.NodeLibrary(CONTROL_OPS, vl, [state_size, 1])
    ff = mt.DynamicEvaluator(env, state_size, h, **_ctl_solver(solver))
    data = mt.control_data(env, R, h, None, seed=seed + 1, n_steps=n_steps, mode=_mode(name))
    pop = sample_population(seed, lib, P, 1, max_init_depth=depth, max_nodes=N)[0]
    return env, lib, ff, data, pop


def static_setup(P=24, R=8, n_steps=60, depth=5, N=30, seed=0, obs_noise=0.0, env="acrobot", h=0.05, solver=None):
    name = env
    env = make_env(name, obs_noise)
    vl = [[f"y{i + 1}" for i in range(env.n_obs)] + [f"tar{i + 1}" for i in range(env.n_targets)]]
    lib = mt.NodeLibrary(CONTROL_OPS, vl, [1])
    ff = mt.FeedforwardEvaluator(env, h, **_ctl_solver(solver))
    data = mt.control_data(env, R, h, None, seed=seed + 1, n_steps=n_steps, mode=_mode(name))
    pop = sample_population(seed, lib, P, 1, max_init_depth=depth, max_nodes=N)[0]
    return env, lib, ff, data, pop


def sr_setup(P=24, R=8, n_save=21, save_every=4, h=0.05, depth=5, N=30, seed=0, n_var=2, solver=None):
    """solver: None (fixed-step RK4) or (rtol, atol, dtmin, max_steps) for Dopri5 + PIDController."""
    env = mt.VanDerPolOscillator(0, 0) if n_var == 2 else mt.LinearSystem(n_var)
    lib = mt.NodeLibrary(SR_OPS, [[f"x{i}" for i in range(n_var)]], [n_var])
    if solver is None:
        ff = mt.SREvaluator(solver=mt.RK4(), dt0=h)
    else:
        rtol, atol, dtmin, max_steps = solver
        ff = mt.SREvaluator(solver=mt.Dopri5(), dt0=h, max_steps=max_steps,
                            stepsize_controller=mt.PIDController(rtol=rtol, atol=atol, dtmin=dtmin))
    rng = np.random.default_rng(seed + 1)
    x0 = env.sample_init_states(R, rng)
    ts = (np.arange(n_save, dtype=np.float32) * np.float32(h * save_every)).astype(np.float32)
    ys = mt.ground_truth(env, x0, ts)
    data = (x0, ts, ys, np.zeros((R, 2), np.uint32))
    pop = sample_population(seed, lib, P, 1, max_init_depth=depth, max_nodes=N)[0]
    return env, lib, ff, data, pop


def oracle_model(ff, d, parsimony=0.0):
    env = getattr(ff, "env", None)
    return dict(model=ff.model_id, n_var=d.get("n_var", 4), state_size=getattr(ff, "state_size", 0),
                n_obs=env.n_obs if env else 0, n_control=env.n_control if env else 0,
                n_targets=env.n_targets if env else 0, n_steps=d["n_steps"], save_every=d["save_every"],
                n_save=d["n_save"], h=ff.dt0, max_fitness=ff.max_fitness, parsimony=parsimony,
                prng_impl=d.get("prng_impl", 0), env=d.get("env", 0), solver=d.get("solver", 0),
                max_steps=d.get("max_steps", 0), rtol=d.get("rtol", 0.0), atol=d.get("atol", 0.0),
                dtmin=d.get("dtmin", 0.0), dtmax=d.get("dtmax", 0.0),
                **{f: d.get(f, 0) for f in ("pid_custom", "pid_c1", "pid_c2", "pid_c3", "pid_safety", "pid_factormin",
                                            "pid_factormax", "no_force_dtmin")})


def oracle_rollouts(d, data=None):
    ys = None
    if d.get("ys_true") is not None:
        ys = np.ascontiguousarray(np.transpose(d["ys_true"], (2, 0, 1)))  # back to [R, S, n_var]
    return dict(x0=d["x0"], params=d.get("params"), targets=d.get("targets"), ts=d["ts"], ys_true=ys,
                obs_keys=d.get("obs_keys"), obs_w=d.get("obs_w"))


def bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | nan))


def mismatch_report(a, b, name):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    diff = ~((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b)))
    idx = np.argwhere(diff)
    return f"{name}: {diff.sum()} / {diff.size} differ; first {idx[:5].tolist()} gpu={a[tuple(idx[0])] if len(idx) else None} ref={b[tuple(idx[0])] if len(idx) else None}"


def tree_from_expr(expr, lib, N=30):
    """Reference [N, 4] tree (root at row N-1, descending rows = preorder, a_idx = k-1,
    b_idx = k-1-|subtree(a)|, empty rows packed at the bottom; initialization.py:46-49,
    gp.py:272-296) from a nested tuple: ("op", child[, child]), a variable name or a float
    coefficient."""
    rows = []

    def pre(e):
        if isinstance(e, str):
            rows.append([lib.string_to_node[e], -1, -1, 0.0])
            return 1
        if isinstance(e, (float, np.floating)):
            rows.append([1, -1, -1, float(e)])
            return 1
        op, *children = e
        at = len(rows)
        rows.append(None)
        sizes = [pre(c) for c in children]
        rows[at] = (op, sizes)
        return 1 + sum(sizes)

    pre(expr)
    if len(rows) > N:
        raise ValueError(f"{len(rows)} nodes > max_nodes {N}")
    t = np.zeros((N, 4), np.float32)
    t[:, 1:3] = -1
    for i, r in enumerate(rows):
        k = N - 1 - i
        if isinstance(r, tuple):
            op, sizes = r
            t[k] = [lib.string_to_node[op], k - 1, (k - 1 - sizes[0]) if len(sizes) == 2 else -1, 0.0]
        else:
            t[k] = r
    return t
