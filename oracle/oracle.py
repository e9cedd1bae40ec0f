"""ctypes wrapper of oracle/build/libmtgp_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / CPU baseline -- never by multitreegp_amd.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libmtgp_oracle.so")


def build(force: bool = False) -> str:
    src = [os.path.join(HERE, "mtgp_oracle.c"), os.path.join(HERE, "..", "include", "mtgp_f32math.h"),
           os.path.join(HERE, "..", "include", "mtgp_prng.h"),
           os.path.join(HERE, "..", "include", "mtgp_dopri5.h"), os.path.join(HERE, "..", "include", "mtgp_dual.h"),
           os.path.join(HERE, "..", "include", "mtgp_cstep.h")]
    if force or not os.path.exists(LIB) or any(os.path.getmtime(s) > os.path.getmtime(LIB) for s in src):
        subprocess.run(["make", "-C", HERE, "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB


class OrModel(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int32), ("n_var", ctypes.c_int32), ("state_size", ctypes.c_int32),
                ("n_obs", ctypes.c_int32), ("n_control", ctypes.c_int32), ("n_targets", ctypes.c_int32),
                ("n_steps", ctypes.c_int32), ("save_every", ctypes.c_int32), ("n_save", ctypes.c_int32),
                ("h", ctypes.c_float), ("max_fitness", ctypes.c_float), ("parsimony", ctypes.c_float),
                ("prng_impl", ctypes.c_int32), ("env", ctypes.c_int32),
                ("solver", ctypes.c_int32), ("max_steps", ctypes.c_int32), ("rtol", ctypes.c_float),
                ("atol", ctypes.c_float), ("dtmin", ctypes.c_float), ("dtmax", ctypes.c_float),
                ("pid_custom", ctypes.c_int32), ("pid_c1", ctypes.c_float), ("pid_c2", ctypes.c_float),
                ("pid_c3", ctypes.c_float), ("pid_safety", ctypes.c_float), ("pid_factormin", ctypes.c_float),
                ("pid_factormax", ctypes.c_float), ("no_force_dtmin", ctypes.c_int32),
                ("dp_alt", ctypes.c_int32)]  # oracle-only alternative Dopri5 readings (OR_DP_ALT_*)

_MODEL_DEFAULTS = dict(prng_impl=0, env=0, solver=0, max_steps=0, rtol=0.0, atol=0.0, dtmin=0.0, dtmax=0.0,
                       pid_custom=0, pid_c1=0.0, pid_c2=0.0, pid_c3=0.0, pid_safety=0.0, pid_factormin=0.0,
                       pid_factormax=0.0, no_force_dtmin=0, dp_alt=0)


class OrRollouts(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_void_p), ("params", ctypes.c_void_p), ("targets", ctypes.c_void_p),
                ("ts", ctypes.c_void_p), ("ys_true", ctypes.c_void_p), ("R", ctypes.c_int32),
                ("obs_keys", ctypes.c_void_p), ("obs_w", ctypes.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.oracle_eval_tree.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int]
        L.oracle_eval_tree.restype = ctypes.c_float
        L.oracle_eval.argtypes = [ctypes.POINTER(OrModel), vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(OrRollouts), vp, vp, vp, vp, vp,
                                  vp]
        L.oracle_eval.restype = ctypes.c_int
        L.oracle_eval_ex.argtypes = L.oracle_eval.argtypes + [vp]
        L.oracle_eval_ex.restype = ctypes.c_int
        L.oracle_sincos.argtypes = [vp, vp, vp, ctypes.c_long]
        L.oracle_wrap.argtypes = [vp, vp, ctypes.c_long]
        L.oracle_unary.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_long]
        L.oracle_acro_drift.argtypes = [vp, vp, ctypes.c_float, vp]
        L.oracle_acro_f_obs.argtypes = [vp, vp]
        L.oracle_expf.argtypes = [vp, vp, ctypes.c_long]
        L.oracle_env_drift.argtypes = [ctypes.c_int, vp, vp, ctypes.c_float, vp]
        L.oracle_env_fitness.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_float, ctypes.c_int]
        L.oracle_env_fitness.restype = ctypes.c_float
        L.oracle_acro_fitness.argtypes = [vp, vp, vp, ctypes.c_int]
        L.oracle_acro_fitness.restype = ctypes.c_float
        L.oracle_pairwise_sum.argtypes = [vp, ctypes.c_int]
        L.oracle_pairwise_sum.restype = ctypes.c_float
        L.oracle_obs_normals.argtypes = [vp, ctypes.c_float, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_random_normals.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_threefry.argtypes = [vp, vp, vp, vp, vp, ctypes.c_long]
        L.oracle_erfinv.argtypes = [vp, vp, ctypes.c_long]
        L.oracle_log1p.argtypes = [vp, vp, ctypes.c_long]
        L.oracle_sr_grad.argtypes = [ctypes.POINTER(OrModel), vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(OrRollouts), vp, ctypes.c_int,
                                     vp, vp]
        L.oracle_sr_grad.restype = ctypes.c_int
        L.oracle_ctl_grad.argtypes = L.oracle_sr_grad.argtypes
        L.oracle_ctl_grad.restype = ctypes.c_int
        L.oracle_cs_steps.argtypes = [vp, ctypes.c_int, ctypes.c_float]
        L.oracle_cs_steps.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def eval_tree(tree: np.ndarray, fn_codes: np.ndarray, n_funcs: int, var_start: int, data: np.ndarray) -> np.float32:
    """gp.py:378-388 foriloop on one [N, 4] tree."""
    t = np.ascontiguousarray(tree, np.float32)
    fn = np.ascontiguousarray(fn_codes, np.int8)
    d = np.ascontiguousarray(data, np.float32).reshape(-1)
    if d.size == 0:
        d = np.zeros(1, np.float32)
    return np.float32(lib().oracle_eval_tree(_p(t), t.shape[0], n_funcs, var_start, _p(fn), _p(d),
                                             max(int(np.asarray(data).size), 1)))


def sincos(x: np.ndarray):
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    lib().oracle_sincos(_p(x), _p(s), _p(c), x.size)
    return s, c


def unary(fn: int, x, dx=None):
    """The unary tree operator `fn` (MTGP_FN_SIN .. MTGP_FN_ABS, include/mtgp_f32math.h specs) on
    float32 x; with dx also its tangent (include/mtgp_dual.h) -> y or (y, dy)."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    if dx is None:
        lib().oracle_unary(int(fn), _p(x), None, _p(y), None, x.size)
        return y
    dx = np.ascontiguousarray(dx, np.float32)
    dy = np.empty_like(x)
    lib().oracle_unary(int(fn), _p(x), _p(dx), _p(y), _p(dy), x.size)
    return y, dy


def wrap(x: np.ndarray):
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().oracle_wrap(_p(x), _p(o), x.size)
    return o


def evaluate(model: dict, pop: np.ndarray, library, rollouts: dict, trajectories: bool = False, steps: bool = False):
    """Evaluate a flat population [P, T, N, 4].

    model: dict(model, n_var, state_size, n_obs, n_control, n_targets, n_steps, save_every, n_save,
                h, max_fitness, parsimony[, prng_impl])
    rollouts: dict(x0 [R, n_var], params [R, 4] or None, targets [R, nt] or None, ts [S],
                   ys_true [R, S, n_var] or None[, obs_keys uint32 [R, 2], obs_w [n_obs, n_obs]])
    Returns dict(fitness [P], rollout_fitness [P, R], xs/ys/us/acts [P, R, S, c][, steps [P, R]: the solve's
    step count, Dopri5 attempts])."""
    pop = np.ascontiguousarray(pop, np.float32)
    P, T, N, _ = pop.shape
    m = OrModel(**{k: model.get(k, _MODEL_DEFAULTS[k]) if k in _MODEL_DEFAULTS else model[k]
                   for k, _ in OrModel._fields_})
    x0 = np.ascontiguousarray(rollouts["x0"], np.float32)
    R = x0.shape[0]
    prm = None if rollouts.get("params") is None else np.ascontiguousarray(rollouts["params"], np.float32)
    tg = rollouts.get("targets")
    tg = None if tg is None or np.asarray(tg).size == 0 else np.ascontiguousarray(tg, np.float32)
    ts = np.ascontiguousarray(rollouts["ts"], np.float32)
    yt = rollouts.get("ys_true")
    yt = None if yt is None else np.ascontiguousarray(yt, np.float32)
    keys = rollouts.get("obs_keys")
    keys = None if keys is None else np.ascontiguousarray(keys, np.uint32)
    W = None if keys is None else np.ascontiguousarray(rollouts["obs_w"], np.float32)
    ro = OrRollouts(_p(x0).value, None if prm is None else _p(prm).value, None if tg is None else _p(tg).value,
                    _p(ts).value, None if yt is None else _p(yt).value, R,
                    None if keys is None else _p(keys).value, None if W is None else _p(W).value)
    S = model["n_save"]
    fit = np.empty(P, np.float32)
    rf = np.empty((P, R), np.float32)
    out = {"fitness": fit, "rollout_fitness": rf}
    bufs = [None, None, None, None]
    if trajectories:
        if model["model"] == 3:
            bufs[0] = np.empty((P, R, S, model["n_var"]), np.float32)
        else:
            bufs[0] = np.empty((P, R, S, model["n_var"]), np.float32)
            bufs[1] = np.empty((P, R, S, model["n_obs"]), np.float32)
            bufs[2] = np.empty((P, R, S, model["n_control"]), np.float32)
            if model["model"] == 1:
                bufs[3] = np.empty((P, R, S, model["state_size"]), np.float32)
        for k, b in zip(("xs", "ys", "us", "acts"), bufs):
            if b is not None:
                out[k] = b
    fn = np.ascontiguousarray(library.fn_codes, np.int8)
    st = np.zeros((P, R), np.int32) if steps else None
    rc = lib().oracle_eval_ex(ctypes.byref(m), _p(pop), P, T, N, library.n_funcs, library.var_start, _p(fn),
                              ctypes.byref(ro), _p(fit), _p(rf), *[_p(b) for b in bufs], _p(st))
    if steps:
        out["steps"] = st
    if rc != 0:
        raise RuntimeError(f"oracle_eval failed {rc}")
    return out


def acro_drift(params4, state4, u):
    p = np.ascontiguousarray(params4, np.float32)
    x = np.ascontiguousarray(state4, np.float32)
    o = np.empty(4, np.float32)
    lib().oracle_acro_drift(_p(p), _p(x), ctypes.c_float(u), _p(o))
    return o


def expf(x):
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().oracle_expf(_p(x), _p(o), x.size)
    return o


def env_drift(env: int, params, state, u):
    p = np.ascontiguousarray(params, np.float32)
    x = np.ascontiguousarray(state, np.float32)
    o = np.empty(x.shape[0], np.float32)
    lib().oracle_env_drift(env, _p(p), _p(x), ctypes.c_float(u), _p(o))
    return o


def env_fitness(env: int, xs, us, ts, params, target):
    xs = np.ascontiguousarray(xs, np.float32)
    us = np.ascontiguousarray(us, np.float32).reshape(-1)
    ts = np.ascontiguousarray(ts, np.float32)
    p = np.ascontiguousarray(params, np.float32)
    return np.float32(lib().oracle_env_fitness(env, _p(xs), _p(us), _p(ts), _p(p), ctypes.c_float(target),
                                               xs.shape[0]))


def acro_f_obs(x4):
    x = np.ascontiguousarray(x4, np.float32)
    o = np.empty(4, np.float32)
    lib().oracle_acro_f_obs(_p(x), _p(o))
    return o


def acro_fitness(xs, us, ts):
    xs = np.ascontiguousarray(xs, np.float32)
    us = np.ascontiguousarray(us, np.float32).reshape(-1)
    ts = np.ascontiguousarray(ts, np.float32)
    return np.float32(lib().oracle_acro_fitness(_p(xs), _p(us), _p(ts), ts.shape[0]))


def obs_normals(key, t, n=4, impl=0):
    """normal(fold_in(key, bitcast(t)), (n,)) of the PRNG spec (include/mtgp_prng.h)."""
    k = np.ascontiguousarray(key, np.uint32)
    o = np.empty(n, np.float32)
    lib().oracle_obs_normals(_p(k), ctypes.c_float(t), n, impl, _p(o))
    return o


def random_normals(key, n, impl=0):
    """jax.random.normal(key, (n,)) of the PRNG spec."""
    k = np.ascontiguousarray(key, np.uint32)
    o = np.empty(n, np.float32)
    lib().oracle_random_normals(_p(k), n, impl, _p(o))
    return o


def threefry(key, x0, x1):
    k = np.ascontiguousarray(key, np.uint32)
    x0 = np.ascontiguousarray(x0, np.uint32)
    x1 = np.ascontiguousarray(x1, np.uint32)
    y0, y1 = np.empty_like(x0), np.empty_like(x1)
    lib().oracle_threefry(_p(k), _p(x0), _p(x1), _p(y0), _p(y1), x0.size)
    return y0, y1


def erfinv(x):
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().oracle_erfinv(_p(x), _p(o), x.size)
    return o


def log1p(x):
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().oracle_log1p(_p(x), _p(o), x.size)
    return o


def cs_steps(ts, dt0) -> int:
    """Steps of diffrax's ConstantStepSize grid from ts[0] to ts[-1] (include/mtgp_cstep.h)."""
    ts = np.ascontiguousarray(ts, np.float32)
    return int(lib().oracle_cs_steps(_p(ts), ts.shape[0], ctypes.c_float(dt0)))


def pairwise_sum(v):
    v = np.ascontiguousarray(v, np.float32)
    return np.float32(lib().oracle_pairwise_sum(_p(v), v.shape[0]))


def sr_grad(model: dict, pop: np.ndarray, library, rollouts: dict):
    """Loss [P] and d loss / d coefficient [P, K] of the SR evaluator (forward mode), one entry per
    coefficient row (f == 1) of each candidate in row-major (tree, row) order; K = the largest
    count (unused entries 0).  -> (loss, grad, rows: list of [(t, i)] per candidate)."""
    return _grad("oracle_sr_grad", model, pop, library, rollouts)


def ctl_grad(model: dict, pop: np.ndarray, library, rollouts: dict):
    """sr_grad for the dynamic / static control evaluators (fixed-step RK4 / Euler, every
    environment, observation noise included): loss = the evaluator's fitness without parsimony."""
    return _grad("oracle_ctl_grad", model, pop, library, rollouts)


def _grad(fname, model, pop, library, rollouts):
    pop = np.ascontiguousarray(pop, np.float32)
    P, T, N, _ = pop.shape
    rows = [np.argwhere(c[..., 0] == np.float32(1.0)) for c in pop]
    K = max([len(r) for r in rows] + [1])
    prow = np.full((P, K), -1, np.int32)
    for p, r in enumerate(rows):
        prow[p, : len(r)] = r[:, 0] * N + r[:, 1]
    m = OrModel(**{k: model.get(k, _MODEL_DEFAULTS[k]) if k in _MODEL_DEFAULTS else model[k]
                   for k, _ in OrModel._fields_})
    x0 = np.ascontiguousarray(rollouts["x0"], np.float32)
    ts = np.ascontiguousarray(rollouts["ts"], np.float32)
    yt = rollouts.get("ys_true")
    yt = None if yt is None else np.ascontiguousarray(yt, np.float32)
    prm = None if rollouts.get("params") is None else np.ascontiguousarray(rollouts["params"], np.float32)
    tg = rollouts.get("targets")
    tg = None if tg is None or np.asarray(tg).size == 0 else np.ascontiguousarray(tg, np.float32)
    keys = rollouts.get("obs_keys")
    keys = None if keys is None else np.ascontiguousarray(keys, np.uint32)
    W = None if keys is None else np.ascontiguousarray(rollouts["obs_w"], np.float32)
    ro = OrRollouts(_p(x0).value, None if prm is None else _p(prm).value, None if tg is None else _p(tg).value,
                    _p(ts).value, None if yt is None else _p(yt).value, x0.shape[0],
                    None if keys is None else _p(keys).value, None if W is None else _p(W).value)
    loss = np.empty(P, np.float32)
    grad = np.empty((P, K), np.float32)
    fn = np.ascontiguousarray(library.fn_codes, np.int8)
    rc = getattr(lib(), fname)(ctypes.byref(m), _p(pop), P, T, N, library.n_funcs, library.var_start, _p(fn),
                               ctypes.byref(ro), _p(prow), K, _p(loss), _p(grad))
    if rc != 0:
        raise RuntimeError(f"{fname} failed {rc}")
    return loss, grad, rows
