"""Fitness-function plugins: MI355X counterparts of MultiTreeGP/evaluators/*.py.

Each class keeps the reference constructor signature and exposes the same two calls --
``__call__(coefficients, nodes, data, tree_evaluator)`` (one candidate -> fitness) and
``evaluate_candidate(candidate, data, tree_evaluator)`` (trajectories + per-rollout fitness)
-- but the work is done by the fused HIP kernel (multitreegp_amd/csrc/mtgp_kernels.hip).
The population path (``GeneticProgramming.evaluate_population``) batches all candidates into
one launch; these per-candidate calls exist for API parity and trajectory inspection.

Solver: BASELINE.json prescribes an explicit fixed-step RK4 (``RK4()`` or "rk4" with
``ConstantStepSize()``); omitting ``solver`` gives the reference's default ``Euler()`` (fixed
step).  Both follow diffrax.ConstantStepSize exactly (include/mtgp_cstep.h): accumulated f32 step
ends, per-step dt, SaveAt(ts) for any non-decreasing ts through the dense output.  The notebooks' adaptive ``Dopri5()`` + ``PIDController(rtol, atol, dtmin)`` (SURVEY.md
§8f row 2, spec include/mtgp_dopri5.h) runs on the GPU for the dynamic and static control
evaluators (every environment) and for ``SREvaluator``.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from .. import _native as nat
from .. import prng


class RK4:
    """Classical 4-stage Runge-Kutta, fixed step dt0 (diffrax.RK4 + ConstantStepSize)."""
    name = "RK4"

    def __repr__(self):
        return "RK4()"


class Euler:
    """Explicit Euler, fixed step dt0 (diffrax.Euler + ConstantStepSize): the reference
    evaluators' default solver (dynamic_evaluate.py:11, feedforward_evaluate.py:11,
    SR_evaluator.py:21); y1 = y0 + f(t0, y0) * dt0, product and sum rounded separately."""
    name = "Euler"

    def __repr__(self):
        return "Euler()"


class ConstantStepSize:
    name = "ConstantStepSize"

    def __repr__(self):
        return "ConstantStepSize()"


class Dopri5:
    """diffrax.Dopri5: Dormand-Prince 5(4), FSAL, with the Shampine dense output."""
    name = "Dopri5"

    def __repr__(self):
        return "Dopri5()"


class PIDController:
    """diffrax.PIDController (defaults: pcoeff 0, icoeff 1, dcoeff 0 -- an integral controller;
    safety 0.9, factormin 0.2, factormax 10, force_dtmin True, rms norm).  Any coefficients run on
    the GPU (include/mtgp_dopri5.h mtgp_dp_factor_pid, restated from diffrax's adapt_step_size);
    force_dtmin=False ends a solve whose step falls below dtmin (RESULTS.dt_min_reached, the
    remaining save points +inf as with throw=False)."""
    name = "PIDController"

    def __init__(self, rtol: float, atol: float, pcoeff: float = 0.0, icoeff: float = 1.0, dcoeff: float = 0.0,
                 dtmin: float = None, dtmax: float = None, force_dtmin: bool = True, factormin: float = 0.2,
                 factormax: float = 10.0, safety: float = 0.9):
        if rtol < 0 or atol < 0:
            raise ValueError("rtol and atol must be >= 0")
        self.rtol, self.atol = float(rtol), float(atol)
        self.dtmin = None if dtmin is None else float(dtmin)
        self.dtmax = None if dtmax is None else float(dtmax)
        self.pcoeff, self.icoeff, self.dcoeff = float(pcoeff), float(icoeff), float(dcoeff)
        self.factormin, self.factormax, self.safety = float(factormin), float(factormax), float(safety)
        self.force_dtmin = bool(force_dtmin)

    def is_default(self) -> bool:
        return (self.pcoeff, self.icoeff, self.dcoeff, self.factormin, self.factormax, self.safety) == \
            (0.0, 1.0, 0.0, 0.2, 10.0, 0.9)

    def model_fields(self) -> dict:
        """MtgpModel ABI v15 fields: error order 5 (Dopri5), exponents rounded to float32."""
        out = dict(no_force_dtmin=0 if self.force_dtmin else 1, pid_custom=0)
        if not self.is_default():
            p, i, d = self.pcoeff, self.icoeff, self.dcoeff
            out.update(pid_custom=1, pid_c1=float(np.float32((i + p + d) / 5.0)),
                       pid_c2=float(np.float32(-(p + 2.0 * d) / 5.0)), pid_c3=float(np.float32(d / 5.0)),
                       pid_safety=float(np.float32(self.safety)), pid_factormin=float(np.float32(self.factormin)),
                       pid_factormax=float(np.float32(self.factormax)))
        return out

    def __repr__(self):
        return (f"PIDController(rtol={self.rtol}, atol={self.atol}, pcoeff={self.pcoeff}, icoeff={self.icoeff}, "
                f"dcoeff={self.dcoeff}, dtmin={self.dtmin}, dtmax={self.dtmax}, force_dtmin={self.force_dtmin})")


def _check_solver(solver, controller, adaptive_ok: bool = False) -> str:
    """-> "rk4", "euler" or "dopri5" (the latter needs a PIDController and an evaluator that
    supports it)."""
    sname = solver.lower() if isinstance(solver, str) else getattr(solver, "name", type(solver).__name__)
    sname = str(sname).lower()
    cname = None if controller is None else getattr(controller, "name", type(controller).__name__)
    if sname == "dopri5":
        if not adaptive_ok:
            raise NotImplementedError(f"solver {solver!r}: adaptive Dopri5 is not implemented here")
        if cname != "PIDController":
            raise NotImplementedError("Dopri5 needs a PIDController (fixed-step Dopri5 is not implemented)")
        return "dopri5"
    if sname not in ("rk4", "euler"):
        raise NotImplementedError(f"solver {solver!r}: implemented solvers are Euler and RK4 (fixed step) and "
                                  "Dopri5 (PID)")
    if cname is not None and cname != "ConstantStepSize":
        raise NotImplementedError(f"stepsize_controller {controller!r}: {sname} runs with ConstantStepSize only")
    return sname


def _check_max_steps(max_steps) -> int:
    """diffeqsolve takes a positive max_steps (or None, which the reference never passes: dyn.py:11,
    ff.py:11, sr.py:21 default 16**4).  The C entry reads max_steps 0 as "no limit" for the
    fixed-step solve; the Python mirror never hands it one."""
    if isinstance(max_steps, bool) or int(max_steps) != max_steps or int(max_steps) <= 0:
        raise ValueError(f"max_steps must be a positive integer, got {max_steps!r}")
    return int(max_steps)


def _solver_fields(kind: str, controller, max_steps: int) -> dict:
    if kind != "dopri5":  # ConstantStepSize: max_steps bounds the fixed-step solve too (ABI v18)
        return dict(solver=nat.SOLVER_EULER if kind == "euler" else nat.SOLVER_RK4, max_steps=int(max_steps), rtol=0.0,
                    atol=0.0, dtmin=0.0, dtmax=0.0)
    return dict(solver=nat.SOLVER_DOPRI5, max_steps=int(max_steps), rtol=controller.rtol, atol=controller.atol,
                dtmin=controller.dtmin or 0.0, dtmax=controller.dtmax or 0.0, **controller.model_fields())


def constant_step_grid(ts: np.ndarray, dt0: float, max_steps: Optional[int] = None) -> np.ndarray:
    """Step ends of diffrax.ConstantStepSize through diffeqsolve(t0=ts[0], t1=ts[-1], dt0)
    (include/mtgp_cstep.h): float32, accumulated t += dt0 (the first end min(t0 + dt0, t1), later
    ends t1 once past t1 - 1e-6), at most max_steps of them, ending before a second step that
    would not advance t (mtgp_cs_advancing).  -> float32 [n_steps + 1] = the step boundaries from
    ts[0].  The kernels follow the same loop on the device; this host copy sizes the work (bench
    unit-steps, MtgpModel.n_steps).  The accumulation runs in chunks (np.add.accumulate adds left
    to right in float32, the device's order), so a grid whose f32 sums need many more steps than
    (t1 - t0) / dt0 is counted exactly, bounded by max_steps."""
    f = np.float32
    ts = np.asarray(ts, dtype=f)
    t0, t1, dt0 = f(ts[0]), f(ts[-1]), f(dt0)
    if not dt0 > 0 or not np.isfinite(dt0):
        raise ValueError(f"dt0 must be a positive finite number, got {dt0}")
    if not t0 < t1:
        return np.array([t0], f)
    limit = int(max_steps) if max_steps is not None and max_steps > 0 else None
    tol = f(t1 - f(1e-6))
    ends = [np.array([min(f(t0 + dt0), t1)], f)]
    n, last = 1, ends[0][0]
    done = last >= t1 or (limit is not None and n >= limit)
    chunk = int(min(np.ceil((float(t1) - float(t0)) / float(dt0)) + 4, 1 << 22))
    while not done:
        if limit is not None:
            chunk = max(1, min(chunk, limit - n))
        e = np.add.accumulate(np.concatenate([[last], np.full(chunk, dt0, f)]).astype(f), dtype=f)[1:]
        over = np.nonzero(e > tol)[0]
        stall = np.nonzero(e <= np.concatenate([[last], e[:-1]]))[0]  # tn <= t: this step would not advance
        cut = len(e)
        if len(stall):
            cut = min(cut, int(stall[0]))
            done = True
        if len(over) and over[0] < cut:
            cut = int(over[0]) + 1
            e = e.copy()
            e[cut - 1] = t1  # _clip_to_end
            done = True
        ends.append(e[:cut])
        n += cut
        last = e[cut - 1] if cut else last
        if limit is not None and n >= limit:
            done = True
        chunk *= 2
    out = np.concatenate(ends)
    if limit is not None:
        out = out[:limit]
    return np.concatenate([[t0], out]).astype(f)


def fixed_schedule(ts: np.ndarray, dt0: float, max_steps: int) -> Tuple[int, int, int]:
    """Euler / RK4 with ConstantStepSize (ABI v18): save points straight from ts, any non-decreasing
    grid (SaveAt(ts) through the dense output), steps from the accumulated dt0 grid.
    -> (n_steps of the grid, save_every 1 (unused), n_save)."""
    ts = np.asarray(ts, dtype=np.float32)
    S = int(ts.shape[0])
    if S < 2 or np.any(np.diff(ts) < 0) or not np.all(np.isfinite(ts)):
        raise ValueError("ts needs at least two finite non-decreasing save points")
    if not ts[0] < ts[-1]:  # diffrax's t0 == t1 special case (y0 at every save point): not built
        raise ValueError("ts[0] == ts[-1]: an empty solve interval")
    n_steps = len(constant_step_grid(ts, dt0, max_steps)) - 1
    return n_steps, 1, S


rk4_schedule = fixed_schedule  # (round-1 name)


def adaptive_schedule(ts: np.ndarray) -> Tuple[int, int, int]:
    """Dopri5: save points straight from ts (SaveAt(ts)), any non-decreasing grid.
    -> (n_steps 0, save_every 1, n_save)."""
    ts = np.asarray(ts, dtype=np.float32)
    S = int(ts.shape[0])
    if S < 2 or np.any(np.diff(ts) < 0):
        raise ValueError("ts needs at least two non-decreasing save points")
    if not ts[0] < ts[-1]:  # diffrax's t0 == t1 special case (y0 at every save point): not built
        raise ValueError("ts[0] == ts[-1]: an empty solve interval")
    return 0, 1, S


def acrobot_mask(ts: np.ndarray) -> Optional[Tuple[np.ndarray, bool]]:
    """The Acrobot cost mask `costs = where(ts / (ts[1] - ts[0]) > first_success, 0, cost)`
    (acrobot.py:82) as the count table MtgpRollouts.fit_kof.  Save k's cost is kept for a
    first_success f unless f32(ratio_k) > f32(f), so it is masked exactly for the integers
    f < m_k with m_k = #{f in [0, S) : f < ratio_k} -- ceil(ratio_k) clipped to [0, S], 0 for a
    NaN ratio (NaN > f is False: kept), S for +inf (masked), 0 for -inf (kept).  When m_k is
    non-decreasing in k the kept costs for every f are the first kof[f] = #{k : m_k <= f} saves.
    That holds for every valid ts: with ts[1] > ts[0] the ratio is non-decreasing, and with
    ts[1] == ts[0] (a repeated first save time) the ratio is NaN where ts_k == 0, -inf below 0 and
    +inf above, i.e. the kept saves are those with ts_k <= 0 for every f.
    None when the ratio of save k lies in (k - 1, k + 1] for every k (ts from 0 on a uniform grid:
    the kernels' one-pass fitness).  -> (kof int32 [S], need_hist: some f >= 1 has
    1 <= kof[f] <= f, so the kernels keep the per-save cost prefixes in MtgpOutputs.fit_hist)."""
    ts = np.asarray(ts, dtype=np.float32)
    S = int(ts.shape[0])
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = ts / np.float32(ts[1] - ts[0])
    k = np.arange(S, dtype=np.float32)
    if np.all(ratio > k - 1) and np.all(ratio <= k + 1):
        return None
    r = ratio.astype(np.float64)  # exact: every f32 ratio and every integer f < S compare the same
    with np.errstate(invalid="ignore"):
        m = np.where(np.isnan(r) | (r <= 0), 0.0, np.minimum(np.ceil(np.where(np.isfinite(r), r, S)), S))
    m = m.astype(np.int64)
    if np.any(np.diff(m) < 0):
        raise NotImplementedError("Acrobot fitness mask: the kept save points are not a prefix for every "
                                  "first_success (ts must be non-decreasing)")
    kof = np.searchsorted(m, np.arange(S), side="right").astype(np.int32)
    f = np.arange(S)
    need_hist = bool(np.any((f >= 1) & (kof >= 1) & (kof <= f)))
    return kof, need_hist


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


class _CandidateAPI:
    """``__call__`` / ``evaluate_candidate`` of the reference evaluators, run on the GPU."""

    def _single(self, candidate, data, tree_evaluator, traj: bool):
        import torch
        if not hasattr(tree_evaluator, "engine"):
            raise TypeError("tree_evaluator must be GeneticProgramming.vmap_foriloop of multitreegp_amd")
        eng = tree_evaluator.engine(self)
        cand = np.asarray(candidate, dtype=np.float32)
        pop = torch.from_numpy(np.ascontiguousarray(cand[None])).to(eng.device)
        res = eng.evaluate(pop, data, trajectories=traj, rollout_fitness=True)
        return res

    def __call__(self, coefficients, nodes, data, tree_evaluator) -> float:
        """dyn.py:37-52 / ff.py:36-51 / sr.py:30-45: one candidate -> clipped mean fitness."""
        cand = np.concatenate([np.asarray(nodes, np.float32), np.asarray(coefficients, np.float32)], axis=-1)
        return float(self._single(cand, data, tree_evaluator, False)["fitness"][0].item())

    def evaluate_candidate(self, candidate, data, tree_evaluator):
        """dyn.py:54-63 -> (xs, ys, us, activities, fitness); ff.py:53-62 -> (xs, ys, us, fitness);
        sr.py:47-55 -> (fitness, pred_ys).  Arrays in the reference layout [R, S, c]."""
        from ..engine import to_reference_layout
        res = self._single(candidate, data, tree_evaluator, True)
        R = res["rollout_fitness"].shape[1]
        fit = res["rollout_fitness"][0].cpu().numpy()
        get = lambda k: to_reference_layout(res[k], 1, R)[0]
        if self.model_id == nat.MODEL_SR:
            return fit, get("xs")
        if self.model_id == nat.MODEL_ACROBOT_STATIC:
            return get("xs"), get("ys"), get("us"), fit
        return get("xs"), get("ys"), get("us"), get("acts"), fit


class _TreeOnly:
    """Pseudo fitness config used by TreeEvaluator: one program per tree, plain data vector."""
    model_id = 0
    state_size = 0
    dt0 = 0.0
    max_fitness = 0.0

    def __init__(self, n_trees: int, n_data: int):
        self._t, self._d = n_trees, n_data

    def prepare(self, data):
        return {}

    def n_data(self):
        return self._d

    def program_specs(self):
        return [(t, self._d, 0) for t in range(self._t)], {}


# environments with a kernel functor (mtgp.h MTGP_ENV_*): class name -> (env id, n_var, n_params)
ENVIRONMENTS = {
    "Acrobot": (nat.ENV_ACROBOT, 4, 4),                          # acrobot.py:7-87
    "HarmonicOscillator": (nat.ENV_HARMONIC_OSCILLATOR, 2, 2),   # harmonic_oscillator.py:8-80
    "StirredTankReactor": (nat.ENV_STIRRED_TANK_REACTOR, 3, 8),  # reactor.py:7-81
}


class _ControlEvaluator(_CandidateAPI):
    max_fitness = 1e4

    def __init__(self, env, dt0: float, solver=None, max_steps: int = 16 ** 4, stepsize_controller=None):
        solver = solver if solver is not None else Euler()  # the reference default (dyn.py:11, ff.py:11)
        self.solver_kind = _check_solver(solver, stepsize_controller, adaptive_ok=True)
        name = type(env).__name__
        if name not in ENVIRONMENTS:
            # CartPole / Acrobot2 / ChangingHarmonicOscillator / HarmonicOscillator2 have no
            # cond_fn_nan, which the reference evaluators require (dyn.py:94, ff.py:91)
            raise NotImplementedError(f"environment {name}: the MI355X path runs {sorted(ENVIRONMENTS)}")
        self.env_id, n_var, self.n_params = ENVIRONMENTS[name]
        if not 1 <= env.n_obs <= n_var:
            raise ValueError(f"{name}: n_obs must be in [1, {n_var}] (C = eye(n_var)[:n_obs])")
        if env.n_control != 1 or (self.env_id != nat.ENV_ACROBOT and env.n_targets != 1):
            raise NotImplementedError(f"{name}: one control and one target only")
        self.env = env
        self.obs_size = env.n_obs
        self.control_size = env.n_control
        self.latent_size = env.n_var * env.n_dim
        self.dt0 = float(dt0)
        self.solver = solver
        self.max_steps = _check_max_steps(max_steps)
        self.stepsize_controller = stepsize_controller

    def obs_gap(self) -> Tuple[int, int]:
        """(gap_at, gap) of MtgpProgramSpec: the kernels hold all n_var observation slots, so with
        n_obs < n_var (C = eye(n_var)[:n_obs], control_environment_base.py:47) the data slots after
        the observations sit n_var - n_obs slots later than in the reference's data vector."""
        return (self.obs_size, self.env.n_var - self.obs_size)

    def prepare(self, data) -> dict:
        """Reference data tuple (x0, ts, targets, process_keys, obs_keys, params) -> arrays.

        With env.obs_noise != 0 the per-rollout obs_noise_keys (uint32 [R, 2], jax.random key
        data) drive the in-kernel observation noise (control_environment_base.py:43-48); the
        random-bits layout follows ``prng.set_threefry_partitionable`` (JAX's config flag)."""
        x0, ts, targets, _pk, obs_keys, params = data
        x0 = _f32(x0)
        R = x0.shape[0]
        nv = self.env.n_var
        if x0.ndim != 2 or x0.shape[1] != nv:
            raise ValueError(f"{type(self.env).__name__} x0 must be [R, {nv}]")
        if params is None:
            raise ValueError("params tuple required (env.sample_params)")
        if len(params) != self.n_params:
            raise ValueError(f"{type(self.env).__name__} takes {self.n_params} parameters per rollout")
        for p in params:
            if np.asarray(p).size != R:
                raise NotImplementedError("time-varying parameters ([R, S]: 'Switch'/'Decay' modes) are not supported")
        prm = np.stack([_f32(p).reshape(R) for p in params], axis=1)
        tg = _f32(targets).reshape(R, -1)
        if tg.shape[1] != self.env.n_targets:
            raise ValueError(f"targets must be [R, {self.env.n_targets}]")
        if self.solver_kind == "dopri5":
            n_steps, save_every, S = adaptive_schedule(ts)
        else:
            n_steps, save_every, S = fixed_schedule(ts, self.dt0, self.max_steps)
        mask = acrobot_mask(ts) if self.env_id == nat.ENV_ACROBOT else None
        out = dict(x0=x0, params=_f32(prm), targets=tg, ts=_f32(ts), ys_true=None, R=R, n_var=nv, env=self.env_id,
                   n_steps=n_steps, save_every=save_every, n_save=S, prng_impl=prng.prng_impl_code(),
                   **_solver_fields(self.solver_kind, self.stepsize_controller, self.max_steps))
        if mask is not None:  # ts off the one-pass mask: the general prefix form (mtgp.h fit_kof)
            out["fit_kof"], out["fit_need_hist"] = mask
        obs_noise = float(getattr(self.env, "obs_noise", 0.0))
        if obs_noise != 0.0:
            keys = np.ascontiguousarray(np.asarray(obs_keys), dtype=np.uint32)
            if keys.shape != (R, 2):
                raise ValueError(f"obs_noise_keys must be uint32 [R, 2] key data, got {keys.shape}")
            out["obs_keys"] = keys
            # W = obs_noise * eye(n_obs) (acrobot.py:49, harmonic_oscillator.py:66), times the
            # per-channel scale for the reactor (reactor.py:43), formed in float32 like the reference
            out["obs_w"] = self.env.obs_matrix()
        return out


class DynamicEvaluator(_ControlEvaluator):
    """dynamic_evaluate.Evaluator (dynamic_evaluate.py:10-118): state_size hidden-state trees
    followed by n_control readout trees."""
    model_id = nat.MODEL_ACROBOT_DYNAMIC

    def __init__(self, env, state_size: int, dt0: float, solver=None, max_steps: int = 16 ** 4,
                 stepsize_controller=None):
        super().__init__(env, dt0, solver, max_steps, stepsize_controller)
        self.state_size = int(state_size)
        if self.state_size < 1:
            raise ValueError("state_size must be >= 1")
        if self.state_size > 3:  # the runtime-state-size interpreter kernels (mtgp_kernels.hip kNaRuntime / kNaWide)
            slots = 16 if self.state_size <= 8 else 24
            need = env.n_var * env.n_dim + self.state_size + env.n_control + env.n_targets
            if self.state_size > 16 or need > slots:
                raise NotImplementedError(f"state_size {self.state_size}: the MI355X kernels run state_size <= 16 "
                                          f"with a data vector of at most {slots} slots (this one needs {need})")

    def n_trees(self) -> int:
        return self.state_size + self.control_size

    def n_data(self) -> int:
        return self.obs_size + self.state_size + self.control_size + self.env.n_targets

    def program_specs(self) -> Tuple[List[Tuple[int, int, int]], dict]:
        no, ss, nu = self.obs_size, self.state_size, self.control_size
        D = self.n_data()
        ymask = (1 << no) - 1
        umask = ((1 << nu) - 1) << (no + ss)
        # order: readout | state equations | save-point readout, so that the JIT can chain the state
        # programs into the save-point readout (mtgp.h MtgpJitChain: it must follow the state programs)
        gap = self.obs_gap()
        specs = [(ss + j, D, ymask | umask) + gap for j in range(nu)]     # readout in _drift (dyn.py:113)
        specs += [(t, D, 0) + gap for t in range(ss)]                     # state equation [y, a, u, tg]
        specs += [(ss + j, D, umask) + gap for j in range(nu)]            # readout at saves (dyn.py:101)
        roles = dict(prog_state=nu, prog_readout=0, prog_readout_save=ss + nu, readout_save_same=-1)
        return specs, roles


class FeedforwardEvaluator(_ControlEvaluator):
    """feedforward_evaluate.Evaluator (feedforward_evaluate.py:10-110): u = policy([y, target])."""
    model_id = nat.MODEL_ACROBOT_STATIC
    state_size = 0

    def n_trees(self) -> int:
        return self.control_size

    def n_data(self) -> int:
        return self.obs_size + self.env.n_targets

    def program_specs(self):
        specs = [(j, self.n_data(), 0) + self.obs_gap() for j in range(self.control_size)]
        roles = dict(prog_state=-1, prog_readout=0, prog_readout_save=0, readout_save_same=1)
        return specs, roles


class SREvaluator(_CandidateAPI):
    """SR_evaluator.Evaluator (SR_evaluator.py:9-94): dx = trees(x), MSE fitness."""
    model_id = nat.MODEL_SR
    max_fitness = 1e5

    def __init__(self, solver=None, dt0: float = 0.01, max_steps: int = 16 ** 4, stepsize_controller=None):
        solver = solver if solver is not None else Euler()  # the reference default (sr.py:21)
        self.solver_kind = _check_solver(solver, stepsize_controller, adaptive_ok=True)
        self.dt0 = float(dt0)
        self.solver = solver
        self.max_steps = _check_max_steps(max_steps)
        self.stepsize_controller = stepsize_controller
        self.state_size = 0
        self._n_var = None

    def prepare(self, data) -> dict:
        """Reference data tuple (x0s, ts, ys, process_noise_keys)."""
        x0, ts, ys = data[0], data[1], data[2]
        x0 = _f32(x0)
        R, nv = x0.shape
        ys = _f32(ys)
        if ys.shape[0] != R or ys.shape[2] != nv:
            raise ValueError("ys must be [R, S, n_var]")
        if self.solver_kind == "dopri5":  # save points straight from ts, steps from the controller
            n_steps, save_every, S = adaptive_schedule(ts)
        else:
            n_steps, save_every, S = fixed_schedule(ts, self.dt0, self.max_steps)
        if ys.shape[1] != S:
            raise ValueError("ys must have len(ts) save points")
        ys_tm = np.ascontiguousarray(np.transpose(ys, (1, 2, 0)))  # [S, n_var, R] time-major
        self._n_var = nv
        return dict(x0=x0, params=None, targets=None, ts=_f32(ts), ys_true=ys_tm, R=R,
                    n_steps=n_steps, save_every=save_every, n_save=S, n_var=nv,
                    **_solver_fields(self.solver_kind, self.stepsize_controller, self.max_steps))

    def n_trees(self) -> int:
        return self._n_var

    def n_data(self) -> int:
        return self._n_var

    def program_specs(self):
        nv = self._n_var
        specs = [(i, nv, 0) for i in range(nv)]
        roles = dict(prog_state=0, prog_readout=-1, prog_readout_save=-1, readout_save_same=0)
        return specs, roles


__all__ = ["RK4", "Euler", "ConstantStepSize", "Dopri5", "PIDController", "DynamicEvaluator", "FeedforwardEvaluator", "SREvaluator",
           "fixed_schedule", "rk4_schedule", "constant_step_grid", "adaptive_schedule", "acrobot_mask"]
