"""Coefficient optimisation (gp.py:418-473).

Every 5th generation after generation 10 the reference takes the 50 best candidates and runs
``gradient_steps`` optimiser steps on their coefficients:

* ``epoch`` (gp.py:435-452): ``loss, grads = vmap(value_and_grad(partial_ff))(values, nodes,
  data)``, ``updates = optimiser.update(grads)``, ``values += updates``, emitting the PRE-update
  candidates and their loss;
* ``optimise`` (gp.py:454-473): the best loss over the epochs and the candidate it belongs to
  (first minimum).

Here the loss and gradient come from ``mtgp_sr_grad`` (the SR evaluator) and ``mtgp_ctl_grad``
(the dynamic and static control evaluators, every environment; csrc/mtgp_grad.hip): forward-mode
dual numbers through the same RK4 / Euler solve as the evaluator, one GPU lane per (candidate,
parameter, rollout).  The parameters are the coefficient rows (``f == 1``) of every tree: the
host turns the rows of one chunk into variable rows that read data slots ``n_data + k`` (after
the evaluator's data vector), so the ordinary flattener produces the programs; other rows keep
their reference meaning.  The optimiser (optax's Adam restated in float32 numpy, ``adam``, or any
object with optax's init / update) runs on the host with one state per candidate, as the
reference's ``jax.vmap(self.optimiser.init)`` / ``jax.vmap(self.optimiser.update)`` do.

Deviation (documented in DESIGN.md): JAX differentiates w.r.t. the whole value column, which
also reaches entries read through a reference to a LATER row (the "original column" case of
body_fun, gp.py:366-372).  Trees built by the reference's operators never read such an entry
(children sit below their parent, leaves ignore their index fields), so for them the gradients
agree; for arbitrary arrays only coefficient rows are optimised.

Adaptive solves (Dopri5 + PIDController): the gradient is the derivative of the discrete
solution along the step sequence the primal solve took -- step sizes, accept / reject decisions
and the NaN event carry no tangent.  That is diffrax's own rule under ``DirectAdjoint``: its
PIDController applies ``lax.stop_gradient`` to the initial step size (``init``) and to the
multiplicative step-size factor (``adapt_step_size``), so every step size has a zero tangent and
``jax.grad`` differentiates the discretised solution, not the ODE solution (diffrax is absent here:
restated from its published source, not executed).  Central differences of the float32 loss DO
move the step sizes, so they differ from it where a perturbation changes the accept / reject
sequence; over every finite, unclipped candidate (no smoothness filter, tests/test_coefficients.py)
the median relative difference is 7e-4, 75th percentile 3e-3, 90th 3e-2.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _native as nat


# ------------------------------------------------------------------------ optimiser
@dataclass
class AdamState:
    count: int
    mu: np.ndarray
    nu: np.ndarray


class Adam:
    """optax.adam(learning_rate, b1, b2, eps, eps_root) restated in float32 (optax
    scale_by_adam + scale_by_learning_rate): mu = (1-b1) g + b1 mu; nu = (1-b2) g^2 + b2 nu;
    mu_hat = mu / (1 - b1^t); nu_hat = nu / (1 - b2^t); update = -lr mu_hat / (sqrt(nu_hat +
    eps_root) + eps).  The reference's default (gp.py:79) is adam(0.001, 0.9, 0.999)."""

    def __init__(self, learning_rate: float = 0.001, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
                 eps_root: float = 0.0):
        self.learning_rate, self.b1, self.b2, self.eps, self.eps_root = learning_rate, b1, b2, eps, eps_root

    def init(self, params) -> AdamState:
        z = np.zeros(np.shape(params), np.float32)
        return AdamState(0, z, z.copy())

    def update(self, updates, state: AdamState, params=None):
        f = np.float32
        g = np.asarray(updates, np.float32)
        count = state.count + 1
        with np.errstate(over="ignore", invalid="ignore", divide="ignore"):  # float32 as jnp: inf / NaN, silently
            mu = f(1 - self.b1) * g + f(self.b1) * state.mu
            nu = f(1 - self.b2) * (g * g) + f(self.b2) * state.nu
            mu_hat = mu / (f(1) - f(self.b1) ** f(count))
            nu_hat = nu / (f(1) - f(self.b2) ** f(count))
            u = mu_hat / (np.sqrt(nu_hat + f(self.eps_root)) + f(self.eps))
        return (f(-self.learning_rate) * u).astype(np.float32), AdamState(count, mu, nu)


def adam(learning_rate: float = 0.001, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
         eps_root: float = 0.0) -> Adam:
    return Adam(learning_rate, b1, b2, eps, eps_root)


# ------------------------------------------------------------------- parameterise
def _f2i_sat(v: np.ndarray) -> np.ndarray:
    """f32 -> int32 truncation, saturating, NaN -> 0 (the flattener's int())."""
    v = np.asarray(v, np.float64)
    out = np.where(np.isnan(v), 0.0, np.clip(np.trunc(v), -2147483648.0, 2147483647.0))
    return out.astype(np.int64)


def coefficient_rows(candidates: np.ndarray) -> List[np.ndarray]:
    """Per candidate: the (tree, row) index pairs of its coefficient rows, row-major order."""
    return [np.argwhere(c[..., 0] == np.float32(1.0)) for c in candidates]


def parameterise(candidates: np.ndarray, rows: List[np.ndarray], lib, n_data: int, lo: int, hi: int):
    """Candidates with coefficient rows lo..hi-1 (per candidate) turned into variable rows that
    read data slots n_data + k.  Every other row keeps its meaning under the extended library:
    operator indices above the library are clamped as lax.switch does, variables past the data
    vector are pointed at its last slot (the flattener's clamp).
    -> (population [B, T, N, 4], theta [B, K], nparam [B], K, extended MtgpNodeLibrary)."""
    B = candidates.shape[0]
    pop = np.array(candidates, np.float32, copy=True)
    f = pop[..., 0]
    fi = _f2i_sat(f)
    coef = f == np.float32(1.0)
    top = lib.n_funcs - 1
    over = (~coef) & (fi > top)
    f[over] = np.float32(top)
    fi = np.where(over, top, fi)
    var_row = (~coef) & (fi >= lib.var_start) & (fi <= top) & (lib.fn_codes[np.clip(fi, 0, top)] == nat.FN_VAR)
    past = var_row & (fi - lib.var_start > n_data - 1)
    f[past] = np.float32(lib.var_start + n_data - 1)
    counts = np.array([max(0, min(hi, len(r)) - lo) for r in rows], np.int32)
    K = max(1, int(counts.max()) if B else 1)
    theta = np.zeros((B, K), np.float32)
    for b, r in enumerate(rows):
        for k in range(counts[b]):
            t, i = r[lo + k]
            theta[b, k] = pop[b, t, i, 3]
            pop[b, t, i, 0] = np.float32(lib.var_start + n_data + k)
    n_funcs = max(lib.n_funcs, lib.var_start + n_data + K)
    if n_funcs > nat.MAX_FUNCS:
        raise ValueError(f"{n_funcs} node functions with {K} parameters > {nat.MAX_FUNCS}")
    fn = np.zeros(n_funcs, np.int8)
    fn[: lib.n_funcs] = lib.fn_codes
    fn[lib.var_start: n_funcs] = nat.FN_VAR
    return pop, theta, counts, K, nat.node_library_struct(n_funcs, lib.var_start, fn)


# ----------------------------------------------------------------------- the loop
class CoefficientOptimiser:
    """GeneticProgramming.optimise on the GPU for one evaluator config (a DeviceEngine with
    size_parsinomy 0: the loss is the evaluator's fitness, gp.py:447)."""

    def __init__(self, engine, jit: Optional[bool] = None):
        self.check_evaluator(engine.ff)
        self.engine = engine
        # the control evaluators' programs as dual-number machine code (mtgp_ctl_grad_jit, ABI v19):
        # on with the engine's program JIT unless disabled here or by MTGP_GRAD_JIT=0
        self.use_jit = (engine.use_jit and os.environ.get("MTGP_GRAD_JIT", "1") != "0") if jit is None else bool(jit)
        self.last_jit_info = None  # device int32 [2] of the last call: [0] < 0 untranslatable, [1] bytes used

    @staticmethod
    def check_evaluator(ff):
        kind = getattr(ff, "solver_kind", "")
        if kind not in ("rk4", "euler", "dopri5"):
            raise NotImplementedError(f"coefficient optimisation: solver {kind!r}")
        if ff.model_id != nat.MODEL_SR and getattr(ff, "state_size", 0) > 3:
            raise NotImplementedError("coefficient optimisation of the dynamic evaluator: state_size <= 3")

    @staticmethod
    def check_data(d: dict) -> None:
        """The data-dependent limits of the gradient kernels on a prepared data dict (the
        evaluator's `prepare`, host only), raised where the data is first seen
        (GeneticProgramming.evaluate_population at every generation with coefficient_optimisation,
        ADVICE r3), not at the first optimising generation (gp.py:418: generation 14): at most 64
        rollouts (one lane set per candidate).  (Since round 5 the general Acrobot cost mask -- ts off
        the one-pass grid, MtgpRollouts.fit_kof -- is differentiated too.)"""
        if d["R"] > 64:
            raise NotImplementedError("coefficient optimisation with more than 64 rollouts")

    def _grad_fn(self):
        eng = self.engine
        return eng.native.mtgp_sr_grad if eng.ff.model_id == nat.MODEL_SR else eng.native.mtgp_ctl_grad

    def param_cap(self, n_data: int) -> int:
        lib = self.engine.lib
        return max(1, min(nat.MAX_DATA - n_data, nat.MAX_FUNCS - lib.var_start - n_data))

    def loss_and_grad(self, candidates: np.ndarray, data, rows=None) -> Tuple[np.ndarray, List[np.ndarray]]:
        """loss [B] (the evaluator's fitness, no parsimony) and, per candidate, d loss / d value of
        each coefficient row in `rows` order."""
        eng = self.engine
        cands = np.ascontiguousarray(candidates, np.float32)
        B, T, N, _ = cands.shape
        rows = coefficient_rows(cands) if rows is None else rows
        d = eng.prepare_data(data)
        self.check_data(d)
        n_data = eng.ff.n_data()
        specs, _ = eng._specs()
        cap = self.param_cap(n_data)
        n_max = max([len(r) for r in rows] + [0])
        grads = [np.zeros(len(r), np.float32) for r in rows]
        loss = None
        dev = eng.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        m = eng.model_struct(d)
        ro = eng.rollouts_struct(d)
        R = d["R"]
        L = eng.program_stride(N)
        grad_fn = self._grad_fn()
        for lo in range(0, max(n_max, 1), cap):
            pop, theta, nparam, K, libs = parameterise(cands, rows, eng.lib, n_data, lo, lo + cap)
            spec_arr = (nat.MtgpProgramSpec * len(specs))()
            for i, sp in enumerate(specs):  # the reference's data vector + K parameter slots (no slot gap)
                spec_arr[i].tree, spec_arr[i].n_data, spec_arr[i].zero_mask = sp[0], sp[1] + K, sp[2]
            spec_dev = torch.frombuffer(bytearray(bytes(spec_arr)), dtype=torch.uint8).to(dev)
            n_prog = len(specs)
            pop_dev = torch.from_numpy(pop).to(dev)
            prog = torch.empty((B * n_prog * L * 2 + 8,), dtype=torch.int32, device=dev)
            plen = torch.empty((B, n_prog), dtype=torch.int32, device=dev)
            nodes = torch.empty((B,), dtype=torch.int32, device=dev)
            status = torch.empty((B, n_prog), dtype=torch.int32, device=dev)
            rc = eng.native.mtgp_flatten(pop_dev.data_ptr(), B, T, N, ctypes.byref(libs), spec_dev.data_ptr(), n_prog,
                                         L, prog.data_ptr(), plen.data_ptr(), nodes.data_ptr(), status.data_ptr(),
                                         stream)
            if rc != nat.OK:
                raise RuntimeError(f"mtgp_flatten (parameterised) failed: {rc}")
            worst = int(status.max().item()) if status.numel() else 0
            if worst != 0:
                raise ValueError(f"parameterised candidate does not flatten (status {worst})")
            th = torch.from_numpy(theta).to(dev)
            npd = torch.from_numpy(nparam).to(dev)
            # (the general Acrobot mask keeps every lane's cost prefixes behind the partials, mtgp.h)
            hist = d["n_save"] if d.get("fit_kof") is not None else 0
            scratch = torch.empty((B * K * R * 2 * (1 + hist),), dtype=torch.float32, device=dev)
            lo_d = torch.empty((B,), dtype=torch.float32, device=dev)
            gr_d = torch.empty((B, K), dtype=torch.float32, device=dev)
            called = grad_fn
            if self.use_jit and (eng.ff.model_id != nat.MODEL_SR or n_data <= 4):
                code, nbytes = eng.grad_code_buffer(nat.grad_jit_bytes(B, n_prog, L))
                offs = torch.empty((B * n_prog + 1,), dtype=torch.int32, device=dev)
                info = torch.empty((2,), dtype=torch.int32, device=dev)
                gj = nat.MtgpGradJit(code, nbytes, offs.data_ptr(), info.data_ptr())
                jit_fn = eng.native.mtgp_sr_grad_jit if eng.ff.model_id == nat.MODEL_SR else eng.native.mtgp_ctl_grad_jit
                called = jit_fn
                rc = jit_fn(ctypes.byref(m), prog.data_ptr(), n_prog, L, B, th.data_ptr(), npd.data_ptr(), K,
                            ctypes.byref(ro), scratch.data_ptr(), lo_d.data_ptr(), gr_d.data_ptr(), ctypes.byref(gj),
                            stream)
                self.last_jit_info = info
            else:
                rc = grad_fn(ctypes.byref(m), prog.data_ptr(), n_prog, L, B, th.data_ptr(), npd.data_ptr(), K,
                             ctypes.byref(ro), scratch.data_ptr(), lo_d.data_ptr(), gr_d.data_ptr(), stream)
            if rc != nat.OK:
                raise RuntimeError(f"{called.__name__} rejected the configuration (code {rc})")
            g = gr_d.cpu().numpy()
            if loss is None:
                loss = lo_d.cpu().numpy()
            for b in range(B):
                grads[b][lo: lo + nparam[b]] = g[b, : nparam[b]]
        return loss, grads

    def optimise(self, candidates: np.ndarray, data, n_epoch: int, optimiser=None):
        """gp.py:454-473 -> (fitness [B] = best loss over the epochs, candidates at that epoch)."""
        opt = optimiser if optimiser is not None else adam()
        cands = np.array(candidates, np.float32, copy=True)
        rows = coefficient_rows(cands)
        sizes = [len(r) for r in rows]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)

        def values(c):
            return np.concatenate([c[b][r[:, 0], r[:, 1], 3] for b, r in enumerate(rows)] + [np.zeros(0, np.float32)])

        vals = values(cands).astype(np.float32)
        # one optimiser state per candidate (gp.py:468 vmaps init, gp.py:448 vmaps update): an
        # optimiser with cross-element state (e.g. global-norm clipping) never couples candidates
        states = [opt.init(vals[offs[b]: offs[b + 1]]) for b in range(len(rows))]
        hist_c, hist_l = [], []
        for _ in range(int(n_epoch)):
            loss, grads = self.loss_and_grad(cands, data, rows)
            hist_c.append(cands.copy())
            hist_l.append(loss)
            for b, r in enumerate(rows):
                v = vals[offs[b]: offs[b + 1]]
                upd, states[b] = opt.update(np.asarray(grads[b], np.float32), states[b], v)
                vals[offs[b]: offs[b + 1]] = (v + np.asarray(upd, np.float32)).astype(np.float32)
                cands[b][r[:, 0], r[:, 1], 3] = vals[offs[b]: offs[b + 1]]
        L = np.stack(hist_l)
        best = np.argmin(L, axis=0)
        out = np.stack([hist_c[e][b] for b, e in enumerate(best)]) if len(best) else cands[:0]
        return L.min(axis=0), out
