"""Environments on the hot path (host-side description + synthetic data generators).

Only the pieces the evaluator needs are restated: dimensions, per-rollout parameters and
initial states.  The dynamics themselves run inside the HIP kernel (Acrobot.drift,
acrobot.py:51-72) -- the numpy drifts below exist only to generate ground-truth data for
symbolic regression (SymbolicRegression.ipynb get_data) and are not on the hot path.
Random draws use numpy PCG64 instead of jax.random (not installable here).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from . import prng


class Acrobot:
    """acrobot.py:7-87.  n_var 4, n_control 1, n_targets 0, n_obs 4 (default)."""

    def __init__(self, process_noise: float, obs_noise: float, n_obs: int = 4):
        self.n_var = 4
        self.n_control = 1
        self.n_targets = 0
        self.n_dim = 1
        self.n_obs = n_obs
        self.process_noise = process_noise
        self.obs_noise = obs_noise
        self.init_bounds = np.array([0.1, 0.1, 0.1, 0.1], dtype=np.float32)
        self.R = np.array([[0.01]], dtype=np.float32)

    def sample_init_states(self, batch_size: int, rng) -> Tuple[np.ndarray, np.ndarray]:
        """acrobot.py:18-22: x0 ~ U(-0.1, 0.1)^4, targets [batch, 0]."""
        rng = np.random.default_rng(rng)
        x0 = rng.uniform(-self.init_bounds, self.init_bounds, size=(batch_size, self.n_var)).astype(np.float32)
        targets = np.zeros((batch_size, self.n_targets), dtype=np.float32)
        return x0, targets

    def sample_params(self, batch_size: int, mode, ts, rng) -> Tuple[np.ndarray, ...]:
        """acrobot.py:24-27: l1 = l2 = m1 = m2 = 1."""
        one = np.ones(batch_size, dtype=np.float32)
        return one, one.copy(), one.copy(), one.copy()

    def obs_matrix(self) -> np.ndarray:
        """W = obs_noise * eye(n_obs) (acrobot.py:49), float32."""
        return (np.float32(self.obs_noise) * np.eye(self.n_obs, dtype=np.float32)).astype(np.float32)


class HarmonicOscillator:
    """harmonic_oscillator.py:8-80.  n_var 2, n_control 1, n_targets 1, n_obs 2 (default).

    The kernel functor (mtgp_kernels.hip EnvHarmonic) restates drift A x + b u,
    A = [[0, 1], [-omega, -zeta]], the quadratic cost with q = r = 0.5 and cond_fn_nan."""

    def __init__(self, process_noise: float, obs_noise: float, n_obs: int = 2):
        self.n_dim = 1
        self.n_var = 2
        self.n_control = 1
        self.n_targets = 1
        self.n_obs = n_obs
        self.process_noise = process_noise
        self.obs_noise = obs_noise
        self.mu0 = np.zeros(self.n_var, np.float32)
        self.P0 = (np.eye(self.n_var) * np.array([3.0, 1.0])).astype(np.float32)
        self.q = self.r = 0.5

    def sample_init_states(self, batch_size: int, rng) -> Tuple[np.ndarray, np.ndarray]:
        """harmonic_oscillator.py:23-27: x0 = mu0 + N(0, 1) @ P0, targets ~ U(-3, 3)."""
        rng = np.random.default_rng(rng)
        x0 = (self.mu0 + rng.standard_normal((batch_size, self.n_var)).astype(np.float32) @ self.P0).astype(np.float32)
        targets = rng.uniform(-3, 3, size=(batch_size, self.n_targets)).astype(np.float32)
        return x0, targets

    def sample_params(self, batch_size: int, mode, ts, rng) -> Tuple[np.ndarray, np.ndarray]:
        """harmonic_oscillator.py:29-31 ("Constant": omega 1, zeta 0) and :32-34 ("Different":
        omega ~ U(0, 2), zeta ~ U(0, 1.5)).  The time-varying modes give [R, S] arrays that the
        reference's own A = [[0, 1], [-omega, -zeta]] cannot take; they are not supported."""
        if mode == "Constant":
            return np.ones(batch_size, np.float32), np.zeros(batch_size, np.float32)
        if mode == "Different":
            rng = np.random.default_rng(rng)
            return (rng.uniform(0.0, 2.0, batch_size).astype(np.float32),
                    rng.uniform(0.0, 1.5, batch_size).astype(np.float32))
        raise NotImplementedError(f"mode {mode!r}")

    def obs_matrix(self) -> np.ndarray:
        """W = obs_noise * eye(n_obs) (harmonic_oscillator.py:66)."""
        return (np.float32(self.obs_noise) * np.eye(self.n_obs, dtype=np.float32)).astype(np.float32)


class StirredTankReactor:
    """reactor.py:7-81.  State (Tc, T, c), n_control 1 (coolant flow, clipped to [0, 300]),
    n_targets 1 (reactor temperature), n_obs 3 (default).  Kernel functor: EnvReactor."""

    def __init__(self, process_noise: float, obs_noise: float, n_obs: int = 3, n_targets: int = 1):
        self.process_noise = process_noise
        self.obs_noise = obs_noise
        self.n_var = 3
        self.n_control = 1
        self.n_dim = 1
        self.n_targets = n_targets
        self.n_obs = n_obs
        self.init_lower_bounds = np.array([275, 350, 0.5], np.float32)
        self.init_upper_bounds = np.array([300, 375, 1.0], np.float32)

    def sample_init_states(self, batch_size: int, rng) -> Tuple[np.ndarray, np.ndarray]:
        """reactor.py:71-75: x0 ~ U(lower, upper), targets ~ U(400, 500)."""
        rng = np.random.default_rng(rng)
        x0 = rng.uniform(self.init_lower_bounds, self.init_upper_bounds,
                         size=(batch_size, self.n_var)).astype(np.float32)
        targets = rng.uniform(400, 500, size=(batch_size, self.n_targets)).astype(np.float32)
        return x0, targets

    def sample_params(self, batch_size: int, mode, ts, rng):
        """reactor.py:46-69 -> (Vol, Cp, dHr, UA, q, Tf, Tcf, Volc), each [batch]."""
        if mode == "Constant":
            vals = (100.0, 239.0, -5.0e4, 5.0e4, 100.0, 300.0, 300.0, 20.0)
            return tuple(np.full(batch_size, v, np.float32) for v in vals)
        if mode == "Different":
            rng = np.random.default_rng(rng)
            bounds = ((75, 150), (200, 350), (-55000, -45000), (25000, 75000), (75, 125), (300, 350), (250, 300),
                      (10, 30))
            return tuple(rng.uniform(lo, hi, batch_size).astype(np.float32) for lo, hi in bounds)
        raise NotImplementedError(f"mode {mode!r}")

    def obs_matrix(self) -> np.ndarray:
        """W = obs_noise * eye(n_obs) * [15, 15, 0.1][:n_obs] (reactor.py:43), float32 ops."""
        w = np.float32(self.obs_noise) * np.eye(self.n_obs, dtype=np.float32)
        return (w * np.array([15, 15, 0.1], np.float32)[: self.n_obs]).astype(np.float32)


class VanDerPolOscillator:
    """SR_environments/vd_pol_oscillator.py:6-29 (mu = 1)."""

    def __init__(self, process_noise: float = 0.0, obs_noise: float = 0.0, n_obs: int = 2):
        self.n_var = 2
        self.n_obs = n_obs
        self.mu = 1.0
        self.process_noise = process_noise
        self.obs_noise = obs_noise

    def sample_init_states(self, batch_size: int, rng) -> np.ndarray:
        rng = np.random.default_rng(rng)
        return rng.standard_normal((batch_size, 2)).astype(np.float32)

    def drift(self, t, state):
        """vd_pol_oscillator.py:22-23 (float64 numpy, ground truth only)."""
        return np.stack([state[..., 1], self.mu * (1 - state[..., 0] ** 2) * state[..., 1] - state[..., 0]], -1)


class LinearSystem:
    """Stable random linear system dx/dt = A x used as the C5 target (BASELINE C5)."""

    def __init__(self, n_var: int, seed: int = 7):
        rng = np.random.default_rng(seed)
        q, _ = np.linalg.qr(rng.standard_normal((n_var, n_var)))
        eig = -rng.uniform(0.1, 1.0, n_var)
        self.A = (q * eig) @ q.T
        self.n_var = n_var
        self.n_obs = n_var

    def sample_init_states(self, batch_size: int, rng) -> np.ndarray:
        rng = np.random.default_rng(rng)
        return rng.standard_normal((batch_size, self.n_var)).astype(np.float32)

    def drift(self, t, state):
        return state @ self.A.T


def ground_truth(env, x0: np.ndarray, ts: np.ndarray, h: float = 1e-3) -> np.ndarray:
    """Fine float64 RK4 solution of env.drift saved at ts -> [R, S, n_var] float32.

    Replaces the notebook's diffrax Dopri5 (atol = rtol = 1e-7) ground-truth generation
    (SymbolicRegression.ipynb get_data)."""
    x = x0.astype(np.float64)
    ts = np.asarray(ts, dtype=np.float64)
    out = np.empty((x0.shape[0], len(ts), x0.shape[1]), dtype=np.float64)
    out[:, 0] = x
    t = ts[0]
    for k in range(1, len(ts)):
        n = max(1, int(round((ts[k] - t) / h)))
        dt = (ts[k] - t) / n
        for _ in range(n):
            k1 = env.drift(t, x)
            k2 = env.drift(t, x + 0.5 * dt * k1)
            k3 = env.drift(t, x + 0.5 * dt * k2)
            k4 = env.drift(t, x + dt * k3)
            x = x + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
            t = t + dt
        out[:, k] = x
    return out.astype(np.float32)


def control_data(env, batch_size: int, dt: float, T: float, seed: int = 1, n_steps: int = None,
                 mode: str = "Constant"):
    """The notebooks' get_data (DynamicPolicy.ipynb cell 2) with numpy RNG:
    (x0, ts, targets, process_noise_keys, obs_noise_keys, params).  The noise keys are
    distinct JAX-format keys (split of PRNGKey(seed)); see jax_control_data for the
    notebook's exact key derivation."""
    rng = np.random.default_rng(seed)
    x0, targets = env.sample_init_states(batch_size, rng)
    if n_steps is None:
        ts = np.arange(0, T, dt, dtype=np.float32)
    else:
        ts = (np.arange(n_steps + 1, dtype=np.float32) * np.float32(dt)).astype(np.float32)
    _, k1, k2 = prng.split(prng.PRNGKey(seed), 3)
    params = env.sample_params(batch_size, mode, ts, rng)
    return x0, ts, targets, prng.split(k1, batch_size), prng.split(k2, batch_size), params


def jax_control_data(key, env, batch_size: int, dt: float, T: float = None, n_steps: int = None):
    """DynamicPolicy.ipynb get_data restated with the JAX-compatible host PRNG:
        init_key, noise_key1, noise_key2, param_key = jr.split(key, 4)
        x0 ~ uniform(split(init_key)[0], (batch, 4), -init_bounds, init_bounds)  (acrobot.py:18-22)
        process/obs noise keys = jr.split(noise_key1/2, batch_size)
        ts = jnp.arange(0, T, dt)
    For Acrobot this reproduces the notebook's arrays bit for bit (threefry restated in prng.py)."""
    key = np.asarray(key, np.uint32)
    init_key, nk1, nk2, _param_key = prng.split(key, 4)
    ik, _tk = prng.split(init_key)
    b = np.asarray(env.init_bounds, np.float32)
    x0 = prng.uniform(ik, (batch_size, env.n_var), -b, b)
    targets = np.zeros((batch_size, env.n_targets), np.float32)
    if n_steps is None:
        ts = np.arange(0, T, dt, dtype=np.float32)
    else:
        ts = (np.arange(n_steps + 1, dtype=np.float32) * np.float32(dt)).astype(np.float32)
    params = env.sample_params(batch_size, "Constant", ts, None)
    return x0, ts, targets, prng.split(nk1, batch_size), prng.split(nk2, batch_size), params


def jax_sr_data(key, env, batch_size: int, T: float, dt: float = 0.2, ground_truth_h: float = 1e-3):
    """SymbolicRegression.ipynb get_data restated with the JAX-compatible host PRNG:
        x_key, noise_key = jr.split(key)
        x0s = env.sample_init_states(batch_size, x_key)   (VanDerPol: 0 + 1 * normal(x_key, (batch, 2)))
        noise_keys = jr.split(noise_key, batch_size)
        ts = jnp.arange(0, T, 0.2)
        xs = vmap(diffeqsolve(Dopri5, PIDController(1e-7, 1e-7, dtmin=0.001), dt0=0.001))(x0s)
    The ground-truth trajectories come from a fine float64 RK4 (`ground_truth`) instead of
    the notebook's float32 Dopri5 at tolerance 1e-7: both approximate the exact solution far
    below the MSE scale the SR fitness resolves.  -> (x0s, ts, xs, noise_keys)."""
    key = np.asarray(key, np.uint32)
    x_key, noise_key = prng.split(key)
    x0 = prng.normal(x_key, (batch_size, env.n_var))
    ts = np.arange(0, T, dt, dtype=np.float32)
    xs = ground_truth(env, x0, ts, h=ground_truth_h)
    return x0, ts, xs, prng.split(noise_key, batch_size)
