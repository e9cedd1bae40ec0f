"""JAX-compatible threefry PRNG keys on the host (numpy uint32).

The reference builds its rollout data with ``jax.random`` (DynamicPolicy.ipynb ``get_data``:
``jr.split`` for the per-rollout observation-noise keys, ``jr.uniform`` for the initial
states, acrobot.py:18-22) and feeds the keys to the observation noise inside the solve
(control_environment_base.py:43-48).  jax is not installed on this machine, so this module
restates the published threefry scheme (jax/_src/prng.py) in numpy: ``PRNGKey``, ``split``,
``fold_in``, ``random_bits`` and ``uniform`` produce the same uint32 words / float32 values
as JAX for the same key, which lets the notebook's data tuples be rebuilt without JAX.
The device kernel draws the noise itself from the keys (include/mtgp_prng.h).

Two random-bits layouts exist in JAX: the "original" one (``jax_threefry_partitionable``
False: the default of every JAX release up to 0.4.x, i.e. when the reference was written) and
the "partitionable" one (default from JAX 0.5.0).  ``set_threefry_partitionable`` selects
it for both the host helpers and the kernel (mirrors ``jax.config.update``).
"""
from __future__ import annotations

import numpy as np

_PARTITIONABLE = False

ROT0 = (13, 15, 26, 6)
ROT1 = (17, 29, 16, 24)


def set_threefry_partitionable(enabled: bool) -> None:
    """Counterpart of ``jax.config.update("jax_threefry_partitionable", enabled)``."""
    global _PARTITIONABLE
    _PARTITIONABLE = bool(enabled)


def threefry_partitionable() -> bool:
    return _PARTITIONABLE


def prng_impl_code() -> int:
    """MtgpModel.prng_impl value (mtgp_prng.h): 0 original, 1 partitionable."""
    return 1 if _PARTITIONABLE else 0


def _rotl(v, r):
    return (v << np.uint32(r)) | (v >> np.uint32(32 - r))


def threefry2x32(key, x0, x1):
    """Threefry-2x32 (20 rounds) of counter arrays x0, x1 under key (k0, k1) -> (y0, y1)."""
    with np.errstate(over="ignore"):
        k0, k1 = np.uint32(key[0]), np.uint32(key[1])
        ks = (k0, k1, k0 ^ k1 ^ np.uint32(0x1BD11BDA))
        x0 = np.asarray(x0, np.uint32) + ks[0]
        x1 = np.asarray(x1, np.uint32) + ks[1]
        for i in range(5):
            for r in (ROT0 if i % 2 == 0 else ROT1):
                x0 = x0 + x1
                x1 = _rotl(x1, r)
                x1 = x0 ^ x1
            x0 = x0 + ks[(i + 1) % 3]
            x1 = x1 + ks[(i + 2) % 3] + np.uint32(i + 1)
    return x0, x1


def _threefry_counts(key, counts):
    """jax threefry_2x32(keypair, count): split the flat counts in halves (padding an odd
    count with one 0) and concatenate the two output words."""
    c = np.asarray(counts, np.uint32).ravel()
    odd = c.size % 2
    if odd:
        c = np.concatenate([c, np.zeros(1, np.uint32)])
    h = c.size // 2
    y0, y1 = threefry2x32(key, c[:h], c[h:])
    out = np.concatenate([y0, y1])
    return out[:-1] if odd else out


def PRNGKey(seed: int) -> np.ndarray:
    """jax.random.PRNGKey(seed) (threefry_seed): [seed >> 32, seed & 0xffffffff]."""
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([s >> 32, s & 0xFFFFFFFF], np.uint32)


def split(key, num: int = 2) -> np.ndarray:
    """jax.random.split(key, num) -> uint32 [num, 2]."""
    key = np.asarray(key, np.uint32)
    if _PARTITIONABLE:
        y0, y1 = threefry2x32(key, np.zeros(num, np.uint32), np.arange(num, dtype=np.uint32))
        return np.stack([y0, y1], axis=1)
    return _threefry_counts(key, np.arange(2 * num, dtype=np.uint32)).reshape(num, 2)


def fold_in(key, data: int) -> np.ndarray:
    """jax.random.fold_in(key, data) for a 32-bit data word."""
    y0, y1 = threefry2x32(np.asarray(key, np.uint32), np.zeros(1, np.uint32),
                          np.array([int(data) & 0xFFFFFFFF], np.uint32))
    return np.array([y0[0], y1[0]], np.uint32)


def random_bits(key, shape) -> np.ndarray:
    """jax.random.bits(key, shape, uint32) / the 32-bit _random_bits."""
    shape = (shape,) if np.isscalar(shape) else tuple(shape)
    n = int(np.prod(shape)) if shape else 1
    key = np.asarray(key, np.uint32)
    if _PARTITIONABLE:
        y0, y1 = threefry2x32(key, np.zeros(n, np.uint32), np.arange(n, dtype=np.uint32))
        return (y0 ^ y1).reshape(shape)
    return _threefry_counts(key, np.arange(n, dtype=np.uint32)).reshape(shape)


def uniform(key, shape=(), minval=0.0, maxval=1.0) -> np.ndarray:
    """jax.random.uniform in float32: mantissa bits -> [1, 2) - 1, scaled, max(minval, .)."""
    shape = (shape,) if np.isscalar(shape) else tuple(shape)
    bits = random_bits(key, shape)
    lo = np.broadcast_to(np.asarray(minval, np.float32), shape)
    hi = np.broadcast_to(np.asarray(maxval, np.float32), shape)
    f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)
    v = (f * (hi - lo) + lo).astype(np.float32)
    return np.maximum(lo, v).astype(np.float32)


# XLA ErfInv32 (Giles 2010, single precision) coefficients, as include/mtgp_prng.h
_ERFINV_SMALL = (2.81022636e-08, 3.43273939e-07, -3.5233877e-06, -4.39150654e-06, 0.00021858087, -0.00125372503,
                 -0.00417768164, 0.246640727, 1.50140941)
_ERFINV_LARGE = (-0.000200214257, 0.000100950558, 0.00134934322, -0.00367342844, 0.00573950773, -0.0076224613,
                 0.00943887047, 1.00167406, 2.83297682)


def _erfinv(x: np.ndarray) -> np.ndarray:
    """float32 erfinv by Giles' polynomial in w = -log1p(-x^2) (host log1p: the C library's)."""
    x = np.asarray(x, np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        w = -np.log1p(-(x * x)).astype(np.float32)
        ws = (w - np.float32(2.5)).astype(np.float32)
        wl = (np.sqrt(w) - np.float32(3.0)).astype(np.float32)
        ps = np.full_like(x, np.float32(_ERFINV_SMALL[0]))
        pl = np.full_like(x, np.float32(_ERFINV_LARGE[0]))
        for cs, cl in zip(_ERFINV_SMALL[1:], _ERFINV_LARGE[1:]):
            ps = (np.float32(cs) + ps * ws).astype(np.float32)
            pl = (np.float32(cl) + pl * wl).astype(np.float32)
        r = (np.where(w < np.float32(5.0), ps, pl) * x).astype(np.float32)
    return np.where(np.abs(x) == np.float32(1.0), x * np.float32(np.inf), r).astype(np.float32)


def normal(key, shape=()) -> np.ndarray:
    """jax.random.normal in float32 (jax/_src/random.py _normal_real):
    u = uniform(key, shape, minval=nextafter(-1, 0), maxval=1); sqrt(2) * erf_inv(u).
    The device's own draws (observation noise) use include/mtgp_prng.h; this host helper
    builds initial states (SymbolicRegression.ipynb get_data: VanDerPol x0 ~ N(0, 1))."""
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    u = uniform(key, shape, lo, np.float32(1.0))
    return (np.float32(np.sqrt(2.0)) * _erfinv(u)).astype(np.float32)
