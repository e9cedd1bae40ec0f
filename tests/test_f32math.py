"""The shared fp32 arithmetic spec (include/mtgp_f32math.h), exercised through the oracle."""
import mpmath
import numpy as np
import pytest

from oracle import oracle as orc

mpmath.mp.prec = 300


def _ulp_err(x, got, fn):
    ref = np.array([float(fn(mpmath.mpf(float(v)))) for v in x])
    sp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return float(np.max(np.abs(got.astype(np.float64) - ref) / sp))


@pytest.mark.parametrize("lo,hi", [(-4, 4), (-1e5, 1e5), (1e5, 3e8), (3e8, 3e38)])
def test_sin_cos_within_2ulp(lo, hi):
    rng = np.random.default_rng(abs(int(lo)) % 997)
    if lo < 0:
        x = rng.uniform(lo, hi, 1500)
    else:
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 1500)) * np.where(rng.random(1500) < 0.5, -1, 1)
    x = x.astype(np.float32)
    s, c = orc.sincos(x)
    assert _ulp_err(x, s, mpmath.sin) <= 2.0
    assert _ulp_err(x, c, mpmath.cos) <= 2.0


def test_sin_cos_near_multiples_of_half_pi():
    x = (np.arange(1, 4000) * np.float64(np.pi / 2) * np.array([1, 997])[:, None]).astype(np.float32).ravel()
    s, c = orc.sincos(x)
    assert _ulp_err(x, s, mpmath.sin) <= 2.0
    assert _ulp_err(x, c, mpmath.cos) <= 2.0


def test_sin_cos_special_values():
    x = np.array([0.0, -0.0, 1e-40, -1e-40, 1e-5, np.inf, -np.inf, np.nan], np.float32)
    s, c = orc.sincos(x)
    assert s[0] == 0 and not np.signbit(s[0]) and s[1] == 0 and np.signbit(s[1])
    assert s[2] == x[2] and s[3] == x[3] and s[4] == x[4]
    assert np.all(c[:5] == 1.0)
    assert np.all(np.isnan(s[5:])) and np.all(np.isnan(c[5:]))


def test_two_over_pi_table():
    mpmath.mp.prec = 600
    words = []
    v = 2 / mpmath.pi
    for _ in range(12):
        v *= 2 ** 32
        w = int(mpmath.floor(v))
        words.append(w)
        v -= w
    text = open(orc.HERE + "/../include/mtgp_f32math.h").read()
    for w in words:
        assert f"0x{w:08x}u" in text


def _jax_remainder(x, b):
    """jnp.remainder: C fmod, then + b where the truncated remainder is non-zero with the
    wrong sign (jax/_src/numpy/ufuncs.py remainder)."""
    fm = np.fmod(x, b)
    return np.where((fm != 0) & ((fm < 0) != (b < 0)), (fm + b).astype(np.float32), fm).astype(np.float32)


@pytest.mark.parametrize("lo,hi", [(-20, 20), (-1e7, 1e7), (-3e38, 3e38)])
def test_wrap_angle_bit_exact(lo, hi):
    rng = np.random.default_rng(3)
    b = np.float32(2 * np.pi)
    pi = np.float32(np.pi)
    y = rng.uniform(lo, hi, 100000).astype(np.float32)
    y = np.concatenate([y, b * np.arange(-60, 60, dtype=np.float32) - pi,
                        np.array([0, -0.0, np.inf, -np.inf, np.nan, pi, -pi], np.float32)])
    got = orc.wrap(y)
    with np.errstate(invalid="ignore"):
        ref = (_jax_remainder((y + pi).astype(np.float32), b) - pi).astype(np.float32)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), (y[~same][:5], got[~same][:5], ref[~same][:5])
