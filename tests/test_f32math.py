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


# ---- the round-3 unary tree operators (include/mtgp_f32math.h, MTGP_FN_EXP .. MTGP_FN_ABS) ----
FN_EXP, FN_LOG, FN_SQRT, FN_TANH, FN_ABS = 8, 9, 10, 11, 12


def test_log_within_1ulp_and_edges():
    rng = np.random.default_rng(5)
    x = np.concatenate([np.exp(rng.uniform(-87, 88, 600)), rng.uniform(0.5, 2.0, 300),
                        np.array([1e-40, 1e-45, 3.4e38], np.float64)]).astype(np.float32)
    x = x[x > 0]
    assert _ulp_err(x, orc.unary(FN_LOG, x), mpmath.log) <= 1.0
    e = np.array([0.0, -0.0, -1.0, np.inf, -np.inf, np.nan, 1.0], np.float32)
    y = orc.unary(FN_LOG, e)
    assert y[0] == -np.inf and y[1] == -np.inf and np.isnan(y[2]) and y[3] == np.inf and np.isnan(y[4])
    assert np.isnan(y[5]) and y[6] == 0.0


def test_sqrt_and_abs_are_ieee():
    rng = np.random.default_rng(6)
    x = np.concatenate([np.exp(rng.uniform(-100, 88, 4000)), np.array([0.0, -0.0, np.inf, 1e-45])]).astype(np.float32)
    assert np.array_equal(orc.unary(FN_SQRT, x).view(np.uint32), np.sqrt(x).view(np.uint32))  # correctly rounded
    assert np.isnan(orc.unary(FN_SQRT, np.array([-1.0, -np.inf, np.nan], np.float32))).all()
    z = (rng.standard_normal(2000) * 10).astype(np.float32)
    z[:3] = [-0.0, np.inf, -np.inf]
    assert np.array_equal(orc.unary(FN_ABS, z).view(np.uint32), np.abs(z).view(np.uint32))


@pytest.mark.parametrize("lo,hi", [(-0.7, 0.7), (-12, 12), (-60, 60)])
def test_tanh_within_3ulp(lo, hi):
    rng = np.random.default_rng(int(hi))
    x = rng.uniform(lo, hi, 600).astype(np.float32)
    assert _ulp_err(x, orc.unary(FN_TANH, x), mpmath.tanh) <= 3.0
    e = orc.unary(FN_TANH, np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30], np.float32))
    assert e.view(np.uint32)[1] == 0x80000000 and e[0] == 0.0 and e[2] == 1.0 and e[3] == -1.0
    assert np.isnan(e[4]) and e[5] == np.float32(1e-30)


def test_exp_through_the_operator_code():
    x = np.random.default_rng(7).uniform(-80, 80, 2000).astype(np.float32)
    assert np.array_equal(orc.unary(FN_EXP, x).view(np.uint32), orc.expf(x).view(np.uint32))
    assert _ulp_err(x[:400], orc.unary(FN_EXP, x[:400]), mpmath.exp) <= 1.0


def test_unary_tangents_match_finite_differences():
    """include/mtgp_dual.h's JVP rules (the coefficient optimiser's forward mode): d/dx f vs a
    float64 central difference of the float64 function."""
    x = np.array([0.3, 1.7, 2.5, 0.05, 4.0], np.float32)
    fns = {FN_EXP: np.exp, FN_LOG: np.log, FN_SQRT: np.sqrt, FN_TANH: np.tanh, FN_ABS: np.abs}
    for fn, f in fns.items():
        y, dy = orc.unary(fn, x, np.ones_like(x))
        xd = x.astype(np.float64)
        fd = (f(xd + 1e-6) - f(xd - 1e-6)) / 2e-6
        assert np.allclose(dy, fd, rtol=1e-5, atol=1e-6), (fn, dy, fd)
    _, d = orc.unary(FN_ABS, np.array([-2.0, 0.0], np.float32), np.array([1.0, 1.0], np.float32))
    assert d[0] == -1.0 and d[1] == 0.0  # jnp.sign(0) = 0
