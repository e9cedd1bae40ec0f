"""Observation-noise PRNG spec (include/mtgp_prng.h) and its host restatement (prng.py).

Pinning: jax is not installable here, so the spec is checked against
published outputs of the reference's own PRNG stack:
  * the Random123 Threefry-2x32-20 known-answer vectors (the same ones JAX's
    random_test.py uses for threefry_2x32);
  * jax.random.split(PRNGKey(0)) = [[4146024105, 967050713], [2718843009, 1272950319]]
    (JAX documentation, "JAX PRNG" / jax.random docs, original threefry layout);
  * jax.random.normal(PRNGKey(0), (10,)) and jax.random.normal(PRNGKey(0)) as printed in
    the JAX quickstart (float32 shortest repr -> these pin the 10 + 1 values bit for bit).
"""
import numpy as np
import pytest
from scipy.special import erfinv as sp_erfinv

from multitreegp_amd import prng
from oracle import oracle as orc

KAT = [  # (key, counter) -> output, Random123 kat_vectors threefry2x32_20
    ((0x00000000, 0x00000000), (0x00000000, 0x00000000), (0x6b200159, 0x99ba4efe)),
    ((0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff), (0x1cb996fc, 0xbb002be7)),
    ((0x13198a2e, 0x03707344), (0x243f6a88, 0x85a308d3), (0xc4923a9c, 0x483df7a0)),
]
JAX_SPLIT_KEY0 = [[4146024105, 967050713], [2718843009, 1272950319]]
JAX_NORMAL_KEY0_10 = "[-0.3721109   0.26423115 -0.18252768 -0.7368197  -0.44030377 -0.1521442\n" \
                     " -0.67135346 -0.5908641   0.73168886  0.5673026 ]"
JAX_NORMAL_KEY0 = "-0.20584226"


@pytest.fixture(autouse=True)
def _original_layout():
    prng.set_threefry_partitionable(False)
    yield
    prng.set_threefry_partitionable(False)


@pytest.mark.parametrize("key,ctr,want", KAT)
def test_threefry_kat_host_and_spec(key, ctr, want):
    y0, y1 = prng.threefry2x32(key, [ctr[0]], [ctr[1]])
    assert (int(y0[0]), int(y1[0])) == want
    c0, c1 = orc.threefry(np.array(key, np.uint32), np.array([ctr[0]], np.uint32), np.array([ctr[1]], np.uint32))
    assert (int(c0[0]), int(c1[0])) == want


def test_threefry_spec_matches_host_on_random_words():
    rng = np.random.default_rng(0)
    key = rng.integers(0, 2 ** 32, 2, dtype=np.uint32)
    x0 = rng.integers(0, 2 ** 32, 5000, dtype=np.uint32)
    x1 = rng.integers(0, 2 ** 32, 5000, dtype=np.uint32)
    a = prng.threefry2x32(key, x0, x1)
    b = orc.threefry(key, x0, x1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_prngkey_and_split_published_vector():
    assert prng.PRNGKey(0).tolist() == [0, 0]
    assert prng.PRNGKey(42).tolist() == [0, 42]
    assert prng.split(prng.PRNGKey(0)).tolist() == JAX_SPLIT_KEY0


def test_normal_published_vectors_bit_exact():
    got = orc.random_normals(prng.PRNGKey(0), 10, 0)
    assert np.array2string(got) == JAX_NORMAL_KEY0_10
    one = orc.random_normals(prng.PRNGKey(0), 1, 0)
    assert str(np.float32(one[0])) == JAX_NORMAL_KEY0


def test_random_bits_layouts():
    key = prng.split(prng.PRNGKey(3))[1]
    for n in (1, 3, 4, 7, 8):
        bits = prng.random_bits(key, (n,))
        c = np.concatenate([np.arange(n, dtype=np.uint32), np.zeros(n % 2, np.uint32)])
        h = c.size // 2
        y0, y1 = prng.threefry2x32(key, c[:h], c[h:])
        assert np.array_equal(bits, np.concatenate([y0, y1])[:n])
    prng.set_threefry_partitionable(True)
    bits = prng.random_bits(key, (5,))
    y0, y1 = prng.threefry2x32(key, np.zeros(5, np.uint32), np.arange(5, dtype=np.uint32))
    assert np.array_equal(bits, y0 ^ y1)
    # split in the partitionable layout is the fold-like (0, i) counter pair
    sp = prng.split(key, 3)
    y0, y1 = prng.threefry2x32(key, np.zeros(3, np.uint32), np.arange(3, dtype=np.uint32))
    assert np.array_equal(sp, np.stack([y0, y1], 1))


@pytest.mark.parametrize("impl", [0, 1])
def test_obs_normals_spec_vs_host_bits(impl):
    """fold_in(key, bitcast(t)) + random_bits + uniform + erfinv chain of the C spec vs the host
    restatement of the integer part and a float64 scipy erfinv of the same uniforms."""
    prng.set_threefry_partitionable(bool(impl))
    rng = np.random.default_rng(1)
    for _ in range(50):
        key = rng.integers(0, 2 ** 32, 2, dtype=np.uint32)
        t = np.float32(rng.uniform(0, 50))
        got = orc.obs_normals(key, t, 4, impl)
        k = prng.fold_in(key, int(t.view(np.uint32)))
        bits = prng.random_bits(k, (4,))
        f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1)
        lo = np.nextafter(np.float32(-1), np.float32(0))
        u = np.maximum(lo, (f * np.float32(2) + lo).astype(np.float32))
        want = np.sqrt(2.0) * sp_erfinv(u.astype(np.float64))
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7)


def test_uniform_host_matches_spec_construction():
    key = prng.PRNGKey(7)
    u = prng.uniform(key, (1000,), -0.1, 0.1)
    assert u.dtype == np.float32 and u.min() >= np.float32(-0.1) and u.max() < np.float32(0.1)
    bits = prng.random_bits(key, (1000,))
    f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1)
    assert np.array_equal(u, np.maximum(np.float32(-0.1), f * np.float32(0.2) + np.float32(-0.1)))


def test_erfinv_and_log1p_accuracy():
    x = np.linspace(-0.9999, 0.9999, 100001).astype(np.float32)
    e = orc.erfinv(x).astype(np.float64)
    r = sp_erfinv(x.astype(np.float64))
    # Giles' single-precision polynomial: ~1e-6 relative in the body, ~5e-6 in the far tails
    assert np.max(np.abs(e - r) / np.maximum(np.abs(r), 1e-30)) < 1e-5
    assert orc.erfinv(np.array([0.0], np.float32))[0] == 0.0
    a = -np.random.default_rng(0).random(100000).astype(np.float32)
    a = np.concatenate([a, np.float32([-1e-30, -1e-8, -0.5, -0.999999, 0.0, 1.0, 1e-3])])
    lp = orc.log1p(a).astype(np.float64)
    ref = np.log1p(a.astype(np.float64))
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(lp - ref) / ulp) <= 2.0
    edge = orc.log1p(np.float32([-1.0, np.nan, np.inf, -2.0]))
    assert edge[0] == -np.inf and np.isnan(edge[1]) and edge[2] == np.inf and np.isnan(edge[3])


def test_normal_distribution_moments():
    key = prng.PRNGKey(11)
    vals = np.concatenate([orc.random_normals(k, 64, 0) for k in prng.split(key, 400)])
    assert abs(vals.mean()) < 0.03 and abs(vals.std() - 1) < 0.03
    assert np.all(np.isfinite(vals))


def test_jax_control_data_layout():
    import multitreegp_amd as mt
    env = mt.Acrobot(0.0, 0.1)
    x0, ts, tg, pk, ok, params = mt.environments.jax_control_data(prng.split(prng.PRNGKey(1))[1], env, 16, 0.2, 50.0)
    assert x0.shape == (16, 4) and x0.dtype == np.float32 and np.all(np.abs(x0) <= 0.1)
    assert ts.shape == (250,) and ts.dtype == np.float32 and ts[1] == np.float32(0.2)
    assert pk.shape == ok.shape == (16, 2) and ok.dtype == np.uint32
    assert len({tuple(k) for k in ok}) == 16 and tg.shape == (16, 0)
