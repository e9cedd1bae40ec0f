/*
 * mtgp_prng.h -- the observation-noise stream of the MultiTreeGP control environments,
 * restated from JAX's PRNG so that it can run inside the HIP kernel.
 *
 * Reference call (control_environment_base.py:43-48, acrobot.py:29-32):
 *     new_key = jrandom.fold_in(key, bitcast_f32_to_i32(t))
 *     out     = C @ x + jrandom.normal(new_key, shape=(n_obs,)) @ W
 * evaluated inside every RHS call of the solve (dynamic_evaluate.py:111,
 * feedforward_evaluate.py:106) and at every save point (dynamic_evaluate.py:99).
 * jax/jaxlib are not installed here; the algorithm below is JAX's published one
 * (jax/_src/prng.py threefry2x32, threefry_seed, threefry_fold_in, the two
 * random_bits layouts; jax/_src/random.py uniform/_normal_real; XLA's ErfInv32):
 *
 *   threefry2x32     Threefry-2x32 with 20 rounds, rotations (13,15,26,6 | 17,29,16,24),
 *                    key schedule (k0, k1, k0^k1^0x1BD11BDA) injected every 4 rounds;
 *                    pinned by the Random123 known-answer vectors (tests/test_prng.py).
 *   fold_in(k, d)    threefry2x32(k, (0, d)) -- threefry_seed(d) = [d >> 32 (= 0), d].
 *   random_bits(k,n) "original" layout (jax_threefry_partitionable = False, the default of
 *                    every JAX release up to 0.4.x, i.e. when the reference was written):
 *                    counts iota(n) (+ one 0 if n is odd) split in halves x0 | x1, output
 *                    concat(y0, y1)[:n];  "partitionable" layout (the default from JAX
 *                    0.5.0): word i = y0 ^ y1 of threefry2x32(k, (0, i)).
 *   uniform          bits >> 9 | 0x3f800000 -> [1, 2) - 1, then * (hi - lo) + lo and
 *                    max(lo, .), lo = nextafter(-1, 0), hi = 1 (so hi - lo = 2.0f).
 *   normal           f32(sqrt 2) * erfinv(u); erfinv = Giles' single-precision
 *                    polynomial in w = -log1p(-u*u) (XLA ErfInv32 coefficients),
 *                    +-inf at |u| = 1.
 * log1p is fixed here by an fdlibm-style float algorithm (basic IEEE operations only),
 * like the sin/cos of mtgp_f32math.h, so the GPU kernel and the CPU oracle agree bit for
 * bit.  XLA's own log1p differs in the last bits: parity vs JAX is unpinned for normal().
 * Must be compiled with -ffp-contract=off (explicit fmaf only).
 */
#ifndef MTGP_PRNG_H
#define MTGP_PRNG_H

#include <stdint.h>
#include "mtgp_f32math.h"

enum { MTGP_PRNG_THREEFRY_ORIGINAL = 0, MTGP_PRNG_THREEFRY_PARTITIONABLE = 1 };

#if defined(__HIP_DEVICE_COMPILE__)
#define MTGP_ROTL32(v, r) __builtin_rotateleft32((v), (r))
#else
#define MTGP_ROTL32(v, r) (((v) << (r)) | ((v) >> (32 - (r))))
#endif

#define MTGP_TF_ROUND(r)            \
  do {                              \
    x0 = x0 + x1;                   \
    x1 = MTGP_ROTL32(x1, r);        \
    x1 = x0 ^ x1;                   \
  } while (0)

/* Threefry-2x32, 20 rounds (jax/_src/prng.py _threefry2x32_lowering / Random123). */
MTGP_INLINE MTGP_HD void mtgp_threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t* y0,
                                           uint32_t* y1) {
  const uint32_t k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  uint32_t x0 = c0 + k0, x1 = c1 + k1;
  MTGP_TF_ROUND(13); MTGP_TF_ROUND(15); MTGP_TF_ROUND(26); MTGP_TF_ROUND(6);
  x0 = x0 + k1; x1 = x1 + k2 + 1u;
  MTGP_TF_ROUND(17); MTGP_TF_ROUND(29); MTGP_TF_ROUND(16); MTGP_TF_ROUND(24);
  x0 = x0 + k2; x1 = x1 + k0 + 2u;
  MTGP_TF_ROUND(13); MTGP_TF_ROUND(15); MTGP_TF_ROUND(26); MTGP_TF_ROUND(6);
  x0 = x0 + k0; x1 = x1 + k1 + 3u;
  MTGP_TF_ROUND(17); MTGP_TF_ROUND(29); MTGP_TF_ROUND(16); MTGP_TF_ROUND(24);
  x0 = x0 + k1; x1 = x1 + k2 + 4u;
  MTGP_TF_ROUND(13); MTGP_TF_ROUND(15); MTGP_TF_ROUND(26); MTGP_TF_ROUND(6);
  x0 = x0 + k2; x1 = x1 + k0 + 5u;
  *y0 = x0;
  *y1 = x1;
}

/* jax.random.fold_in(key, data) for a 32-bit data word: threefry2x32(key, (0, data)). */
MTGP_INLINE MTGP_HD void mtgp_fold_in(uint32_t k0, uint32_t k1, uint32_t data, uint32_t* n0, uint32_t* n1) {
  mtgp_threefry2x32(k0, k1, 0u, data, n0, n1);
}

/* Counter pair and output half of word i of random_bits(key, 32, (n,)).
 *   original:       block j = i mod half (half = ceil(n/2)), counters (j, j + half) with
 *                   the padding counter (value n when n is odd) replaced by 0; word i is
 *                   y0 for i < half, y1 otherwise.
 *   partitionable:  counters (0, i), word = y0 ^ y1. */
MTGP_INLINE MTGP_HD uint32_t mtgp_random_bits_word(uint32_t k0, uint32_t k1, int i, int n, int impl) {
  uint32_t y0, y1;
  if (impl == MTGP_PRNG_THREEFRY_PARTITIONABLE) {
    mtgp_threefry2x32(k0, k1, 0u, (uint32_t)i, &y0, &y1);
    return y0 ^ y1;
  }
  const int half = (n + 1) >> 1;
  const int j = i < half ? i : i - half;
  const uint32_t c1 = (j + half < n) ? (uint32_t)(j + half) : 0u;
  mtgp_threefry2x32(k0, k1, (uint32_t)j, c1, &y0, &y1);
  return i < half ? y0 : y1;
}

/* ---- log1p on mtgp_logf_pos (include/mtgp_f32math.h) ---- */
/* log1p(a) for a >= -1 (jnp.log1p semantics at the edges: -1 -> -inf, nan -> nan). */
MTGP_INLINE MTGP_HD float mtgp_log1pf(float a) {
  if (mtgp_isnan(a)) return a;
  if (a == -1.0f) return -__builtin_huge_valf();
  if (a < -1.0f) return mtgp_qnan();
  if (!mtgp_isfinite(a)) return a; /* +inf */
  const float u = 1.0f + a;
  if (u == 1.0f) return a; /* |a| below half an ulp of 1 */
  /* log1p(a) = log(u) * a / (u - 1): cancels the rounding error of u (Goldberg/Kahan) */
  return mtgp_logf_pos(u) * (a / (u - 1.0f));
}

/* erfinv for |x| <= 1 (XLA ErfInv32 / Giles 2010 single precision). */
MTGP_INLINE MTGP_HD float mtgp_erfinvf(float x) {
  float w = -mtgp_log1pf(-(x * x));
  float p;
  if (w < 5.0f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = 3.43273939e-07f + p * w;
    p = -3.5233877e-06f + p * w;
    p = -4.39150654e-06f + p * w;
    p = 0.00021858087f + p * w;
    p = -0.00125372503f + p * w;
    p = -0.00417768164f + p * w;
    p = 0.246640727f + p * w;
    p = 1.50140941f + p * w;
  } else {
    w = __builtin_sqrtf(w) - 3.0f;
    p = -0.000200214257f;
    p = 0.000100950558f + p * w;
    p = 0.00134934322f + p * w;
    p = -0.00367342844f + p * w;
    p = 0.00573950773f + p * w;
    p = -0.0076224613f + p * w;
    p = 0.00943887047f + p * w;
    p = 1.00167406f + p * w;
    p = 2.83297682f + p * w;
  }
  const float r = p * x;
  return (MTGP_FABSF(x) == 1.0f) ? x * 3.40282347e+38f : r;
}

/* jax.random.uniform(minval = nextafter(-1, 0), maxval = 1) from 32 random bits. */
MTGP_INLINE MTGP_HD float mtgp_uniform_pm1(uint32_t bits) {
  const float lo = -0.99999994039535522461f; /* nextafter(-1, 0) */
  const float f = mtgp_u2f((bits >> 9) | 0x3f800000u) - 1.0f;
  const float v = f * 2.0f + lo; /* (maxval - minval) = 1 - lo rounds to 2.0f */
  return v < lo ? lo : v;
}

/* one standard-normal sample from 32 random bits (jax.random._normal_real) */
MTGP_INLINE MTGP_HD float mtgp_normal_from_bits(uint32_t bits) {
  return 1.41421354f * mtgp_erfinvf(mtgp_uniform_pm1(bits));
}

/* random_bits(key, 32, (n,)) -> out[0..n-1], each threefry block computed once */
MTGP_INLINE MTGP_HD void mtgp_random_bits(uint32_t k0, uint32_t k1, int n, int impl, uint32_t* out) {
  uint32_t y0, y1;
  if (impl == MTGP_PRNG_THREEFRY_PARTITIONABLE) {
    for (int i = 0; i < n; ++i) {
      mtgp_threefry2x32(k0, k1, 0u, (uint32_t)i, &y0, &y1);
      out[i] = y0 ^ y1;
    }
    return;
  }
  const int half = (n + 1) >> 1;
  for (int j = 0; j < half; ++j) {
    const uint32_t c1 = (j + half < n) ? (uint32_t)(j + half) : 0u;
    mtgp_threefry2x32(k0, k1, (uint32_t)j, c1, &y0, &y1);
    out[j] = y0;
    if (j + half < n) out[j + half] = y1;
  }
}

/* jax.random.normal(fold_in(key, bitcast(t)), (n,)) -> out[0..n-1], n <= 8 */
MTGP_INLINE MTGP_HD void mtgp_obs_normals(uint32_t k0, uint32_t k1, float t, int n, int impl, float* out) {
  uint32_t n0, n1, bits[8];
  mtgp_fold_in(k0, k1, mtgp_f2u(t), &n0, &n1);
  mtgp_random_bits(n0, n1, n, impl, bits);
  for (int i = 0; i < n; ++i) out[i] = mtgp_normal_from_bits(bits[i]);
}

#endif /* MTGP_PRNG_H */
