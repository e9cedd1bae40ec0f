/*
 * mtgp_f32math.h -- the fp32 arithmetic specification of the MultiTreeGP hot path.
 *
 * The reference evaluates everything in float32 under XLA (SURVEY.md §2.1 "Arithmetic").
 * Its transcendental functions (jnp.sin / jnp.cos in the tree lambdas, gp.py:24-31 +
 * DynamicPolicy.ipynb operator_list; acrobot.py:56-63,78) and the floor-mod angle wrap
 * (acrobot.py:31, jnp.remainder) are XLA's own implementations, which cannot run here.
 *
 * This header fixes ONE deterministic fp32 implementation of those primitives, written
 * only with IEEE-754 basic operations (+ - * / fma, rint, trunc, int64<->double) so that
 * the HIP kernel (gfx950) and the host C oracle produce bit-identical results.  That is
 * what lets the parity tests compare GPU and CPU trajectories exactly even though the
 * Acrobot is chaotic (SURVEY.md §7 "Hard parts" 1).
 *
 *   mtgp_sinf / mtgp_cosf : |error| <= ~2 ulp over the whole float range; reduction onto
 *       the pi grid (sin: x - 2k pi/2, cos: x - (2k+1) pi/2) and one odd polynomial (spec v2)
 *       |x| < 2^-12        : sin x = x, cos x = 1
 *       |x| < 2^17         : 3-constant float Cody-Waite reduction with fma (exact first step)
 *       |x| < 2^28         : 3-constant double Cody-Waite reduction
 *       otherwise (finite) : Payne-Hanek reduction against a 96-bit window of 2/pi
 *   mtgp_floor_mod_2pi    : jnp.remainder(a, float32(2*pi)) semantics, exact fmod core
 *
 * Must be compiled with -ffp-contract=off on both sides (explicit fmaf only).
 * Pure C99 + optional HIP host/device qualifiers; no libm transcendental is called.
 */
#ifndef MTGP_F32MATH_H
#define MTGP_F32MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define MTGP_HD __host__ __device__
#define MTGP_NOINLINE __attribute__((noinline))
#define MTGP_FMAF(a, b, c) __builtin_fmaf((a), (b), (c))
#define MTGP_RINTF(a) __builtin_rintf(a)
#define MTGP_RINT(a) __builtin_rint(a)
#define MTGP_TRUNCF(a) __builtin_truncf(a)
#define MTGP_FABSF(a) __builtin_fabsf(a)
#define MTGP_SQRTF(a) __builtin_sqrtf(a) /* correctly rounded (HIP's default f32 sqrt) */
#else
#include <math.h>
#define MTGP_HD
#define MTGP_NOINLINE
#define MTGP_FMAF(a, b, c) fmaf((a), (b), (c))
#define MTGP_RINTF(a) rintf(a)
#define MTGP_RINT(a) rint(a)
#define MTGP_TRUNCF(a) truncf(a)
#define MTGP_FABSF(a) fabsf(a)
#define MTGP_SQRTF(a) sqrtf(a)
#endif

/* wave-uniform "does any lane need the rare path" test: a single scalar branch on the GPU,
 * the per-element condition on the host (same result per element either way) */
#if defined(__HIP_DEVICE_COMPILE__)
#define MTGP_ANY(c) (__builtin_amdgcn_ballot_w64(c) != 0)
#else
#define MTGP_ANY(c) (c)
#endif

#ifdef __cplusplus
#define MTGP_INLINE static inline
#else
#define MTGP_INLINE static inline
#endif

/* float32 images of the Python constants the reference uses (weak-typed -> f32). */
#define MTGP_PI_F        3.14159274101257324e+00f /* f32(jnp.pi)      acrobot.py:31,59,61 */
#define MTGP_TWO_PI_F    6.28318548202514648e+00f /* f32(2*jnp.pi)    acrobot.py:31       */
#define MTGP_HALF_PI_F   1.57079637050628662e+00f /* f32(jnp.pi/2)    acrobot.py:59,61    */
#define MTGP_8PI_F       2.51327419281005859e+01f /* f32(8*jnp.pi)    acrobot.py:87       */
#define MTGP_18PI_F      5.65486679077148438e+01f /* f32(18*jnp.pi)   acrobot.py:87       */

MTGP_INLINE MTGP_HD uint32_t mtgp_f2u(float f) {
  union { float f; uint32_t u; } c; c.f = f; return c.u;
}
MTGP_INLINE MTGP_HD float mtgp_u2f(uint32_t u) {
  union { float f; uint32_t u; } c; c.u = u; return c.f;
}
MTGP_INLINE MTGP_HD int mtgp_isfinite(float x) { return (mtgp_f2u(x) & 0x7f800000u) != 0x7f800000u; }
MTGP_INLINE MTGP_HD int mtgp_isnan(float x) { return (mtgp_f2u(x) & 0x7fffffffu) > 0x7f800000u; }
MTGP_INLINE MTGP_HD float mtgp_qnan(void) { return mtgp_u2f(0x7fc00000u); }

/* ---- sin / cos on the pi grid (spec v2) ------------------------------------------------
 * Both functions reduce to r = x - j*pi/2 with j of a fixed parity -- j = 2k (sin) or
 * j = 2k+1 (cos), k = rint(x/pi) or rint(x/pi - 1/2) -- so |r| <= pi/2 (+ rounding slack) and
 * ONE odd polynomial serves both:
 *     sin x = (-1)^k sin r,      cos x = (-1)^(k+1) sin r,
 * i.e. the result is sin_poly(r) with the sign bit flipped by bit 0 of (k + [cos]).  The
 * polynomial is r + r^3 (c3 + c5 s + c7 s^2 + c9 s^3), s = r^2, a relative-error fit on
 * |r| <= 1.0021 pi/2 with f32 coefficients (approximation error 6.3e-9, ~0.1 ulp; fit script
 * scripts/fit_sin_poly.py).  One polynomial per lane instead of two plus quadrant selects;
 * zeros of both functions are at r = 0, so relative accuracy near them is kept. */
#define MTGP_SIN_C3 -1.66666597127914428711e-01f
#define MTGP_SIN_C5 8.33306834101676940918e-03f
#define MTGP_SIN_C7 -1.98096662643365561962e-04f
#define MTGP_SIN_C9 2.60578394772892352194e-06f
#define MTGP_INV_PI_F 3.18309873342514038086e-01f /* f32(1/pi) */
#define MTGP_TRIG_FAST_MAX 131072.0f              /* 2^17: float Cody-Waite range */

MTGP_INLINE MTGP_HD float mtgp_sin_poly(float r) {
  const float s = r * r;
  float p = MTGP_SIN_C9;
  p = MTGP_FMAF(p, s, MTGP_SIN_C7);
  p = MTGP_FMAF(p, s, MTGP_SIN_C5);
  p = MTGP_FMAF(p, s, MTGP_SIN_C3);
  return MTGP_FMAF(r * s, p, r);
}

/* 2/pi, 384 bits, most significant word first (checked against mpmath in tests). */
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint32_t mtgp_two_over_pi_bits[12] = {
    0xa2f9836eu, 0x4e441529u, 0xfc2757d1u, 0xf534ddc0u, 0xdb629599u, 0x3c439041u,
    0xfe5163abu, 0xdebbc561u, 0xb7246e3au, 0x424dd2e0u, 0x06492eeau, 0x09d1921cu};

#if defined(__HIPCC__)
/* host copy (the __constant__ table above is device-side under HIP) */
static const uint32_t mtgp_two_over_pi_bits_host[12] = {
    0xa2f9836eu, 0x4e441529u, 0xfc2757d1u, 0xf534ddc0u, 0xdb629599u, 0x3c439041u,
    0xfe5163abu, 0xdebbc561u, 0xb7246e3au, 0x424dd2e0u, 0x06492eeau, 0x09d1921cu};
#endif

MTGP_INLINE MTGP_HD uint32_t mtgp_twoopi_word(int k) {
#if defined(__HIPCC__) && !defined(__HIP_DEVICE_COMPILE__)
  return mtgp_two_over_pi_bits_host[k];
#else
  return mtgp_two_over_pi_bits[k];
#endif
}

/* Payne-Hanek for finite |x| >= 2^28 (|x| = m * 2^e, 24-bit m, e >= 5): the 96-bit window W
 * of 2/pi bits [b+1, b+96], b = e - 2, makes m*W*2^-94 = |x|*2/pi mod 4 with the binary point
 * at a FIXED bit (94) of the product, so no limb is indexed dynamically.  v = |x|*2/pi mod 4
 * = vi + f (vi = 0..3, f in [0, 1) as 64 fraction bits); the nearest j of parity `odd` is vi
 * when vi has it (r = f pi/2), else vi + 1 (r = (f - 1) pi/2).  Returns r, *j = j mod 4. */
MTGP_INLINE MTGP_HD float mtgp_reduce_payne_hanek_pi(float ax, int odd, int* j) {
  const uint32_t u = mtgp_f2u(ax);
  const uint32_t m = (u & 0x7fffffu) | 0x800000u;
  const int e = (int)((u >> 23) & 0xffu) - 150;
  const int b = e - 2;
  const int k = b >> 5, s = b & 31;
  const uint64_t w0 = mtgp_twoopi_word(k), w1 = mtgp_twoopi_word(k + 1), w2 = mtgp_twoopi_word(k + 2),
                 w3 = mtgp_twoopi_word(k + 3);
  const uint64_t Whi = (uint32_t)(((w0 << 32) | w1) >> (32 - s));
  const uint64_t Wmid = (uint32_t)(((w1 << 32) | w2) >> (32 - s));
  const uint64_t Wlo = (uint32_t)(((w2 << 32) | w3) >> (32 - s));
  const uint64_t lo = (uint64_t)m * Wlo;
  const uint64_t mid = (uint64_t)m * Wmid + (lo >> 32);
  const uint64_t hi = (uint64_t)m * Whi + (mid >> 32);
  const int vi = (int)((hi >> 30) & 3u);
  const uint64_t frac = ((hi & 0x3fffffffull) << 34) | ((mid & 0xffffffffull) << 2) | ((lo & 0xffffffffull) >> 30);
  double f = (double)frac * 5.42101086242752217e-20; /* 2^-64 */
  int jj = vi;
  if ((vi & 1) != odd) { jj = vi + 1; f = f - 1.0; }
  *j = jj & 3;
  return (float)(f * 1.57079632679489656e+00);
}

/* slow reduction for finite |x| >= 2^17 onto the pi grid of parity `odd` (0 sin, 1 cos):
 * r, and j mod 4 in *j */
MTGP_INLINE MTGP_HD float mtgp_reduce_pi_slow(float x, int odd, int* j) {
  const float ax = MTGP_FABSF(x);
  if (ax < 268435456.0f) { /* 2^28: double Cody-Waite, 24+24+53-bit pi/2, first steps exact */
    const double xd = (double)x;
    const double k = MTGP_RINT(xd * 3.1830988618379069e-01 - (odd ? 0.5 : 0.0)); /* 1/pi */
    const double jd = 2.0 * k + (odd ? 1.0 : 0.0);
    double r = xd - jd * 1.570796251296997e+00;
    r = r - jd * 7.549789415861596e-08;
    r = r - jd * 5.390302858158119e-15;
    *j = ((int)(int64_t)jd) & 3;
    return (float)r;
  }
  int jj;
  float r = mtgp_reduce_payne_hanek_pi(ax, odd, &jj);
  if (x < 0.0f) { r = -r; jj = (4 - jj) & 3; }
  *j = jj;
  return r;
}

/* sin (odd = 0) or cos (odd = 1) on the pi grid, fast path: exact spec result for |x| < 2^17
 * (f32 Cody-Waite with the 3-constant pi/2 split, exact first step) and for non-finite x (NaN);
 * *slow = 1 for the lanes (finite |x| >= 2^17) that need mtgp_trig_pi_slow instead.  Callers
 * evaluating several arguments test all their slow flags with ONE wave-uniform branch.
 * |x| < 2^-12: sin x = x (keeps -0 and denormals), cos x = 1. */
MTGP_INLINE MTGP_HD float mtgp_trig_pi_fast(float x, int odd, int* slow) {
  const float ax = MTGP_FABSF(x);
  const float t = x * MTGP_INV_PI_F;
  const float k = MTGP_RINTF(odd ? t - 0.5f : t);
  const float j = odd ? MTGP_FMAF(k, 2.0f, 1.0f) : k + k;
  float r = MTGP_FMAF(j, -1.57079637e+00f, x);
  r = MTGP_FMAF(j, 4.37113883e-08f, r);
  r = MTGP_FMAF(j, 1.71512451e-15f, r);
  const int fast = ax < MTGP_TRIG_FAST_MAX;
#if defined(__HIP_DEVICE_COMPILE__)
  const int ki = (int)k; /* v_cvt_i32_f32 saturates (NaN -> 0): defined for every lane */
#else
  const int ki = fast ? (int)k : 0;
#endif
  *slow = !fast && mtgp_isfinite(x);
  /* sign: bit 0 of k + odd (= bit 1 of j + odd) */
  const float v = mtgp_u2f(mtgp_f2u(mtgp_sin_poly(r)) ^ ((uint32_t)(ki + odd) << 31));
  return (ax < 2.44140625e-04f) ? (odd ? 1.0f : x) : v; /* 2^-12 */
}

/* the slow lanes: finite |x| >= 2^17 (double Cody-Waite below 2^28, Payne-Hanek above) */
MTGP_INLINE MTGP_HD float mtgp_trig_pi_slow(float x, int odd) {
  int ji;
  const float r = mtgp_reduce_pi_slow(x, odd, &ji);
  return mtgp_u2f(mtgp_f2u(mtgp_sin_poly(r)) ^ ((uint32_t)(ji + odd) << 30 & 0x80000000u));
}

MTGP_INLINE MTGP_HD float mtgp_trig_pi(float x, int odd) {
  int slow;
  float v = mtgp_trig_pi_fast(x, odd, &slow);
  if (MTGP_ANY(slow)) {
    if (slow) v = mtgp_trig_pi_slow(x, odd);
  }
  return v;
}

MTGP_INLINE MTGP_HD float mtgp_sinf(float x) { return mtgp_trig_pi(x, 0); }
MTGP_INLINE MTGP_HD float mtgp_cosf(float x) { return mtgp_trig_pi(x, 1); }

/* sin and cos of one x (bit-identical to mtgp_sinf / mtgp_cosf) */
MTGP_INLINE MTGP_HD void mtgp_sincosf(float x, float* s, float* c) {
  *s = mtgp_trig_pi(x, 0);
  *c = mtgp_trig_pi(x, 1);
}

/* large |a|: exact binary long division by power-of-two multiples of b (rare path) */
MTGP_INLINE MTGP_HD float mtgp_fmod_2pi_large(float a) {
  const float b = MTGP_TWO_PI_F;
  float r = MTGP_FABSF(a);
  while (r >= b) {
    float t = b;
    while (t <= r * 0.5f) t = t * 2.0f; /* exact scaling */
    r = r - t;                          /* exact: r in [t, 2t) */
  }
  return (a < 0.0f) ? -r : r;
}

/* Exact C fmod(a, b) for b = f32(2*pi) > 0 (truncated remainder, sign of a).
 * Fast path (|a| < 2^20): q = trunc(|a| * up(1/b)) is never below the true quotient (the
 * reciprocal is rounded UP) and at most one above it, so r = fma(-q, b, |a|) lies in (-b, b)
 * with the lsb of b -> exact; one "+ b" (also exact) fixes the overshoot.  Lanes with
 * |a| >= 2^20 or non-finite a take the slow path behind one wave-uniform branch. */
MTGP_INLINE MTGP_HD float mtgp_fmod_2pi(float a) {
  const float b = MTGP_TWO_PI_F;
  const float aa = MTGP_FABSF(a);
  const float q = MTGP_TRUNCF(aa * 1.59154951572418213e-01f); /* up(1/f32(2pi)) */
  float r = MTGP_FMAF(-q, b, aa);
  r = (r < 0.0f) ? r + b : r;
  const int slow = !(aa < 1048576.0f);
  if (MTGP_ANY(slow)) {
    if (slow) r = mtgp_isfinite(a) ? mtgp_fmod_2pi_large(aa) : mtgp_qnan();
  }
  return mtgp_u2f(mtgp_f2u(r) | (mtgp_f2u(a) & 0x80000000u));
}

/* jnp.remainder(a, 2pi) (floor-mod): trunc remainder, then + b when signs differ. */
MTGP_INLINE MTGP_HD float mtgp_floor_mod_2pi(float a) {
  const float r = mtgp_fmod_2pi(a);
  return (r < 0.0f) ? r + MTGP_TWO_PI_F : r;
}

/* Acrobot angle wrap (acrobot.py:31): (v + pi) % (2 pi) - pi, all in f32. */
MTGP_INLINE MTGP_HD float mtgp_wrap_angle(float v) {
  return mtgp_floor_mod_2pi(v + MTGP_PI_F) - MTGP_PI_F;
}

/* jnp.clip(u, -1, 1) = minimum(maximum(u, -1), 1), NaN-propagating (acrobot.py:53). */
MTGP_INLINE MTGP_HD float mtgp_clip1(float u) {
  if (mtgp_isnan(u)) return u;
  return u < -1.0f ? -1.0f : (u > 1.0f ? 1.0f : u);
}

/* jnp.clip(u, lo, hi) = minimum(maximum(u, lo), hi), NaN-propagating (reactor.py:63). */
MTGP_INLINE MTGP_HD float mtgp_clip(float u, float lo, float hi) {
  if (mtgp_isnan(u)) return u;
  return u < lo ? lo : (u > hi ? hi : u);
}

/* exp(x) (StirredTankReactor.k, reactor.py:40: k0 * exp(-Ea/R/T)).  n = rint(x / ln2),
 * r = x - n ln2 by a two-constant fma Cody-Waite step, exp(r) by the degree-6 Cephes expf
 * polynomial, then y * 2^n as two exact power-of-two scalings (one rounding, gradual
 * underflow).  NaN -> NaN, x > 88.7228394 -> +inf, x < -103.972084 -> +0.  Max error
 * ~1 ulp vs float64 exp (tests/test_f32math.py). */
MTGP_INLINE MTGP_HD float mtgp_expf(float x) {
  if (mtgp_isnan(x)) return x;
  if (x > 88.7228394f) return mtgp_u2f(0x7f800000u);
  if (x < -103.972084f) return 0.0f;
  const float n = MTGP_RINTF(x * 1.44269502162933350e+00f);
  float r = MTGP_FMAF(-n, 6.93147182464599609e-01f, x);
  r = MTGP_FMAF(-n, -1.90465429995776804e-09f, r);
  float p = 1.9875691500e-4f;
  p = MTGP_FMAF(p, r, 1.3981999507e-3f);
  p = MTGP_FMAF(p, r, 8.3334519073e-3f);
  p = MTGP_FMAF(p, r, 4.1665795894e-2f);
  p = MTGP_FMAF(p, r, 1.6666665459e-1f);
  p = MTGP_FMAF(p, r, 5.0000001201e-1f);
  float y = MTGP_FMAF(p, r * r, r) + 1.0f;
  const int ni = (int)n, n1 = ni / 2, n2 = ni - n1; /* |n1|, |n2| <= 75: normal powers of two */
  y = y * mtgp_u2f((uint32_t)(n1 + 127) << 23);
  return y * mtgp_u2f((uint32_t)(n2 + 127) << 23);
}

/* ---- log, fdlibm-style (FreeBSD e_logf.c polynomial), basic operations only ---- */
/* log(u) for finite u > 0 (u == 1 -> 0). */
MTGP_INLINE MTGP_HD float mtgp_logf_pos(float u) {
  uint32_t ix = mtgp_f2u(u);
  int k = 0;
  if (ix < 0x00800000u) { /* subnormal: scale by 2^25 (exact) */
    u = u * 33554432.0f;
    ix = mtgp_f2u(u);
    k = -25;
  }
  k += (int)(ix >> 23) - 127;
  ix &= 0x007fffffu;
  /* normalise m into [sqrt(2)/2, sqrt(2)): i = 0x800000 when the mantissa is >= ~sqrt(2)
   * (0x800000 - 0x4afb20 = 0x3504e0, sqrt(2) = 0x3fb504f3), then m is halved */
  const uint32_t i = (ix + 0x4afb20u) & 0x800000u;
  const float m = mtgp_u2f(ix | (i ^ 0x3f800000u)); /* m or m/2 */
  k += (int)(i >> 23);
  const float f = m - 1.0f;
  const float s = f / (2.0f + f);
  const float z = s * s;
  const float w = z * z;
  const float t1 = w * (0.40000972152f + w * 0.24279078841f);
  const float t2 = z * (0.66666662693f + w * 0.28498786688f);
  const float R = t2 + t1;
  const float hfsq = 0.5f * f * f;
  const float dk = (float)k;
  /* ln2 split: hi has 16 trailing zero bits so dk * hi is exact */
  return dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
}


/* ---- further unary operators a reference operator_list may name (round 3) ----
 * Each is one fixed f32 algorithm of basic IEEE operations (plus mtgp_expf / mtgp_logf_pos), so
 * the kernels and the oracle agree bit for bit; the accuracy vs float64 is tested in
 * tests/test_f32math.py (XLA's own exp / log / tanh may differ in the last bits: unpinnable here). */

/* jnp.log: NaN -> NaN, x < 0 -> NaN, +-0 -> -inf, +inf -> +inf, else mtgp_logf_pos */
MTGP_INLINE MTGP_HD float mtgp_logf(float x) {
  if (mtgp_isnan(x)) return x;
  if (x < 0.0f) return mtgp_qnan();
  if (x == 0.0f) return -__builtin_huge_valf();
  if (!mtgp_isfinite(x)) return x;
  return mtgp_logf_pos(x);
}

/* jnp.sqrt: the correctly rounded IEEE square root (x < 0 -> NaN, -0 -> -0) */
MTGP_INLINE MTGP_HD float mtgp_sqrtf(float x) { return MTGP_SQRTF(x); }

/* jnp.abs: the sign bit cleared */
MTGP_INLINE MTGP_HD float mtgp_absf(float x) { return mtgp_u2f(mtgp_f2u(x) & 0x7fffffffu); }

/* jnp.tanh (Cephes tanhf): |x| < 0.625: x + x^3 P(x^2) (degree-4 P, fma chain); otherwise
 * sign(x) * (1 - 2 / (exp(2|x|) + 1)) (exp overflow -> +-1).  NaN -> NaN, -0 -> -0. */
MTGP_INLINE MTGP_HD float mtgp_tanhf(float x) {
  if (mtgp_isnan(x)) return x;
  const float a = MTGP_FABSF(x);
  if (a >= 0.625f) {
    const float e = mtgp_expf(a + a);
    const float t = 1.0f - 2.0f / (e + 1.0f);
    return x < 0.0f ? -t : t;
  }
  if (a == 0.0f) return x; /* +-0 */
  const float z = x * x;
  float p = -5.70498872745e-3f;
  p = MTGP_FMAF(p, z, 2.06390887954e-2f);
  p = MTGP_FMAF(p, z, -5.37397155531e-2f);
  p = MTGP_FMAF(p, z, 1.33314422036e-1f);
  p = MTGP_FMAF(p, z, -3.33332819422e-1f);
  return MTGP_FMAF(p * z, x, x);
}

#endif /* MTGP_F32MATH_H */
