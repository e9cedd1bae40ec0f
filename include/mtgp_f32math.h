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
 *   mtgp_sinf / mtgp_cosf : |error| <= ~2 ulp over the whole float range
 *       |x| < 2^-12        : sin x = x, cos x = 1
 *       |x| < 2^17         : 3-constant Cody-Waite reduction with fma (exact first step)
 *       otherwise (finite) : Payne-Hanek reduction against 128 bits of 2/pi
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
#define MTGP_TRUNCF(a) __builtin_truncf(a)
#define MTGP_FABSF(a) __builtin_fabsf(a)
#else
#include <math.h>
#define MTGP_HD
#define MTGP_NOINLINE
#define MTGP_FMAF(a, b, c) fmaf((a), (b), (c))
#define MTGP_RINTF(a) rintf(a)
#define MTGP_TRUNCF(a) truncf(a)
#define MTGP_FABSF(a) fabsf(a)
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

/* ---- polynomial kernels on |r| <= pi/4 (+ slack), Taylor, evaluated with fma ---- */
MTGP_INLINE MTGP_HD float mtgp_sin_poly(float r) {
  const float r2 = r * r;
  float p = 2.75573192e-06f;               /*  1/9!  */
  p = MTGP_FMAF(p, r2, -1.98412698e-04f);  /* -1/7!  */
  p = MTGP_FMAF(p, r2, 8.33333377e-03f);   /*  1/5!  */
  p = MTGP_FMAF(p, r2, -1.66666672e-01f);  /* -1/3!  */
  return MTGP_FMAF(r * r2, p, r);
}
MTGP_INLINE MTGP_HD float mtgp_cos_poly(float r) {
  const float r2 = r * r;
  float p = -2.75573188e-07f;              /* -1/10! */
  p = MTGP_FMAF(p, r2, 2.48015876e-05f);   /*  1/8!  */
  p = MTGP_FMAF(p, r2, -1.38888892e-03f);  /* -1/6!  */
  p = MTGP_FMAF(p, r2, 4.16666679e-02f);   /*  1/4!  */
  p = MTGP_FMAF(p, r2, -5.0e-01f);         /* -1/2!  */
  return MTGP_FMAF(r2, p, 1.0f);
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

/* Payne-Hanek: for finite |x| >= 2^17 returns r in [-pi/4, pi/4] and quadrant q (0..3)
 * with |x| = q*pi/2 + r (mod 2*pi).  Fixed-point product of the 24-bit significand
 * with 128 bits of 2/pi taken at the exponent's window; the fraction is rounded to
 * double then float (all IEEE, so host and device agree). */
MTGP_NOINLINE MTGP_HD static float mtgp_reduce_large(float ax, int* quadrant) {
  const uint32_t u = mtgp_f2u(ax);
  const int bexp = (int)((u >> 23) & 0xffu);
  const uint32_t m = (u & 0x7fffffu) | 0x800000u;
  const int e = bexp - 127 - 23; /* ax = m * 2^e, e >= -6 here */
  const int k0 = (e >= 2) ? ((e - 2) >> 5) : 0;
  uint32_t q[5];
  uint64_t carry = 0;
  for (int i = 3; i >= 0; --i) {
    const uint64_t t = (uint64_t)m * (uint64_t)mtgp_twoopi_word(k0 + i) + carry;
    q[i + 1] = (uint32_t)t;
    carry = t >> 32;
  }
  q[0] = (uint32_t)carry;
  /* Q = q[0..4] (160 bits, q[4] least significant); value = Q * 2^-(sh) with: */
  const int sh = 32 * (k0 + 4) - e; /* number of fractional bits, in [95, 134] */
  /* bit b of Q (b = 0 is the lsb) lives in q[4 - (b >> 5)] at (b & 31) */
#define MTGP_QBIT64(b)                                                              \
  ((((b) >> 5) <= 4) ? (uint64_t)q[4 - ((b) >> 5)] : (uint64_t)0)
  /* 64 fraction bits: Q bits [sh-64, sh) ; quadrant: Q bits [sh, sh+2) */
  const int lo = sh - 64;
  const int wlo = lo >> 5, blo = lo & 31;
  uint64_t w0 = MTGP_QBIT64(32 * wlo), w1 = MTGP_QBIT64(32 * (wlo + 1)),
           w2 = MTGP_QBIT64(32 * (wlo + 2));
  uint64_t frac;
  if (blo == 0) frac = w0 | (w1 << 32);
  else frac = (w0 >> blo) | (w1 << (32 - blo)) | (w2 << (64 - blo));
  const int wq = sh >> 5, bq = sh & 31;
  uint64_t qa = MTGP_QBIT64(32 * wq), qb = MTGP_QBIT64(32 * (wq + 1));
  uint32_t quad = (uint32_t)(((qa >> bq) | (qb << (32 - bq))) & 3u);
  if (bq == 0) quad = (uint32_t)(qa & 3u);
#undef MTGP_QBIT64
  /* round the fraction to the nearest quadrant boundary: f in [-1/2, 1/2) */
  int64_t sf = (int64_t)frac;
  if (frac & 0x8000000000000000ull) quad = (quad + 1u) & 3u; /* sf already f - 1 */
  const double fd = (double)sf * 5.42101086242752217e-20; /* 2^-64 */
  const double rd = fd * 1.57079632679489656e+00;         /* pi/2 (double) */
  *quadrant = (int)quad;
  return (float)rd;
}

/* shared reduction: returns r, quadrant in *q.  Handles finite x only. */
MTGP_INLINE MTGP_HD float mtgp_reduce(float x, int* q) {
  const float ax = MTGP_FABSF(x);
  if (ax < 131072.0f) { /* 2^17 */
    const float j = MTGP_RINTF(x * 6.36619747e-01f); /* f32(2/pi) */
    float r = MTGP_FMAF(j, -1.57079637e+00f, x);     /* exact */
    r = MTGP_FMAF(j, 4.37113883e-08f, r);
    r = MTGP_FMAF(j, 1.71512451e-15f, r);
    *q = ((int)j) & 3;
    return r;
  }
  int qq;
  float r = mtgp_reduce_large(ax, &qq);
  if (x < 0.0f) { r = -r; qq = (4 - qq) & 3; }
  *q = qq;
  return r;
}

MTGP_INLINE MTGP_HD float mtgp_sinf(float x) {
  if (MTGP_FABSF(x) < 2.44140625e-04f) return x; /* 2^-12, keeps -0 and denormals */
  if (!mtgp_isfinite(x)) return mtgp_qnan();
  int q;
  const float r = mtgp_reduce(x, &q);
  const float s = (q & 1) ? mtgp_cos_poly(r) : mtgp_sin_poly(r);
  return (q & 2) ? -s : s;
}

MTGP_INLINE MTGP_HD float mtgp_cosf(float x) {
  if (MTGP_FABSF(x) < 2.44140625e-04f) return 1.0f;
  if (!mtgp_isfinite(x)) return mtgp_qnan();
  int q;
  const float r = mtgp_reduce(x, &q);
  const float c = (q & 1) ? mtgp_sin_poly(r) : mtgp_cos_poly(r);
  return ((q + 1) & 2) ? -c : c;
}

/* large |a|: exact binary long division by power-of-two multiples of b (rare path) */
MTGP_NOINLINE MTGP_HD static float mtgp_fmod_2pi_large(float a) {
  const float b = MTGP_TWO_PI_F;
  float r = MTGP_FABSF(a);
  while (r >= b) {
    float t = b;
    while (t <= r * 0.5f) t = t * 2.0f; /* exact scaling */
    r = r - t;                          /* exact: r in [t, 2t) */
  }
  return (a < 0.0f) ? -r : r;
}

/* Exact C fmod(a, b) for b = f32(2*pi) > 0 (truncated remainder, sign of a). */
MTGP_INLINE MTGP_HD float mtgp_fmod_2pi(float a) {
  const float b = MTGP_TWO_PI_F;
  if (!mtgp_isfinite(a)) return mtgp_qnan();
  const float aa = MTGP_FABSF(a);
  float r;
  if (aa < b) return a; /* fmod(a, b) = a, keeps the sign of zero */
  if (aa < 1048576.0f) { /* 2^20: quotient exact, fma remainder exact */
    const float qt = MTGP_TRUNCF(a / b);
    r = MTGP_FMAF(-qt, b, a);
    if (a >= 0.0f) {
      if (r < 0.0f) r = r + b;       /* quotient rounded up: exact fix */
      else if (r >= b) r = r - b;
    } else {
      if (r > 0.0f) r = r - b;
      else if (r <= -b) r = r + b;
    }
    return r;
  }
  return mtgp_fmod_2pi_large(a);
}

/* jnp.remainder(a, 2pi) (floor-mod): trunc remainder, then + b when signs differ. */
MTGP_INLINE MTGP_HD float mtgp_floor_mod_2pi(float a) {
  float r = mtgp_fmod_2pi(a);
  if (r != 0.0f && r < 0.0f) r = r + MTGP_TWO_PI_F;
  return r;
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

#endif /* MTGP_F32MATH_H */
