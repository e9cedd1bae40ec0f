/*
 * mtgp_dual.h -- forward-mode (value, tangent) arithmetic of the control environments: the fp32
 * spec of the derivative that coefficient optimisation takes through the control evaluators
 * (GeneticProgramming.epoch's value_and_grad, gp.py:435-452, vmapped at gp.py:253), shared by the
 * GPU kernel (csrc/mtgp_grad.hip) and the CPU oracle (oracle/mtgp_oracle.c) like mtgp_f32math.h.
 *
 * Values: exactly the operations of the evaluators' environment code (acrobot.py:51-72,
 * harmonic_oscillator.py:58-69, reactor.py:60-69 in the oracle's evaluation order), so a dual
 * solve's value half equals the evaluator's bit for bit.  Tangents: JAX's JVP rules with its
 * symbolic zeros -- an operand that does not depend on the coefficients (a parameter, a literal)
 * contributes no tangent term (the _c forms), max/min split a tie 1/2 : 1/2 (jnp.clip's
 * maximum/minimum), floor-mod passes the tangent through (jnp.remainder), sin' = cos, cos' =
 * -sin, exp' = exp.  JAX itself differentiates in reverse mode, whose roundings differ; the
 * derivative is pinned to complex-step float64 (tests/test_coefficients.py), not bit for bit.
 */
#ifndef MTGP_DUAL_H
#define MTGP_DUAL_H

#include "mtgp.h"
#include "mtgp_f32math.h"

typedef struct {
  float v, d;
} MtgpDual;

MTGP_INLINE MTGP_HD MtgpDual mtgp_dl(float v, float d) {
  MtgpDual r;
  r.v = v;
  r.d = d;
  return r;
}
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_add(MtgpDual a, MtgpDual b) { return mtgp_dl(a.v + b.v, a.d + b.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_sub(MtgpDual a, MtgpDual b) { return mtgp_dl(a.v - b.v, a.d - b.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_mul(MtgpDual a, MtgpDual b) { return mtgp_dl(a.v * b.v, a.d * b.v + a.v * b.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_div(MtgpDual a, MtgpDual b) {
  const float q = a.v / b.v;
  return mtgp_dl(q, (a.d - q * b.d) / b.v);
}
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_neg(MtgpDual a) { return mtgp_dl(-a.v, -a.d); }
/* with a constant operand c (no tangent) */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_cmul(float c, MtgpDual a) { return mtgp_dl(c * a.v, c * a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_mulc(MtgpDual a, float c) { return mtgp_dl(a.v * c, a.d * c); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_addc(MtgpDual a, float c) { return mtgp_dl(a.v + c, a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_cadd(float c, MtgpDual a) { return mtgp_dl(c + a.v, a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_subc(MtgpDual a, float c) { return mtgp_dl(a.v - c, a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_csub(float c, MtgpDual a) { return mtgp_dl(c - a.v, -a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_divc(MtgpDual a, float c) { return mtgp_dl(a.v / c, a.d / c); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_cdiv(float c, MtgpDual b) {
  const float q = c / b.v;
  return mtgp_dl(q, (-(q * b.d)) / b.v);
}
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_sin(MtgpDual a) { return mtgp_dl(mtgp_sinf(a.v), mtgp_cosf(a.v) * a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_cos(MtgpDual a) { return mtgp_dl(mtgp_cosf(a.v), -mtgp_sinf(a.v) * a.d); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_exp(MtgpDual a) {
  const float e = mtgp_expf(a.v);
  return mtgp_dl(e, e * a.d);
}
/* the round-3 unary tree operators, tangents as jax.lax defines their JVPs:
 * log: g / x;  sqrt: g * (0.5 / ans);  tanh: (g + g * ans) * (1 - ans);  abs: sign(x) * g */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_log(MtgpDual a) { return mtgp_dl(mtgp_logf(a.v), a.d / a.v); }
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_sqrt(MtgpDual a) {
  const float s = mtgp_sqrtf(a.v);
  return mtgp_dl(s, a.d * (0.5f / s));
}
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_tanh(MtgpDual a) {
  const float t = mtgp_tanhf(a.v);
  return mtgp_dl(t, (a.d + a.d * t) * (1.0f - t));
}
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_abs(MtgpDual a) {
  const float sg = a.v > 0.0f ? 1.0f : (a.v < 0.0f ? -1.0f : a.v);  /* jnp.sign: +-0 -> +-0, NaN -> NaN */
  return mtgp_dl(mtgp_absf(a.v), sg * a.d);
}
/* one of the unary tree operators by function code (MTGP_FN_*): sin .. abs */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_unary(int fn, MtgpDual a) {
  switch (fn) {
    case MTGP_FN_SIN: return mtgp_dl_sin(a);
    case MTGP_FN_COS: return mtgp_dl_cos(a);
    case MTGP_FN_EXP: return mtgp_dl_exp(a);
    case MTGP_FN_LOG: return mtgp_dl_log(a);
    case MTGP_FN_SQRT: return mtgp_dl_sqrt(a);
    case MTGP_FN_TANH: return mtgp_dl_tanh(a);
    default: return mtgp_dl_abs(a);
  }
}

/* jnp.clip(u, lo, hi) = minimum(maximum(u, lo), hi): value as mtgp_clip (NaN propagates), tangent
 * through maximum then minimum, each 1 / 1/2 (tie) / 0 */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_clip(MtgpDual u, float lo, float hi) {
  const float m = mtgp_isnan(u.v) ? u.v : (u.v < lo ? lo : u.v);
  const float w1 = u.v > lo ? 1.0f : (u.v == lo ? 0.5f : 0.0f);
  const float t1 = u.d * w1;
  const float w2 = m < hi ? 1.0f : (m == hi ? 0.5f : 0.0f);
  return mtgp_dl(mtgp_clip(u.v, lo, hi), t1 * w2);
}

/* Acrobot angle wrap (acrobot.py:31): floor-mod passes the tangent through */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_wrap_angle(MtgpDual a) { return mtgp_dl(mtgp_wrap_angle(a.v), a.d); }

/* Acrobot.drift (acrobot.py:51-72), prm = (l1, l2, m1, m2): the oracle's acro_drift in duals */
MTGP_INLINE MTGP_HD void mtgp_dl_acro_drift(const float* prm, const MtgpDual* st, MtgpDual u_raw, MtgpDual* dx) {
  const MtgpDual control = mtgp_dl_clip(u_raw, -1.0f, 1.0f);
  const MtgpDual th1 = st[0], th2 = st[1], thd1 = st[2], thd2 = st[3];
  const float l1 = prm[0], l2 = prm[1], m1 = prm[2], m2 = prm[3];
  const float lc1 = 0.5f * l1, lc2 = 0.5f * l2;
  const float moi1 = 1.0f, moi2 = 1.0f, g = 9.81f;
  const MtgpDual c2 = mtgp_dl_cos(th2), s2 = mtgp_dl_sin(th2), s1 = mtgp_dl_sin(th1);
  const MtgpDual ca = mtgp_dl_cos(mtgp_dl_subc(mtgp_dl_add(th1, th2), MTGP_HALF_PI_F));
  const MtgpDual cb = mtgp_dl_cos(mtgp_dl_subc(th1, MTGP_HALF_PI_F));
  const MtgpDual d1 = mtgp_dl_addc(
      mtgp_dl_addc(mtgp_dl_cadd(m1 * (lc1 * lc1),
                                mtgp_dl_cmul(m2, mtgp_dl_cadd((l1 * l1) + (lc2 * lc2), mtgp_dl_cmul((2.0f * l1) * lc2, c2)))),
                   moi1),
      moi2);
  const MtgpDual d2 = mtgp_dl_addc(mtgp_dl_cmul(m2, mtgp_dl_cadd(lc2 * lc2, mtgp_dl_cmul(l1 * lc2, c2))), moi2);
  const MtgpDual phi2 = mtgp_dl_cmul((m2 * lc2) * g, ca);
  const MtgpDual t1 = mtgp_dl_mul(mtgp_dl_cmul(((-m2) * l1) * lc2, mtgp_dl_mul(thd2, thd2)), s2);
  const MtgpDual t2 = mtgp_dl_mul(mtgp_dl_mul(mtgp_dl_cmul(((2.0f * m2) * l1) * lc2, thd1), thd2), s1);
  const MtgpDual t3 = mtgp_dl_cmul(((m1 * lc1) + (m2 * l1)) * g, cb);
  const MtgpDual phi1 = mtgp_dl_add(mtgp_dl_add(mtgp_dl_sub(t1, t2), t3), phi2);
  const MtgpDual num = mtgp_dl_sub(
      mtgp_dl_sub(mtgp_dl_add(control, mtgp_dl_mul(mtgp_dl_div(d2, d1), phi1)),
                  mtgp_dl_mul(mtgp_dl_cmul((m2 * l1) * lc2, mtgp_dl_mul(thd1, thd1)), s2)),
      phi2);
  const MtgpDual den = mtgp_dl_csub((m2 * (lc2 * lc2)) + moi2, mtgp_dl_div(mtgp_dl_mul(d2, d2), d1));
  const MtgpDual th2acc = mtgp_dl_div(num, den);
  const MtgpDual th1acc = mtgp_dl_div(mtgp_dl_neg(mtgp_dl_add(mtgp_dl_mul(d2, th2acc), phi1)), d1);
  dx[0] = thd1;
  dx[1] = thd2;
  dx[2] = th1acc;
  dx[3] = th2acc;
}

/* HarmonicOscillator.drift (harmonic_oscillator.py:58-69), prm = (omega, zeta) */
MTGP_INLINE MTGP_HD void mtgp_dl_ho_drift(const float* prm, const MtgpDual* x, MtgpDual u, MtgpDual* dx) {
  const float A[2][2] = {{0.0f, 1.0f}, {-prm[0], -prm[1]}};
  const float b[2] = {0.0f, 1.0f};
  for (int i = 0; i < 2; ++i)
    dx[i] = mtgp_dl_add(mtgp_dl_add(mtgp_dl_cmul(A[i][0], x[0]), mtgp_dl_cmul(A[i][1], x[1])), mtgp_dl_cmul(b[i], u));
}

/* StirredTankReactor.drift (reactor.py:60-69), prm = (Vol, Cp, dHr, UA, q, Tf, Tcf, Volc) */
MTGP_INLINE MTGP_HD void mtgp_dl_reactor_drift(const float* prm, const MtgpDual* x, MtgpDual u, MtgpDual* dx) {
  const float Vol = prm[0], Cp = prm[1], dHr = prm[2], UA = prm[3], q = prm[4], Tf = prm[5], Tcf = prm[6],
              Volc = prm[7];
  const MtgpDual Tc = x[0], T = x[1], cc = x[2];
  const MtgpDual control = mtgp_dl_clip(u, 0.0f, 300.0f);
  const MtgpDual kT = mtgp_dl_cmul(7.2e10f, mtgp_dl_exp(mtgp_dl_cdiv((float)(-72750.0 / 8.314), T)));
  const MtgpDual dc = mtgp_dl_sub(mtgp_dl_cmul(q / Vol, mtgp_dl_csub(1.0f, cc)), mtgp_dl_mul(kT, cc));
  const MtgpDual dT = mtgp_dl_add(mtgp_dl_add(mtgp_dl_cmul(q / Vol, mtgp_dl_csub(Tf, T)),
                                              mtgp_dl_mul(mtgp_dl_cmul((-dHr) / Cp, kT), cc)),
                                  mtgp_dl_cmul((UA / Vol) / Cp, mtgp_dl_sub(Tc, T)));
  const MtgpDual dTc = mtgp_dl_add(mtgp_dl_mul(mtgp_dl_divc(control, Volc), mtgp_dl_csub(Tcf, Tc)),
                                   mtgp_dl_cmul((UA / Volc) / Cp, mtgp_dl_sub(T, Tc)));
  dx[0] = dTc;
  dx[1] = dT;
  dx[2] = dc;
}

/* (e^T Q) e, every product summed left to right (the oracle's quad_form), Q constant */
MTGP_INLINE MTGP_HD MtgpDual mtgp_dl_quad_form(const MtgpDual* e, const float* Q, int n) {
  MtgpDual out = mtgp_dl(0.0f, 0.0f);
  for (int j = 0; j < n; ++j) {
    MtgpDual v = mtgp_dl_mulc(e[0], Q[0 * n + j]);
    for (int i = 1; i < n; ++i) v = mtgp_dl_add(v, mtgp_dl_mulc(e[i], Q[i * n + j]));
    out = (j == 0) ? mtgp_dl_mul(v, e[0]) : mtgp_dl_add(out, mtgp_dl_mul(v, e[j]));
  }
  return out;
}

#endif /* MTGP_DUAL_H */
