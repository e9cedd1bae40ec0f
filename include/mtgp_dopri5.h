/*
 * mtgp_dopri5.h -- fp32 arithmetic spec of the adaptive Dopri5 + PID solve.
 *
 * The notebooks run every evaluator with
 *     solver=diffrax.Dopri5(), stepsize_controller=diffrax.PIDController(rtol, atol, dtmin=0.001)
 *     (SymbolicRegression.ipynb:136, DynamicPolicy.ipynb:105, StaticPolicy.ipynb:102)
 * through diffeqsolve(..., saveat=SaveAt(ts), event=Event(cond_fn_nan), throw=False)
 *     (SR_evaluator.py:76-79, dynamic_evaluate.py:93-96, feedforward_evaluate.py:90-93).
 * diffrax is a third-party dependency absent from this image and unpinned by the reference (no
 * lock file; diffrax.Event implies >= 0.6): this header restates its published algorithm, and
 * like mtgp_f32math.h it is the shared arithmetic spec that the GPU kernel (k_sr_dopri5) and the
 * CPU oracle (oracle/mtgp_oracle.c solve_dopri5) both follow, so that they agree bit for bit.
 * The stepping loop itself is written independently on each side.
 *
 * Per rollout (state y, time t, step h, FSAL derivative f0 = f(t, y)):
 *   stages  f_i = f(t + c_i h, y + h * sum_{j<i} a_ij f_j), i = 1..6 (ascending-j fma chain, first
 *           term a_i0 * f0, zero entries included: fma(0, f_j, acc) -- a non-finite f_j makes the
 *           sum NaN as in diffrax's dot product over the padded tableau row, mtgp_cstep.h);
 *           y1 = stage-6 input (Dopri5 is FSAL: b = a_6j, whose b_1 = 0 is such an entry);
 *   error   err = h * sum_j e_j f_j (e = b - b_hat, same chain form, e_1 = 0 included);
 *   norm    m = mean_i (err_i / (atol + rtol * max(|y_i|, |y1_i|)))^2  (rms_norm squared,
 *           summed in index order; "scaled error < 1" is tested as m < 1);
 *   accept  keep = m < 1 || at_dtmin  (force_dtmin=True);
 *   factor  PIDController defaults pcoeff 0, icoeff 1, dcoeff 0, safety 0.9, factormin 0.2,
 *           factormax 10, error_order = Dopri5.order = 5:
 *             factor = clip(0.9 * m^(-1/10), keep ? 1 : 0.2, 10); m == 0 -> 10; m inf/NaN -> the
 *             lower clip (diffrax: inv_scaled_error 0; a NaN error is treated like inf here)
 *   next    dt = h * factor; dt = min(dt, dtmax); at_dtmin = dt <= dtmin; dt = max(dt, dtmin)
 *           t <- keep ? t + h : t;  tnext = t + dt, and if tnext > t_end - 1e-6:
 *           tnext = keep ? t_end : t + 0.5 (t_end - t)        (diffrax _clip_to_end, f32 tol)
 *   saves   SaveAt(ts): ts[0] -> y0; each accepted step [t, t + h] saves every pending ts[k] with
 *           ts[k] <= t + h through the Dopri5 dense output: y_mid = y + h sum_j cmid_j f_j,
 *           k0 = h f0, k1 = h f6, the quartic through (y, y1, y_mid, k0, k1)
 *           (diffrax FourthOrderPolynomialInterpolation) at theta = (ts[k] - t) / h;
 *   stop    after an accepted step whose y1 makes the event condition negative (saves of that
 *           step are written first); after max_steps attempts (accepted + rejected); at t_end.
 *           Unsaved points are +inf (throw=False).
 */
#ifndef MTGP_DOPRI5_H
#define MTGP_DOPRI5_H
#include "mtgp_f32math.h"
#include "mtgp_prng.h" /* mtgp_logf_pos: the fdlibm log spec shared with the PRNG */

/* Dormand-Prince 5(4) tableau, each entry the f32 rounding of the exact rational */
#define MTGP_DP_F(num, den) ((float)((double)(num) / (double)(den)))
#define MTGP_DP_END_TOL 1e-6f
#define MTGP_DP_SAFETY 0.9f
#define MTGP_DP_FACTORMIN 0.2f
#define MTGP_DP_FACTORMAX 10.0f

/* c_i */
#define MTGP_DP_C1 MTGP_DP_F(1, 5)
#define MTGP_DP_C2 MTGP_DP_F(3, 10)
#define MTGP_DP_C3 MTGP_DP_F(4, 5)
#define MTGP_DP_C4 MTGP_DP_F(8, 9)

/* a_ij rows 1..6 (row 6 = b); zero entries below the diagonal are multiplied by the chain */
#define MTGP_DP_TABLE_A                                                                          \
  {                                                                                              \
    {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f},                                                        \
    {MTGP_DP_F(1, 5), 0.0f, 0.0f, 0.0f, 0.0f, 0.0f},                                             \
    {MTGP_DP_F(3, 40), MTGP_DP_F(9, 40), 0.0f, 0.0f, 0.0f, 0.0f},                                \
    {MTGP_DP_F(44, 45), MTGP_DP_F(-56, 15), MTGP_DP_F(32, 9), 0.0f, 0.0f, 0.0f},                 \
    {MTGP_DP_F(19372, 6561), MTGP_DP_F(-25360, 2187), MTGP_DP_F(64448, 6561),                    \
     MTGP_DP_F(-212, 729), 0.0f, 0.0f},                                                          \
    {MTGP_DP_F(9017, 3168), MTGP_DP_F(-355, 33), MTGP_DP_F(46732, 5247), MTGP_DP_F(49, 176),     \
     MTGP_DP_F(-5103, 18656), 0.0f},                                                             \
    {MTGP_DP_F(35, 384), 0.0f, MTGP_DP_F(500, 1113), MTGP_DP_F(125, 192),                        \
     MTGP_DP_F(-2187, 6784), MTGP_DP_F(11, 84)},                                                 \
  }
/* error weights e = b - b_hat over f0..f6 */
#define MTGP_DP_TABLE_E                                                                          \
  {MTGP_DP_F(71, 57600), 0.0f, MTGP_DP_F(-71, 16695), MTGP_DP_F(71, 1920),                       \
   MTGP_DP_F(-17253, 339200), MTGP_DP_F(22, 525), MTGP_DP_F(-1, 40)}
/* dense-output midpoint weights (diffrax _Dopri5Interpolation.c_mid = Shampine's) */
#define MTGP_DP_TABLE_CMID                                                                       \
  {MTGP_DP_F(6025192743.0, 2.0 * 30085553152.0), 0.0f,                                           \
   MTGP_DP_F(51252292925.0, 2.0 * 65400821598.0), MTGP_DP_F(-2691868925.0, 2.0 * 45128329728.0), \
   MTGP_DP_F(187940372067.0, 2.0 * 1594534317056.0), MTGP_DP_F(-1776094331.0, 2.0 * 19743644256.0), \
   MTGP_DP_F(11237099.0, 2.0 * 235043384.0)}

/* stage time offset c_i (i = 0..6) */
MTGP_INLINE MTGP_HD float mtgp_dp_c(int i) {
  return i == 0 ? 0.0f : i == 1 ? MTGP_DP_C1 : i == 2 ? MTGP_DP_C2 : i == 3 ? MTGP_DP_C3 : i == 4 ? MTGP_DP_C4 : 1.0f;
}

/* one term of a weighted chain: acc + w * f (fma), the first term (first != 0) w * f; a zero weight
 * is a term too (0 * f: +-0, or NaN for a non-finite f) */
MTGP_INLINE MTGP_HD float mtgp_dp_term(float acc, float w, float f, int first) {
  return first ? w * f : MTGP_FMAF(w, f, acc);
}

/* PID step factor from m = mean squared scaled error (see the header comment) */
MTGP_INLINE MTGP_HD float mtgp_dp_factor(float m, int keep) {
  const float lo = keep ? 1.0f : MTGP_DP_FACTORMIN;
  if (m == 0.0f) return MTGP_DP_FACTORMAX;
  if (!mtgp_isfinite(m)) return lo;
  float f = MTGP_DP_SAFETY * mtgp_expf(-0.1f * mtgp_logf_pos(m));
  f = f < lo ? lo : f;
  return f > MTGP_DP_FACTORMAX ? MTGP_DP_FACTORMAX : f;
}

/* General PIDController (diffrax.PIDController(pcoeff, icoeff, dcoeff, safety, factormin,
 * factormax)), restated from diffrax's published adapt_step_size: with error order 5,
 *   c1 = (i + p + d) / 5, c2 = -(p + 2 d) / 5, c3 = d / 5,
 *   factor = clip(safety * inv^c1 * prev^c2 * prev2^c3, keep ? 1 : factormin, factormax)
 * (a factor with a zero exponent is 1, products left to right), inv = 1 / rms = m^(-1/2) of the
 * mean square m, prev / prev2 the inverse errors of the last two ACCEPTED steps (initially 1; an
 * inverse error of 0 or inf is stored as 1).  inv^c1 is exp(-(c1/2) log m) so that the default
 * (c1 = 0.2, safety 0.9, factormin 0.2, factormax 10) reproduces mtgp_dp_factor bit for bit; the
 * m == 0 / non-finite m rules are mtgp_dp_factor's. */
typedef struct {
  float c1, c2, c3, safety, factormin, factormax;
} MtgpDpPid;

MTGP_INLINE MTGP_HD float mtgp_dp_factor_pid(float m, int keep, float prev, float prev2, const MtgpDpPid* c) {
  const float lo = keep ? 1.0f : c->factormin;
  if (!(m == 0.0f) && !mtgp_isfinite(m)) return lo;
  float f = c->safety;
  if (c->c1 != 0.0f)  /* inv^c1; m == 0: inv = inf, so inf (c1 > 0) or 0 (c1 < 0) */
    f = f * (m == 0.0f ? (c->c1 > 0.0f ? mtgp_u2f(0x7f800000u) : 0.0f) : mtgp_expf((-0.5f * c->c1) * mtgp_logf_pos(m)));
  if (c->c2 != 0.0f) f = f * mtgp_expf(c->c2 * mtgp_logf_pos(prev));
  if (c->c3 != 0.0f) f = f * mtgp_expf(c->c3 * mtgp_logf_pos(prev2));
  f = f < lo ? lo : f;
  return f > c->factormax ? c->factormax : f;
}

/* the inverse error carried to the next steps: 1 / rms of m, with 0 / inf (and NaN) stored as 1 */
MTGP_INLINE MTGP_HD float mtgp_dp_inv_error(float m) {
  if (!(m > 0.0f) || !mtgp_isfinite(m)) return 1.0f;
  const float v = mtgp_expf(-0.5f * mtgp_logf_pos(m));
  return (v == 0.0f || !mtgp_isfinite(v)) ? 1.0f : v;
}

/* Controller state of one solve (init {1, 1, 0}) and one controller decision after an attempt with
 * mean squared scaled error ms and size h: keep (accept), the next dt after the factor, dtmax and
 * dtmin, the state update (at_dtmin; on accept the inverse errors shift), and fail = 1 when
 * force_dtmin is off and dt fell below dtmin (diffrax RESULTS.dt_min_reached: the solve ends after
 * this attempt; with throw=False the unsaved points are +inf).  With the default coefficients and
 * force_dtmin this is the round-1 rule bit for bit. */
typedef struct {
  float prev, prev2;
  int at_dtmin;
} MtgpDpCtl;

MTGP_INLINE MTGP_HD float mtgp_dp_control(float ms, float h, float dtmin, float dtmax, int force_dtmin,
                                          const MtgpDpPid* c, MtgpDpCtl* st, int* keep_out, int* fail_out) {
  const int keep = (ms < 1.0f) || (force_dtmin && st->at_dtmin);
  float dt = h * mtgp_dp_factor_pid(ms, keep, st->prev, st->prev2, c);
  if (dtmax > 0.0f && dt > dtmax) dt = dtmax;
  int fail = 0;
  if (dtmin > 0.0f) {
    if (!force_dtmin && dt < dtmin) fail = 1;
    st->at_dtmin = dt <= dtmin;
    dt = dt < dtmin ? dtmin : dt;
  }
  if (keep && (c->c2 != 0.0f || c->c3 != 0.0f)) {
    st->prev2 = st->prev;
    st->prev = mtgp_dp_inv_error(ms);
  }
  *keep_out = keep;
  *fail_out = fail;
  return dt;
}

/* the default controller's coefficients (diffrax PIDController defaults) */
#define MTGP_DP_PID_DEFAULT {0.2f, 0.0f, 0.0f, MTGP_DP_SAFETY, MTGP_DP_FACTORMIN, MTGP_DP_FACTORMAX}

/* scaled error of one component: err / (atol + rtol * max(|y0|, |y1|)) */
MTGP_INLINE MTGP_HD float mtgp_dp_scaled(float err, float y0, float y1, float rtol, float atol) {
  const float a0 = MTGP_FABSF(y0), a1 = MTGP_FABSF(y1);
  const float ym = (mtgp_isnan(a0) || mtgp_isnan(a1)) ? mtgp_qnan() : (a0 > a1 ? a0 : a1); /* jnp.maximum */
  return err / MTGP_FMAF(rtol, ym, atol);
}

/* the next attempt's end time (diffrax _clip_to_end) */
MTGP_INLINE MTGP_HD float mtgp_dp_clip_end(float t, float dt, float t_end, int keep) {
  const float tn = t + dt;
  if (tn > t_end - MTGP_DP_END_TOL) return keep ? t_end : MTGP_FMAF(0.5f, t_end - t, t);
  return tn;
}

/* dense output of one component at theta in [0, 1] of an accepted step:
 * y0, y1 (= y0 + ...), ymid = y0 + h * sum cmid_j f_j, k0 = h f0, k1 = h f6 */
MTGP_INLINE MTGP_HD float mtgp_dp_interp(float y0, float y1, float ymid, float k0, float k1, float th) {
  const float a = (2.0f * (k1 - k0) - 8.0f * (y1 + y0)) + 16.0f * ymid;
  const float b = (((5.0f * k0 - 3.0f * k1) + 18.0f * y0) + 14.0f * y1) - 32.0f * ymid;
  const float c = (((k1 - 4.0f * k0) - 11.0f * y0) - 5.0f * y1) + 16.0f * ymid;
  return MTGP_FMAF(MTGP_FMAF(MTGP_FMAF(MTGP_FMAF(a, th, b), th, c), th, k0), th, y0);
}

#endif /* MTGP_DOPRI5_H */
