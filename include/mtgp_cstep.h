/*
 * mtgp_cstep.h -- fp32 arithmetic spec of the fixed-step solve: diffrax.ConstantStepSize with the
 * Euler or classical RK4 solver, SaveAt(ts) through the solver's dense output (ABI v18).
 *
 * The reference evaluators integrate with
 *     diffeqsolve(ODETerm(_drift), solver, ts[0], ts[-1], dt0, y0, saveat=SaveAt(ts),
 *                 stepsize_controller=ConstantStepSize(), max_steps, event=Event(cond_fn), throw=False)
 *     (dynamic_evaluate.py:11, 88-96; feedforward_evaluate.py:11, 86-93; SR_evaluator.py:21, 70-79)
 * diffrax is a third-party dependency absent from this image and unpinned by the reference (no lock
 * file; diffrax.Event implies >= 0.6).  This header restates its published algorithm; like
 * mtgp_dopri5.h it is the shared arithmetic spec that the GPU kernels and the CPU oracle
 * (oracle/mtgp_oracle.c) both follow, the stepping loop itself being written on each side.
 *
 * Time grid (wave-uniform: ts is shared by every rollout, dyn.py:63 in_axes None):
 *   t_0 = ts[0];  tn_0 = min(t_0 + dt0, t1)          ConstantStepSize.init + diffeqsolve's minimum
 *   step n integrates [t_n, tn_n] with dt_n = tn_n - t_n (ODETerm.contr)
 *   t_{n+1} = tn_n;  tn_{n+1} = t_{n+1} + dt0, and t1 when > t1 - 1e-6   adapt_step_size + _clip_to_end
 *   the loop runs while t_n < t1 and fewer than max_steps steps were taken (max_steps reached:
 *   the unsaved points stay +inf, throw=False), and ends early on a stalled grid
 *   (mtgp_cs_advancing).  The step ends are ACCUMULATED in f32, so they
 *   drift off n * dt0 (C3: 189 of 200 step ends differ) and the step count can exceed the
 *   nominal one (t1 = 2, dt0 = 0.01: 201 steps, the last 1.5e-6 long).
 * Stages (ODETerm: is_vf_expensive False, so diffrax keeps the vector-field values f_i and forms each
 * increment as (sum_j a_ij f_j) * dt; products and sums rounded separately, ascending j).  Zero
 * tableau entries are MULTIPLIED, not skipped (round 6): diffrax's
 * AbstractRungeKutta runs its stages as a loop over a zero-padded lower-triangular tableau and forms
 * each stage's increment as one dot product of that padded row with the buffer of stage values, so
 * a_ij = 0 still contributes 0 * f_j -- +-0 for a finite f_j, NaN for an infinite or NaN one.  (The
 * diffrax source is not in this image, and the reference pins no version: this is its published
 * implementation as restated here, not a quotation.)  The padded row's trailing 0 * 0 terms of the
 * stages not yet computed can only turn a -0 sum into +0 and are not restated.
 *   Euler   f0 = f(t, y);  y1 = y + f0 * dt
 *   RK4     f0 = f(t, y)
 *           f1 = f(t + 0.5 dt, y + (0.5 f0) dt)
 *           f2 = f(t + 0.5 dt, y + (0 f0 + 0.5 f1) dt)
 *           f3 = f(t + 1.0 dt, y + ((0 f0 + 0 f1) + 1.0 f2) dt)
 *           y1 = y + (((b0 f0 + b1 f1) + b2 f2) + b3 f3) dt,  b = f32(1/6, 1/3, 1/3, 1/6)
 *           The zero-entry part z = 0 f0 / 0 f0 + 0 f1 is +-0 for finite derivatives and NaN
 *           otherwise; the spec reads a +-0 z as an exact no-op (its only effect on a sum is the
 *           sign of an all-zero increment, the convention that also drops the trailing 0 * 0 terms)
 *           and a NaN z as NaN: a non-finite earlier stage derivative makes the stage input NaN in
 *           that component, where skipping the entry would not.  So with finite f0, f1 the inputs
 *           are the plain y + (0.5 f1) dt, y + (1.0 f2) dt; the kernels test the running
 *           b-weighted sum instead of carrying z (mtgp_rk4_in_acc).
 * SaveAt(ts): after each step every pending ts[k] <= tn (k ascending, ts[0] included at step 0) is
 *   evaluated through the step's dense output at theta = linear_rescale(t, ts[k], tn):
 *   Euler   LocalLinearInterpolation: y + theta (y1 - y)
 *   RK4     ThirdOrderHermitePolynomialInterpolation.from_k (k0 = f0 dt, k1 = f3 dt, the first and
 *           last stage increments): a = ((k0 + k1) + 2 y) - 2 y1, b = (((-2 k0) - k1) - 3 y) + 3 y1,
 *           value = jnp.polyval([a, b, k0, y], theta) (Horner from 0: v = v * theta + c)
 *   so a save on a step end is the interpolant at theta = 1, not the step's y1 bit for bit.
 * Event: after a step whose y1 turns the condition negative the solve ends; that step's saves are
 *   written first, the later ones are +inf.
 */
#ifndef MTGP_CSTEP_H
#define MTGP_CSTEP_H
#include "mtgp_f32math.h"

#define MTGP_CS_END_TOL 1e-6f /* diffrax _clip_to_end, float32 */
#define MTGP_RK4_B0 ((float)(1.0 / 6.0))
#define MTGP_RK4_B1 ((float)(1.0 / 3.0))

/* end of the first step: jnp.minimum(t0 + dt0, t1) */
MTGP_INLINE MTGP_HD float mtgp_cs_first_end(float t0, float dt0, float t1) {
  const float tn = t0 + dt0;
  return tn < t1 ? tn : t1;
}

/* end of the step after one that ended at t (a kept step: _clip_to_end's keep_step branch) */
MTGP_INLINE MTGP_HD float mtgp_cs_next_end(float t, float dt0, float t1) {
  const float tn = t + dt0;
  return tn > t1 - MTGP_CS_END_TOL ? t1 : tn;
}

/* Loop guard against a stalled grid: when dt0 is below half an ulp of t, t + dt0 rounds back to t
 * and diffrax keeps taking dt = 0 steps until max_steps (then the unsaved points are +inf).  Only
 * the FIRST such step can save anything (ts[k] <= tn = t; every later stalled step has the same
 * tn, whose points are then already saved) and none of them moves a saved value, so ending the
 * solve before the second stalled step gives the same outputs and cannot loop forever when the
 * solve has no max_steps (C entry: max_steps 0). */
MTGP_INLINE MTGP_HD int mtgp_cs_advancing(int steps, float t, float tn) { return steps == 0 || tn > t; }

/* diffrax misc.linear_rescale: (t - t0) / (t1 - t0), 0 when t0 == t1 */
MTGP_INLINE MTGP_HD float mtgp_cs_rescale(float t0, float t, float t1) {
  return t0 == t1 ? 0.0f : (t - t0) / (t1 - t0);
}

/* ThirdOrderHermitePolynomialInterpolation of one component (see the header comment).  Every
 * product and sum rounds as written (an fma for "s + 2 y" would differ where 2 y overflows), except
 * jnp.polyval's first step 0 * th + a: th = linear_rescale(...) is finite and >= +0 on every call
 * (ts[k] >= t, tn > t), so 0 * th = +0 and +0 + a = a + 0.0f exactly (-0 -> +0, NaN stays NaN). */
MTGP_INLINE MTGP_HD float mtgp_cs_hermite(float y0, float y1, float k0, float k1, float th) {
  const float a = ((k0 + k1) + 2.0f * y0) - 2.0f * y1;
  const float b = (((-2.0f * k0) - k1) - 3.0f * y0) + 3.0f * y1;
  float v = a + 0.0f;
  v = v * th + b;
  v = v * th + k0;
  return v * th + y0;
}

/* LocalLinearInterpolation of one component */
MTGP_INLINE MTGP_HD float mtgp_cs_linear(float y0, float y1, float th) { return y0 + th * (y1 - y0); }

/* the zero-entry sum z (+-0, or NaN when an earlier zero-weighted derivative was not finite) joined
 * to the stage row's other terms v: NaN propagates, a +-0 z is a no-op */
MTGP_INLINE MTGP_HD float mtgp_rk4_nz(float z, float v) { return z != z ? z : v; }
/* RK4 stage input for stage st = 1, 2, 3 from f = the previous stage's derivative and z = the
 * zero-entry terms of the stage's tableau row (stage 2: 0 f0; stage 3: 0 f0 + 0 f1; unused at
 * stage 1): y + (0.5 f0) dt, y + [z; 0.5 f1] dt, y + [z; 1.0 f2] dt */
MTGP_INLINE MTGP_HD float mtgp_rk4_in(int st, float y, float f, float z, float dt) {
  return st == 1 ? y + (0.5f * f) * dt : st == 2 ? y + mtgp_rk4_nz(z, 0.5f * f) * dt : y + mtgp_rk4_nz(z, f) * dt;
}
/* The same in the kernels' register-free form: acc = the b-weighted sum of the earlier stage
 * derivatives WITHOUT f's term (mtgp_rk4_acc through stage st - 2: b0 f0 at stage 2, b0 f0 + b1 f1
 * at stage 3).  acc is non-finite exactly when one of those derivatives is (|b0 f0 + b1 f1| <=
 * FLT_MAX / 2 for finite f0, f1: no overflow), i.e. exactly when z is NaN, so [z; v] is
 * (acc finite ? v : NaN) -- mtgp_rk4_in bit for bit up to the NaN payload, with no z carried. */
MTGP_INLINE MTGP_HD float mtgp_rk4_in_acc(int st, float y, float f, float acc, float dt) {
  if (st == 1) return y + (0.5f * f) * dt;
  const float v = st == 2 ? 0.5f * f : f;
  return y + (mtgp_isfinite(acc) ? v : mtgp_u2f(0x7fc00000u)) * dt;
}
/* the zero-entry sum after stage st's input was formed from f = f_{st-1}: stage 1 starts it (0 f0,
 * for stage 2), stage 2 adds 0 f1 (for stage 3); stage 3 leaves it */
MTGP_INLINE MTGP_HD float mtgp_rk4_zero(int st, float z, float f) {
  return st == 1 ? 0.0f * f : st == 2 ? z + 0.0f * f : z;
}
/* RK4 stage time t + c dt for stage st = 1, 2, 3 (c = 0.5, 0.5, 1.0) */
MTGP_INLINE MTGP_HD float mtgp_rk4_time(int st, float t, float dt) {
  return st == 3 ? t + 1.0f * dt : t + 0.5f * dt;
}
/* running b-weighted sum: stage 0 starts it, stages 1..3 add (ascending j) */
MTGP_INLINE MTGP_HD float mtgp_rk4_acc(int st, float acc, float f) {
  return st == 0 ? MTGP_RK4_B0 * f : acc + (st == 3 ? MTGP_RK4_B0 : MTGP_RK4_B1) * f;
}
/* the step's end state from the full sum */
MTGP_INLINE MTGP_HD float mtgp_rk4_out(float y, float acc, float dt) { return y + acc * dt; }

#endif /* MTGP_CSTEP_H */
