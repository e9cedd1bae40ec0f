/*
 * mtgp_oracle.c -- CPU restatement of the MultiTreeGP population-fitness hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (multitreegp_amd) never calls it.
 *
 * It restates the reference's algorithm literally, independently of the product's
 * program flattener: trees are interpreted row by row over all N rows exactly like
 * GeneticProgramming.body_fun/foriloop (gp.py:356-388), the fitness is computed from
 * the full saved trajectory arrays the way the environments do (acrobot.py:77-84,
 * SR_evaluator.py:24), not online.  The only shared code is the fp32 arithmetic spec
 * (include/mtgp_f32math.h: sin/cos/floor-mod), which pins the numerics that the
 * reference delegates to XLA; fixed-step RK4 replaces diffrax.diffeqsolve as
 * BASELINE.json prescribes.
 *
 * Parity status: the reference (JAX/diffrax) cannot be imported here
 * (ModuleNotFoundError) and ships no golden vectors -> parity vs the
 * reference is UNPINNED; this oracle is pinned by analytic known-answer tests, a
 * float64 numpy restatement and sympy evaluation of the reference's printed
 * expressions (tests/test_oracle.py).  The observation noise uses the PRNG spec
 * include/mtgp_prng.h, pinned by the Random123 threefry KATs and JAX's published
 * split/normal outputs for PRNGKey(0) (tests/test_prng.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "mtgp_f32math.h"
#include "mtgp_prng.h"
#include "mtgp_dopri5.h"
#include "mtgp_cstep.h"
#include "mtgp_dual.h"

#define OR_MAX_N 256
#define OR_MAX_D 64
#define OR_MAX_S 64 /* state dims */

/* node-function codes (same numbering as include/mtgp.h MTGP_FN_*) */
enum { FN_ZERO = 0, FN_VAR = 1, FN_ADD = 2, FN_SUB = 3, FN_MUL = 4, FN_DIV = 5, FN_SIN = 6, FN_COS = 7,
       FN_EXP = 8, FN_LOG = 9, FN_SQRT = 10, FN_TANH = 11, FN_ABS = 12 };

typedef struct {
  int32_t n_funcs, var_start;
  const int8_t* fn;
} OrLib;

/* f32 -> int32: truncation, saturating, NaN -> 0 (astype(int), gp.py:370-372) */
static int32_t or_f2i(float v) {
  if (v != v) return 0;
  if (v >= 2147483648.0f) return 2147483647;
  if (v <= -2147483648.0f) return -2147483647 - 1;
  return (int32_t)v;
}
/* jnp dynamic index: negative -> + N, then clamp */
static int or_index(float v, int N) {
  int64_t j = or_f2i(v);
  if (j < 0) j += N;
  if (j < 0) j = 0;
  if (j > N - 1) j = N - 1;
  return (int)j;
}

/* gp.py:356-388: evaluate rows 0..N-1 in order, return the value of row N-1. */
float oracle_eval_tree(const float* tree, int N, int n_funcs, int var_start, const int8_t* fn,
                       const float* data, int n_data) {
  float val[OR_MAX_N];
  for (int i = 0; i < N; ++i) val[i] = tree[4 * i + 3];
  for (int i = 0; i < N; ++i) {
    const float f = tree[4 * i + 0];
    const float x = val[or_index(tree[4 * i + 1], N)];
    const float y = val[or_index(tree[4 * i + 2], N)];
    float v;
    if (f == 1.0f) {
      v = tree[4 * i + 3];
    } else {
      int32_t k = or_f2i(f);
      if (k < 0) k = 0;
      if (k > n_funcs - 1) k = n_funcs - 1;
      switch (fn[k]) {
        case FN_VAR: {
          int d = k - var_start;
          if (d > n_data - 1) d = n_data - 1;
          v = data[d];
          break;
        }
        case FN_ADD: v = x + y; break;
        case FN_SUB: v = x - y; break;
        case FN_MUL: v = x * y; break;
        case FN_DIV: v = x / y; break;
        case FN_SIN: v = mtgp_sinf(x); break;
        case FN_COS: v = mtgp_cosf(x); break;
        case FN_EXP: v = mtgp_expf(x); break;
        case FN_LOG: v = mtgp_logf(x); break;
        case FN_SQRT: v = mtgp_sqrtf(x); break;
        case FN_TANH: v = mtgp_tanhf(x); break;
        case FN_ABS: v = mtgp_absf(x); break;
        default: v = 0.0f; break;
      }
    }
    val[i] = v;
  }
  return val[N - 1];
}

/* ------------------------------------------------------------------ models */
typedef struct {
  int32_t model; /* 1 dynamic acrobot, 2 static acrobot, 3 SR */
  int32_t n_var, state_size, n_obs, n_control, n_targets;
  int32_t n_steps, save_every, n_save;
  float h, max_fitness, parsimony;
  int32_t prng_impl; /* mtgp_prng.h: 0 threefry original layout, 1 partitionable */
  int32_t env;       /* control models: 0 Acrobot, 1 HarmonicOscillator, 2 StirredTankReactor */
  int32_t solver;    /* 0 fixed-step RK4 (BASELINE.json), 1 Dopri5 + PIDController (notebooks), 2 Euler */
  int32_t max_steps; /* Dopri5: step attempts, accepted + rejected (diffeqsolve max_steps) */
  float rtol, atol, dtmin, dtmax; /* PIDController; dtmin / dtmax <= 0: None */
  int32_t pid_custom;             /* 0: diffrax's default PID coefficients (mtgp.h ABI v15) */
  float pid_c1, pid_c2, pid_c3, pid_safety, pid_factormin, pid_factormax;
  int32_t no_force_dtmin;         /* 1: force_dtmin=False (dt < dtmin ends the solve) */
  /* Oracle-only alternative readings of diffrax rules for the Dopri5 solve (scripts/dp_gap_study.py,
   * DESIGN.md "Parity pins"); 0 = the spec (include/mtgp_dopri5.h) that the product follows.  Bits
   * OR_DP_ALT_*.  Never part of the product ABI. */
  int32_t dp_alt;
} OrModel;

enum {
  OR_DP_ALT_EO6 = 1,           /* error order 6 (AbstractSolver.error_order = order + 1): exponent 1/6 */
  OR_DP_ALT_FSAL_T1 = 2,       /* the last (FSAL) stage evaluated at t1 instead of t + 1 * h          */
  OR_DP_ALT_DTMIN_ATTEMPT = 4, /* at_dtmin from the attempted step (h <= dtmin), not carried         */
  OR_DP_ALT_SUM_LITERAL = 8,   /* stage sums sum(a f) with separate products / adds, then y + sum * h */
  OR_DP_ALT_NORM_X = 16,       /* error norm over the environment state only (not the hidden state)  */
  OR_DP_ALT_MAXSTEPS_ACC = 32, /* max_steps counts accepted steps only                                */
  OR_DP_ALT_EVENT_ALL = 64,    /* the Event tested on every attempt's candidate, rejected ones too    */
  OR_DP_ALT_INTERP_T0 = 128    /* ts[0] saved through the first step's dense output (not y0 directly) */
};

enum { ENV_ACROBOT = 0, ENV_HARMONIC = 1, ENV_REACTOR = 2 };

typedef struct {
  const float* x0;      /* [R, n_var] */
  const float* params;  /* [R, n_params]: Acrobot (l1, l2, m1, m2), HarmonicOscillator (omega,
                           zeta), StirredTankReactor (Vol, Cp, dHr, UA, q, Tf, Tcf, Volc) */
  const float* targets; /* [R, n_targets] */
  const float* ts;      /* [n_save] */
  const float* ys_true; /* SR: [R, n_save, n_var] (reference layout) */
  int32_t R;
  const uint32_t* obs_keys; /* [R, 2] obs_noise_keys (dyn.py:65) or NULL: noise-free */
  const float* obs_w;       /* [n_obs, n_obs] W = obs_noise * I (acrobot.py:49) */
} OrRollouts;

typedef struct {
  const OrModel* m;
  const float* cand; /* [T, N, 4] */
  int N;
  OrLib lib;
  const float* target;
  const float* prm;    /* this rollout's environment parameters */
  const uint32_t* key; /* this rollout's obs_noise_key or NULL */
  const float* W;
  int32_t* save_at;    /* diagnostic: attempt index at which each save point was written, or NULL */
} OrCtx;

/* Diagnostic (scripts/dp_save_spread.py): Dopri5 save-point timing per rollout, [P, R, S] int32
 * -- the attempt count when save k was written (0 for ts[0], -1 never); NULL turns it off. */
static int32_t* g_save_trace = NULL;
void oracle_set_save_trace(int32_t* buf) { g_save_trace = buf; }

/* EnvironmentBase.f_obs (cbase.py:43-48) with C = eye(n_var)[:n_obs] (acrobot.py:48,
 * harmonic_oscillator.py:65, reactor.py:42):
 *   out = C@x + normal(fold_in(key, bitcast_i32(t)), (n_obs,)) @ W
 * matrix products summed in index order; without a key (obs_noise = 0) the noise term is
 * +0.  Then Acrobot wraps out[0:2] (acrobot.py:29-32). */
static void ctl_f_obs(const OrCtx* c, float t, const float* x, float* y) {
  const int nv = c->m->n_var, no = c->m->n_obs;
  float nz[OR_MAX_D];
  if (c->key) {
    float n[OR_MAX_D];
    mtgp_obs_normals(c->key[0], c->key[1], t, no, c->m->prng_impl, n);
    for (int j = 0; j < no; ++j) {
      float s = n[0] * c->W[0 * no + j];
      for (int i = 1; i < no; ++i) s = s + n[i] * c->W[i * no + j];
      nz[j] = s;
    }
  } else {
    for (int j = 0; j < no; ++j) nz[j] = 0.0f;
  }
  for (int i = 0; i < no; ++i) {
    float s = 0.0f;
    int first = 1;
    for (int j = 0; j < nv; ++j) {
      const float term = (i == j ? 1.0f : 0.0f) * x[j];
      if (first) { s = term; first = 0; } else s = s + term;
    }
    y[i] = s + nz[i];
  }
  if (c->m->env == ENV_ACROBOT) {
    y[0] = mtgp_wrap_angle(y[0]);
    y[1] = mtgp_wrap_angle(y[1]);
  }
}

/* Acrobot.drift (acrobot.py:51-72), evaluation order of the Python source. */
static void acro_drift(const OrCtx* c, const float* st, float u_raw, float* dx) {
  const float control = mtgp_clip1(u_raw);
  const float th1 = st[0], th2 = st[1], thd1 = st[2], thd2 = st[3];
  const float l1 = c->prm[0], l2 = c->prm[1], m1 = c->prm[2], m2 = c->prm[3];
  const float lc1 = 0.5f * l1, lc2 = 0.5f * l2;
  const float moi1 = 1.0f, moi2 = 1.0f, g = 9.81f;
  (void)l2;
  const float d1 = m1 * (lc1 * lc1) + m2 * ((l1 * l1) + (lc2 * lc2) + ((2.0f * l1) * lc2) * mtgp_cosf(th2)) + moi1 + moi2;
  const float d2 = m2 * ((lc2 * lc2) + (l1 * lc2) * mtgp_cosf(th2)) + moi2;
  const float phi2 = ((m2 * lc2) * g) * mtgp_cosf((th1 + th2) - MTGP_HALF_PI_F);
  const float phi1 = ((((-m2) * l1) * lc2) * (thd2 * thd2)) * mtgp_sinf(th2)
                     - (((((2.0f * m2) * l1) * lc2) * thd1) * thd2) * mtgp_sinf(th1)
                     + (((m1 * lc1) + (m2 * l1)) * g) * mtgp_cosf(th1 - MTGP_HALF_PI_F) + phi2;
  const float th2acc = (control + (d2 / d1) * phi1 - (((m2 * l1) * lc2) * (thd1 * thd1)) * mtgp_sinf(th2) - phi2)
                       / ((m2 * (lc2 * lc2)) + moi2 - (d2 * d2) / d1);
  const float th1acc = (-((d2 * th2acc) + phi1)) / d1;
  dx[0] = thd1;
  dx[1] = thd2;
  dx[2] = th1acc;
  dx[3] = th2acc;
}

/* HarmonicOscillator.drift (harmonic_oscillator.py:58-69): A@state + b@args with
 * A = [[0, 1], [-omega, -zeta]], b = [[0], [1]], each product summed in index order. */
static void ho_drift(const OrCtx* c, const float* x, float u, float* dx) {
  const float omega = c->prm[0], zeta = c->prm[1];
  const float A[2][2] = {{0.0f, 1.0f}, {-omega, -zeta}};
  const float b[2] = {0.0f, 1.0f};
  for (int i = 0; i < 2; ++i) dx[i] = (A[i][0] * x[0] + A[i][1] * x[1]) + b[i] * u;
}

/* StirredTankReactor.drift (reactor.py:60-69), evaluation order of the Python source.
 * k(T) = k0 * exp(-Ea / R / T) with -Ea/R formed in Python float64 (an int over a float)
 * and rounded to f32 as a weak-typed scalar; k0 = f32(7.2e10).  The clipped `state` of
 * reactor.py:64 is never read (dc uses the unclipped c). */
#define REACTOR_MEAR_F ((float)(-72750.0 / 8.314))
#define REACTOR_K0_F 7.2e10f
static void reactor_drift(const OrCtx* c, const float* x, float u, float* dx) {
  const float Vol = c->prm[0], Cp = c->prm[1], dHr = c->prm[2], UA = c->prm[3], q = c->prm[4], Tf = c->prm[5],
              Tcf = c->prm[6], Volc = c->prm[7];
  const float Tc = x[0], T = x[1], cc = x[2];
  const float control = mtgp_clip(u, 0.0f, 300.0f);
  const float kT = REACTOR_K0_F * mtgp_expf(REACTOR_MEAR_F / T);
  const float dc = (q / Vol) * (1.0f - cc) - kT * cc;
  const float dT = (q / Vol) * (Tf - T) + ((-dHr) / Cp) * kT * cc + ((UA / Vol) / Cp) * (Tc - T);
  const float dTc = (control / Volc) * (Tcf - Tc) + ((UA / Volc) / Cp) * (T - Tc);
  dx[0] = dTc;
  dx[1] = dT;
  dx[2] = dc;
}

static void env_drift(const OrCtx* c, const float* x, float u, float* dx) {
  if (c->m->env == ENV_HARMONIC) ho_drift(c, x, u, dx);
  else if (c->m->env == ENV_REACTOR) reactor_drift(c, x, u, dx);
  else acro_drift(c, x, u, dx);
}

static float tree_eval(const OrCtx* c, int t, const float* data, int n_data) {
  return oracle_eval_tree(c->cand + (size_t)t * c->N * 4, c->N, c->lib.n_funcs, c->lib.var_start, c->lib.fn,
                          data, n_data);
}

/* dynamic_evaluate._drift (dyn.py:107-118) */
static void dyn_rhs(const OrCtx* c, float t, const float* s, float* ds) {
  const OrModel* m = c->m;
  const int no = m->n_obs, na = m->state_size, nu = m->n_control, nt = m->n_targets;
  const int D = no + na + nu + nt, nv = m->n_var;
  float y[OR_MAX_D], data[OR_MAX_D], u[8];
  ctl_f_obs(c, t, s, y);
  /* readout sees [0_obs, a, 0_u, target] */
  for (int i = 0; i < D; ++i) data[i] = 0.0f;
  for (int i = 0; i < na; ++i) data[no + i] = s[nv + i];
  for (int i = 0; i < nt; ++i) data[no + na + nu + i] = c->target[i];
  for (int j = 0; j < nu; ++j) u[j] = tree_eval(c, na + j, data, D);
  env_drift(c, s, u[0], ds);
  /* state equation sees [y, a, u, target] */
  for (int i = 0; i < no; ++i) data[i] = y[i];
  for (int j = 0; j < nu; ++j) data[no + na + j] = u[j];
  for (int i = 0; i < na; ++i) ds[nv + i] = tree_eval(c, i, data, D);
}

/* feedforward_evaluate._drift (ff.py:104-110) */
static void ff_rhs(const OrCtx* c, float t, const float* s, float* ds) {
  const OrModel* m = c->m;
  const int no = m->n_obs, nt = m->n_targets;
  float y[OR_MAX_D], data[OR_MAX_D];
  ctl_f_obs(c, t, s, y);
  for (int i = 0; i < no; ++i) data[i] = y[i];
  for (int i = 0; i < nt; ++i) data[no + i] = c->target[i];
  const float u = tree_eval(c, 0, data, no + nt);
  env_drift(c, s, u, ds);
}

/* SR_evaluator._drift (sr.py:85-88) */
static void sr_rhs(const OrCtx* c, float t, const float* s, float* ds) {
  (void)t;
  for (int i = 0; i < c->m->n_var; ++i) ds[i] = tree_eval(c, i, s, c->m->n_var);
}

static void rhs(const OrCtx* c, float t, const float* s, float* ds) {
  if (c->m->model == 1) dyn_rhs(c, t, s, ds);
  else if (c->m->model == 2) ff_rhs(c, t, s, ds);
  else sr_rhs(c, t, s, ds);
}

static int state_dim(const OrModel* m) { return m->model == 1 ? m->n_var + m->state_size : m->n_var; }

/* diffrax.Event(cond_fn) with a float condition: +1 valid, -1 terminate. */
static float cond_fn(const OrModel* m, const float* s) {
  const int n = state_dim(m);
  int bad = 0;
  for (int i = 0; i < n; ++i) bad |= !mtgp_isfinite(s[i]);
  if (m->model != 3 && m->env == ENV_ACROBOT) { /* acrobot.py:86-87 (the others: any inf/NaN only,
                                                   harmonic_oscillator.py:79-80, reactor.py:80-81) */
    bad |= (mtgp_isnan(s[2]) ? 0 : (MTGP_FABSF(s[2]) > MTGP_8PI_F));
    bad |= (mtgp_isnan(s[3]) ? 0 : (MTGP_FABSF(s[3]) > MTGP_18PI_F));
  }
  return bad ? -1.0f : 1.0f;
}

/* diffeqsolve(solver, ts[0], ts[-1], dt0 = h, SaveAt(ts), ConstantStepSize(), max_steps,
 * Event(cond_fn), throw=False) with solver = Euler (the reference evaluators' default, dyn.py:11,
 * ff.py:11, sr.py:21) or classical RK4 (BASELINE.json) -- diffrax restated in the fp32 spec of
 * include/mtgp_cstep.h (see its header comment for every rule used here): accumulated step ends
 * t += dt0 with the end clip, each step over dt = tn - t, stage times t + c_i dt, stage sums
 * (sum a_ij f_j) dt, every save point through the step's dense output, Event after the step.
 * saved[n_save][dim]; unsaved points (after the event or max_steps) = +inf.  Returns the number of
 * steps taken. */
static int solve_fixed(const OrCtx* c, const float* ts, const float* s0, float* saved) {
  const OrModel* m = c->m;
  const int n = state_dim(m), S = m->n_save, euler = m->solver == 2;
  const float t_end = ts[S - 1], dt0 = m->h;
  float y[OR_MAX_S], f0[OR_MAX_S], f[OR_MAX_S], acc[OR_MAX_S], yi[OR_MAX_S], y1[OR_MAX_S], z[OR_MAX_S];
  for (int i = 0; i < n; ++i) y[i] = s0[i];
  float prev = cond_fn(m, y);
  int k = 0, steps = 0;
  float t = ts[0], tn = mtgp_cs_first_end(t, dt0, t_end);
  while (t < t_end && mtgp_cs_advancing(steps, t, tn) && (m->max_steps <= 0 || steps < m->max_steps)) {
    const float dt = tn - t;
    rhs(c, t, y, f0);
    if (euler) {
      for (int i = 0; i < n; ++i) y1[i] = y[i] + f0[i] * dt;
    } else {
      for (int i = 0; i < n; ++i) { acc[i] = mtgp_rk4_acc(0, 0.0f, f0[i]); f[i] = f0[i]; z[i] = 0.0f; }
      for (int st = 1; st <= 3; ++st) {
        for (int i = 0; i < n; ++i) {
          yi[i] = mtgp_rk4_in(st, y[i], f[i], z[i], dt);
          z[i] = mtgp_rk4_zero(st, z[i], f[i]);
        }
        rhs(c, mtgp_rk4_time(st, t, dt), yi, f);
        for (int i = 0; i < n; ++i) acc[i] = mtgp_rk4_acc(st, acc[i], f[i]);
      }
      for (int i = 0; i < n; ++i) y1[i] = mtgp_rk4_out(y[i], acc[i], dt);
    }
    ++steps;
    while (k < S && ts[k] <= tn) { /* SaveAt(ts) by the dense output */
      const float th = mtgp_cs_rescale(t, ts[k], tn);
      for (int i = 0; i < n; ++i)
        saved[(size_t)k * n + i] = euler ? mtgp_cs_linear(y[i], y1[i], th)
                                         : mtgp_cs_hermite(y[i], y1[i], f0[i] * dt, f[i] * dt, th);
      ++k;
    }
    for (int i = 0; i < n; ++i) y[i] = y1[i];
    t = tn;
    const float cur = cond_fn(m, y);
    if (prev > 0.0f && cur < 0.0f) break;
    prev = cur;
    tn = mtgp_cs_next_end(t, dt0, t_end);
  }
  for (; k < S; ++k)
    for (int i = 0; i < n; ++i) saved[(size_t)k * n + i] = mtgp_u2f(0x7f800000u);
  return steps;
}

/* the number of steps of the fixed-step grid (mtgp_cstep.h) from ts[0] to ts[S-1] */
int oracle_cs_steps(const float* ts, int S, float dt0) {
  const float t_end = ts[S - 1];
  float t = ts[0], tn = mtgp_cs_first_end(t, dt0, t_end);
  int steps = 0;
  while (t < t_end && mtgp_cs_advancing(steps, t, tn)) {
    ++steps;
    t = tn;
    tn = mtgp_cs_next_end(t, dt0, t_end);
  }
  return steps;
}

/* diffeqsolve(Dopri5(), t0=ts[0], t1=ts[-1], dt0=h, SaveAt(ts), PIDController(rtol, atol, dtmin,
 * dtmax), Event(cond_fn), max_steps, throw=False) -- diffrax restated in the fp32 spec of
 * include/mtgp_dopri5.h (see its header comment for every rule used below). */
/* one weighted stage sum: the spec's fma chain (mtgp_dp_term) or, OR_DP_ALT_SUM_LITERAL, separate
 * products and adds */
static float dp_sum(const float* w, const float (*f)[OR_MAX_S], int n_terms, int i, int literal) {
  float acc = 0.0f;
  int first = 1;
  for (int j = 0; j < n_terms; ++j) {
    if (!literal) { acc = mtgp_dp_term(acc, w[j], f[j][i], j == 0); continue; }
    const float p = w[j] * f[j][i];  /* (zero entries included, as the spec's chain) */
    acc = first ? p : acc + p;
    first = 0;
  }
  return acc;
}
static float dp_apply(float y, float h, float acc, int literal) { return literal ? y + acc * h : MTGP_FMAF(h, acc, y); }

static int solve_dopri5(const OrCtx* c, const float* ts, const float* s0, float* saved) {
  static const float A[7][6] = MTGP_DP_TABLE_A;
  static const float E[7] = MTGP_DP_TABLE_E;
  static const float CM[7] = MTGP_DP_TABLE_CMID;
  const OrModel* m = c->m;
  const int alt = m->dp_alt, lit = (alt & OR_DP_ALT_SUM_LITERAL) != 0;
  const int n = state_dim(m), S = m->n_save;
  const int n_err = (alt & OR_DP_ALT_NORM_X) && m->model != 3 ? m->n_var : n;
  const float t_end = ts[S - 1];
  float y[OR_MAX_S], f[7][OR_MAX_S], yi[OR_MAX_S], y1[OR_MAX_S];
  for (int i = 0; i < n; ++i) y[i] = s0[i];
  int k = 1, steps = 0, accepted = 0;
  if (alt & OR_DP_ALT_INTERP_T0) k = 0;
  else for (int i = 0; i < n; ++i) saved[i] = y[i];
  if (c->save_at) {
    for (int q = 0; q < S; ++q) c->save_at[q] = -1;
    if (k == 1) c->save_at[0] = 0;
  }
  float t = ts[0];
  float tnext = t + m->h;
  if (tnext > t_end) tnext = t_end;
  float prev = cond_fn(m, y);
  rhs(c, t, y, f[0]);
  const MtgpDpPid def_pid = MTGP_DP_PID_DEFAULT;
  MtgpDpPid pid = def_pid;
  if (m->pid_custom) {
    pid.c1 = m->pid_c1; pid.c2 = m->pid_c2; pid.c3 = m->pid_c3;
    pid.safety = m->pid_safety; pid.factormin = m->pid_factormin; pid.factormax = m->pid_factormax;
  }
  if (alt & OR_DP_ALT_EO6) pid.c1 = (float)(1.0 / 6.0);
  MtgpDpCtl ctl = {1.0f, 1.0f, 0};
  while (t < t_end && ((alt & OR_DP_ALT_MAXSTEPS_ACC) ? accepted : steps) < m->max_steps) {
    const float h = tnext - t;
    for (int st = 1; st <= 6; ++st) {
      for (int i = 0; i < n; ++i) {
        yi[i] = dp_apply(y[i], h, dp_sum(A[st], (const float (*)[OR_MAX_S])f, st, i, lit), lit);
        if (st == 6) y1[i] = yi[i];
      }
      rhs(c, (st == 6 && (alt & OR_DP_ALT_FSAL_T1)) ? tnext : t + mtgp_dp_c(st) * h, yi, f[st]);
    }
    float msum = 0.0f;
    for (int i = 0; i < n_err; ++i) {
      const float acc = dp_sum(E, (const float (*)[OR_MAX_S])f, 7, i, lit);
      const float sc = mtgp_dp_scaled(h * acc, y[i], y1[i], m->rtol, m->atol);
      msum = (i == 0) ? sc * sc : msum + sc * sc;
    }
    const float ms = msum / (float)n_err;
    int keep, fail;
    if (alt & OR_DP_ALT_DTMIN_ATTEMPT) ctl.at_dtmin = m->dtmin > 0.0f && h <= m->dtmin;
    const float dt = mtgp_dp_control(ms, h, m->dtmin, m->dtmax, !m->no_force_dtmin, &pid, &ctl, &keep, &fail);
    ++steps;
    int done = fail; /* dt_min_reached: the solve ends after this attempt */
    if (!keep && (alt & OR_DP_ALT_EVENT_ALL)) {
      if (prev > 0.0f && cond_fn(m, y1) < 0.0f) done = 1;
    }
    if (keep) {
      ++accepted;
      const float t1 = tnext;
      while (k < S && ts[k] <= t1) { /* SaveAt(ts) by the dense output */
        const float th = (ts[k] - t) / h;
        for (int i = 0; i < n; ++i) {
          const float ymid = dp_apply(y[i], h, dp_sum(CM, (const float (*)[OR_MAX_S])f, 7, i, lit), lit);
          saved[(size_t)k * n + i] = mtgp_dp_interp(y[i], y1[i], ymid, h * f[0][i], h * f[6][i], th);
        }
        if (c->save_at) c->save_at[k] = steps;
        ++k;
      }
      t = t1;
      for (int i = 0; i < n; ++i) {
        y[i] = y1[i];
        f[0][i] = f[6][i]; /* FSAL */
      }
      const float cur = cond_fn(m, y);
      if (prev > 0.0f && cur < 0.0f) done = 1;
      prev = cur;
    }
    if (done) break;
    tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
  }
  for (; k < S; ++k)
    for (int i = 0; i < n; ++i) saved[(size_t)k * n + i] = mtgp_u2f(0x7f800000u);
  return steps;
}

/* Acrobot.fitness_function (acrobot.py:77-84) on full arrays. */
static float acro_fitness(const float* xs, const float* us, const float* ts, int S) {
  int fs = 0, found = 0;
  for (int k = 0; k < S && !found; ++k) {
    const float t1 = xs[4 * k + 0], t2 = xs[4 * k + 1];
    const int reached = ((-mtgp_cosf(t1)) - mtgp_cosf(t1 + t2)) > 1.5f;
    if (reached) { fs = k; found = 1; }
  }
  const float dts = ts[1] - ts[0];
  float cs = 0.0f;
  for (int k = 0; k < S; ++k) {
    const float cost = (us[k] * 0.01f) * us[k];
    const float ratio = ts[k] / dts;
    const float masked = (ratio > (float)fs) ? 0.0f : cost;
    cs = cs + masked;
  }
  return (float)(fs + (fs == 0) * S) + cs;
}

/* HarmonicOscillator.fitness_function (harmonic_oscillator.py:71-77) on full arrays:
 * x_d = [target, 0], u_d = -pinv(b) @ A @ x_d with pinv(b) = [[0, 1]] taken exact (XLA's SVD
 * pinv of b is not restated: parity unpinned), costs (x - x_d)^T Q (x - x_d) + (u - u_d) R
 * (u - u_d) with Q = [[q, 0], [0, 0]], R = [[r]], q = r = 0.5; every matrix product is the
 * literal left-to-right index-order sum (zeros included), the sum over time sequential. */
static float quad_form(const float* e, const float* Q, int n) {
  float out = 0.0f;
  for (int j = 0; j < n; ++j) {
    float v = e[0] * Q[0 * n + j];
    for (int i = 1; i < n; ++i) v = v + e[i] * Q[i * n + j];
    out = (j == 0) ? v * e[0] : out + v * e[j];
  }
  return out;
}

static float ho_u_target(const float* prm, float tg) {
  const float A[2][2] = {{0.0f, 1.0f}, {-prm[0], -prm[1]}};
  const float nb[2] = {-0.0f, -1.0f}; /* -pinv(b) */
  const float M0 = nb[0] * A[0][0] + nb[1] * A[1][0], M1 = nb[0] * A[0][1] + nb[1] * A[1][1];
  return M0 * tg + M1 * 0.0f;
}

static float ho_fitness(const float* xs, const float* us, const float* prm, float tg, int S) {
  const float Q[4] = {0.5f, 0.0f, 0.0f, 0.0f}, r = 0.5f;
  const float ud = ho_u_target(prm, tg);
  float cs = 0.0f;
  for (int k = 0; k < S; ++k) {
    const float e[2] = {xs[2 * k + 0] - tg, xs[2 * k + 1] - 0.0f};
    const float du = us[k] - ud;
    cs = cs + (quad_form(e, Q, 2) + (du * r) * du);
  }
  return cs;
}

/* StirredTankReactor.fitness_function (reactor.py:73-78): x_d = [0, target, 0],
 * Q = diag(0, 0.01, 0) (full 3x3), r = [[0.0001]]. */
static float reactor_fitness(const float* xs, const float* us, float tg, int S) {
  const float Q[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.01f, 0.0f, 0.0f, 0.0f, 0.0f}, r = 0.0001f;
  float cs = 0.0f;
  for (int k = 0; k < S; ++k) {
    const float e[3] = {xs[3 * k + 0] - 0.0f, xs[3 * k + 1] - tg, xs[3 * k + 2] - 0.0f};
    cs = cs + (quad_form(e, Q, 3) + (us[k] * r) * us[k]);
  }
  return cs;
}

/* pairwise (xor-butterfly) sum over padded chunks of 64 -- the kernel's reduction order */
static float pairwise_sum(const float* v, int R) {
  const int nch = (R + 63) / 64;
  int np2 = 1;
  while (np2 < nch) np2 *= 2;
  float chunk[1024];
  for (int ch = 0; ch < np2; ++ch) {
    float lane[64];
    for (int l = 0; l < 64; ++l) {
      const int r = ch * 64 + l;
      lane[l] = (ch < nch && r < R) ? v[r] : 0.0f;
    }
    for (int w = 1; w < 64; w *= 2)
      for (int l = 0; l < 64; l += 2 * w) lane[l] = lane[l] + lane[l + w];
    chunk[ch] = lane[0];
  }
  for (int w = 1; w < np2; w *= 2)
    for (int ch = 0; ch < np2; ch += 2 * w) chunk[ch] = chunk[ch] + chunk[ch + w];
  return chunk[0];
}

/*
 * Evaluate P candidates (pop [P, T, N, 4]).  Outputs:
 *   fitness[P]; rollout_fitness[P, R] (raw, before NaN/inf replacement) or NULL;
 *   trajectories in the reference's evaluate_candidate layout, each nullable:
 *   xs[P, R, S, n_var], ys[P, R, S, n_obs], us[P, R, S, n_control], acts[P, R, S, state_size].
 */
int oracle_eval_ex(const OrModel* m, const float* pop, int P, int T, int N, int n_funcs, int var_start,
                   const int8_t* fn, const OrRollouts* ro, float* fitness, float* rollout_fitness, float* xs,
                   float* ys, float* us, float* acts, int32_t* steps_out);
int oracle_eval(const OrModel* m, const float* pop, int P, int T, int N, int n_funcs, int var_start,
                const int8_t* fn, const OrRollouts* ro, float* fitness, float* rollout_fitness, float* xs,
                float* ys, float* us, float* acts) {
  return oracle_eval_ex(m, pop, P, T, N, n_funcs, var_start, fn, ro, fitness, rollout_fitness, xs, ys, us, acts, NULL);
}

/* oracle_eval plus the solve's step count per rollout (steps_out [P, R] or NULL; Dopri5: attempts) */
int oracle_eval_ex(const OrModel* m, const float* pop, int P, int T, int N, int n_funcs, int var_start,
                   const int8_t* fn, const OrRollouts* ro, float* fitness, float* rollout_fitness, float* xs,
                   float* ys, float* us, float* acts, int32_t* steps_out) {
  if (N > OR_MAX_N || state_dim(m) > OR_MAX_S || ro->R > 65536) return -1;
  const int R = ro->R, S = m->n_save, dim = state_dim(m);
#pragma omp parallel for schedule(dynamic, 1)
  for (int p = 0; p < P; ++p) {
    OrCtx c = {0};
    c.m = m;
    c.cand = pop + (size_t)p * T * N * 4;
    c.N = N;
    c.lib.n_funcs = n_funcs;
    c.lib.var_start = var_start;
    c.lib.fn = fn;
    float* saved = (float*)malloc(sizeof(float) * (size_t)S * dim);
    float* uu = (float*)malloc(sizeof(float) * (size_t)S * 8);
    float* fr = (float*)malloc(sizeof(float) * (size_t)R);
    for (int r = 0; r < R; ++r) {
      c.target = ro->targets ? ro->targets + (size_t)r * m->n_targets : NULL;
      static const float ones[8] = {1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f};
      const int npar = m->env == ENV_HARMONIC ? 2 : (m->env == ENV_REACTOR ? 8 : 4);
      c.prm = ro->params ? ro->params + (size_t)r * npar : ones;
      float s0[OR_MAX_S];
      for (int i = 0; i < dim; ++i) s0[i] = 0.0f;
      for (int i = 0; i < m->n_var; ++i) s0[i] = ro->x0[(size_t)r * m->n_var + i];
      c.key = ro->obs_keys ? ro->obs_keys + 2 * (size_t)r : NULL;
      c.W = ro->obs_w;
      c.save_at = g_save_trace ? g_save_trace + ((size_t)p * R + r) * S : NULL;
      const int nst = m->solver == 1 ? solve_dopri5(&c, ro->ts, s0, saved) : solve_fixed(&c, ro->ts, s0, saved);
      if (steps_out) steps_out[(size_t)p * R + r] = nst;
      float f;
      const size_t base = ((size_t)p * R + r) * S;
      if (m->model == 3) {
        /* MSE: mean over time of sum over dims (sr.py:24) */
        float tot = 0.0f;
        for (int k = 0; k < S; ++k) {
          float sq = 0.0f;
          for (int d = 0; d < m->n_var; ++d) {
            const float e = saved[(size_t)k * dim + d] - ro->ys_true[((size_t)r * S + k) * m->n_var + d];
            sq = (d == 0) ? e * e : sq + e * e;
          }
          tot = tot + sq;
        }
        f = tot / (float)S;
        if (xs)
          for (int k = 0; k < S; ++k)
            for (int d = 0; d < m->n_var; ++d) xs[(base + k) * m->n_var + d] = saved[(size_t)k * dim + d];
      } else {
        /* observations at the saved points (lax.scan f_obs) and the readout/policy */
        const int nv = m->n_var;
        float yk[OR_MAX_D], data[OR_MAX_D];
        float xk[OR_MAX_D];
        for (int k = 0; k < S; ++k) {
          for (int i = 0; i < nv; ++i) xk[i] = saved[(size_t)k * dim + i];
          ctl_f_obs(&c, ro->ts[k], xk, yk); /* lax.scan(f_obs, key, (ts, xs)), dyn.py:99 */
          if (m->model == 1) { /* dyn.py:101: readout([y, a, 0_u, target]) */
            const int no = m->n_obs, na = m->state_size, nu = m->n_control, nt = m->n_targets;
            const int D = no + na + nu + nt;
            for (int i = 0; i < no; ++i) data[i] = yk[i];
            for (int i = 0; i < na; ++i) data[no + i] = saved[(size_t)k * dim + nv + i];
            for (int i = 0; i < nu; ++i) data[no + na + i] = 0.0f;
            for (int i = 0; i < nt; ++i) data[no + na + nu + i] = c.target[i];
            for (int j = 0; j < nu; ++j) uu[(size_t)k * 8 + j] = tree_eval(&c, na + j, data, D);
          } else { /* ff.py:97: policy([y, target]) */
            const int no = m->n_obs, nt = m->n_targets;
            for (int i = 0; i < no; ++i) data[i] = yk[i];
            for (int i = 0; i < nt; ++i) data[no + i] = c.target[i];
            uu[(size_t)k * 8] = tree_eval(&c, 0, data, no + nt);
          }
          if (xs) for (int i = 0; i < nv; ++i) xs[(base + k) * nv + i] = xk[i];
          if (ys) for (int i = 0; i < m->n_obs; ++i) ys[(base + k) * m->n_obs + i] = yk[i];
          if (us) for (int j = 0; j < m->n_control; ++j) us[(base + k) * m->n_control + j] = uu[(size_t)k * 8 + j];
          if (acts && m->model == 1)
            for (int i = 0; i < m->state_size; ++i)
              acts[(base + k) * m->state_size + i] = saved[(size_t)k * dim + nv + i];
        }
        /* the fitness functions use the first control only (n_control = 1) */
        float ucol[4096];
        float* up = (S <= 4096) ? ucol : (float*)malloc(sizeof(float) * S);
        float xcol[4 * 4096];
        float* xp = (S <= 4096) ? xcol : (float*)malloc(sizeof(float) * 4 * S);
        for (int k = 0; k < S; ++k) {
          up[k] = uu[(size_t)k * 8];
          for (int i = 0; i < nv; ++i) xp[nv * k + i] = saved[(size_t)k * dim + i];
        }
        if (m->env == ENV_HARMONIC) f = ho_fitness(xp, up, c.prm, c.target[0], S);
        else if (m->env == ENV_REACTOR) f = reactor_fitness(xp, up, c.target[0], S);
        else f = acro_fitness(xp, up, ro->ts, S);
        if (up != ucol) free(up);
        if (xp != xcol) free(xp);
      }
      if (rollout_fitness) rollout_fitness[(size_t)p * R + r] = f;
      /* dyn.py:49-50 / sr.py:42-43: NaN or inf -> max_fitness */
      fr[r] = mtgp_isfinite(f) ? f : m->max_fitness;
    }
    /* mean over rollouts, clip (dyn.py:51-52) */
    float mean = pairwise_sum(fr, R) / (float)R;
    if (mean < 0.0f) mean = 0.0f;
    if (mean > m->max_fitness) mean = m->max_fitness;
    /* parsimony on non-empty rows of all trees (gp.py:424) */
    int cnt = 0;
    for (int i = 0; i < T * N; ++i) cnt += (c.cand[4 * i] != 0.0f);
    fitness[p] = mean + m->parsimony * (float)cnt;
    free(saved);
    free(uu);
    free(fr);
  }
  return 0;
}

int oracle_abi_version(void) { return 1; }

/* vectorised helpers for tests */
void oracle_sincos(const float* x, float* s, float* c, long n) {
  for (long i = 0; i < n; ++i) { s[i] = mtgp_sinf(x[i]); c[i] = mtgp_cosf(x[i]); }
}
/* the unary tree operators by function code (FN_SIN .. FN_ABS) and their tangents (include/mtgp_dual.h) */
void oracle_unary(int fn, const float* x, const float* dx, float* y, float* dy, long n) {
  for (long i = 0; i < n; ++i) {
    const MtgpDual r = mtgp_dl_unary(fn, mtgp_dl(x[i], dx ? dx[i] : 0.0f));
    y[i] = r.v;
    if (dy) dy[i] = r.d;
  }
}
void oracle_wrap(const float* x, float* o, long n) {
  for (long i = 0; i < n; ++i) o[i] = mtgp_wrap_angle(x[i]);
}

/* unit-test hooks: Acrobot pieces in isolation */
void oracle_acro_drift(const float* params4, const float* state4, float u, float* out4) {
  OrCtx c = {0};
  memset(&c, 0, sizeof(c));
  c.prm = params4;
  acro_drift(&c, state4, u, out4);
}
void oracle_expf(const float* x, float* o, long n) {
  for (long i = 0; i < n; ++i) o[i] = mtgp_expf(x[i]);
}
void oracle_env_drift(int env, const float* params, const float* state, float u, float* out) {
  OrModel m;
  memset(&m, 0, sizeof(m));
  m.env = env;
  OrCtx c = {0};
  memset(&c, 0, sizeof(c));
  c.m = &m;
  c.prm = params;
  env_drift(&c, state, u, out);
}
float oracle_env_fitness(int env, const float* xs, const float* us, const float* ts, const float* params, float tg,
                         int S) {
  if (env == ENV_HARMONIC) return ho_fitness(xs, us, params, tg, S);
  if (env == ENV_REACTOR) return reactor_fitness(xs, us, tg, S);
  return acro_fitness(xs, us, ts, S);
}
void oracle_acro_f_obs(const float* x4, float* y4) {
  OrModel m;
  memset(&m, 0, sizeof(m));
  m.n_var = m.n_obs = 4;
  m.env = ENV_ACROBOT;
  OrCtx c = {0};
  memset(&c, 0, sizeof(c));
  c.m = &m;
  ctl_f_obs(&c, 0.0f, x4, y4);
}
/* PRNG spec hooks: normals of fold_in(key, bitcast(t)), normals of a key, threefry, erfinv, log1p */
void oracle_obs_normals(const uint32_t* key, float t, int n, int impl, float* out) {
  mtgp_obs_normals(key[0], key[1], t, n, impl, out);
}
void oracle_random_normals(const uint32_t* key, int n, int impl, float* out) {
  uint32_t bits[64];
  if (n > 64) n = 64;
  mtgp_random_bits(key[0], key[1], n, impl, bits);
  for (int i = 0; i < n; ++i) out[i] = mtgp_normal_from_bits(bits[i]);
}
void oracle_threefry(const uint32_t* key, const uint32_t* x0, const uint32_t* x1, uint32_t* y0, uint32_t* y1,
                     long n) {
  for (long i = 0; i < n; ++i) mtgp_threefry2x32(key[0], key[1], x0[i], x1[i], &y0[i], &y1[i]);
}
void oracle_erfinv(const float* x, float* o, long n) {
  for (long i = 0; i < n; ++i) o[i] = mtgp_erfinvf(x[i]);
}
void oracle_log1p(const float* x, float* o, long n) {
  for (long i = 0; i < n; ++i) o[i] = mtgp_log1pf(x[i]);
}
float oracle_acro_fitness(const float* xs, const float* us, const float* ts, int S) {
  return acro_fitness(xs, us, ts, S);
}
float oracle_pairwise_sum(const float* v, int R) { return pairwise_sum(v, R); }

/* ------------------------------------------------------------ coefficient optimisation
 * GeneticProgramming.epoch's value_and_grad (gp.py:435-452, vmap_gradients gp.py:253) of the SR
 * evaluator (sr.py:30-45) restated in forward mode: dual numbers (value, d/d theta) through the
 * row-order interpreter, the fixed-step solve and the MSE.  theta = the value column entry
 * tree[t][i][3] of one coefficient row; as in JAX, the entry is differentiated both where the
 * coefficient row selects it (gp.py:372) and where an earlier row reads the original column of a
 * later row (gp.py:366-369).  Reverse mode (JAX) and forward mode give the same derivative up to
 * rounding; this oracle fixes the forward-mode operation order the GPU kernel must reproduce. */
typedef struct {
  float v, d;
} ODual;

static ODual od(float v, float d) { ODual r; r.v = v; r.d = d; return r; }
static ODual od_add(ODual a, ODual b) { return od(a.v + b.v, a.d + b.d); }
static ODual od_sub(ODual a, ODual b) { return od(a.v - b.v, a.d - b.d); }
static ODual od_mul(ODual a, ODual b) { return od(a.v * b.v, a.d * b.v + a.v * b.d); }
static ODual od_div(ODual a, ODual b) { const float q = a.v / b.v; return od(q, (a.d - q * b.d) / b.v); }
static ODual od_sin(ODual a) { return od(mtgp_sinf(a.v), mtgp_cosf(a.v) * a.d); }
static ODual od_cos(ODual a) { return od(mtgp_cosf(a.v), -mtgp_sinf(a.v) * a.d); }

/* gp.py:356-388 in dual numbers; prow = the row of this tree holding theta (-1: none) */
static ODual tree_eval_dual(const float* tree, int N, const OrLib* lib, const ODual* data, int n_data, int prow) {
  ODual val[OR_MAX_N];
  for (int i = 0; i < N; ++i) val[i] = od(tree[4 * i + 3], i == prow ? 1.0f : 0.0f);
  for (int i = 0; i < N; ++i) {
    const float f = tree[4 * i + 0];
    const ODual x = val[or_index(tree[4 * i + 1], N)];
    const ODual y = val[or_index(tree[4 * i + 2], N)];
    ODual v;
    if (f == 1.0f) {
      v = od(tree[4 * i + 3], i == prow ? 1.0f : 0.0f);
    } else {
      int32_t k = or_f2i(f);
      if (k < 0) k = 0;
      if (k > lib->n_funcs - 1) k = lib->n_funcs - 1;
      switch (lib->fn[k]) {
        case FN_VAR: {
          int d = k - lib->var_start;
          if (d > n_data - 1) d = n_data - 1;
          v = data[d];
          break;
        }
        case FN_ADD: v = od_add(x, y); break;
        case FN_SUB: v = od_sub(x, y); break;
        case FN_MUL: v = od_mul(x, y); break;
        case FN_DIV: v = od_div(x, y); break;
        case FN_SIN: v = od_sin(x); break;
        case FN_COS: v = od_cos(x); break;
        case FN_EXP: case FN_LOG: case FN_SQRT: case FN_TANH: case FN_ABS: {
          const MtgpDual r = mtgp_dl_unary(lib->fn[k], mtgp_dl(x.v, x.d));  /* include/mtgp_dual.h */
          v = od(r.v, r.d);
          break;
        }
        default: v = od(0.0f, 0.0f); break;
      }
    }
    val[i] = v;
  }
  return val[N - 1];
}

/* solve_fixed in dual numbers: the value half is solve_fixed bit for bit, the tangent half applies
 * the same linear maps (stage sums, step update, the dense output at the primal theta) to the
 * tangents; the step grid and the event are primal.  The state has n = state_dim(m) components;
 * rhs(ctx, t, s, ds) is the model's dual RHS.  saved[k * n + i] for k < the returned count (the
 * first unsaved save index). */
typedef void (*OrDualRhs)(const void* ctx, float t, const ODual* s, ODual* ds);

static int fixed_dual(const OrModel* m, const float* ts, const ODual* s0, OrDualRhs rhs, const void* ctx,
                      ODual* saved) {
  const int n = state_dim(m), S = m->n_save, euler = m->solver == 2;
  const float t_end = ts[S - 1], dt0 = m->h;
  ODual y[OR_MAX_S], f0[OR_MAX_S], f[OR_MAX_S], acc[OR_MAX_S], yi[OR_MAX_S], y1[OR_MAX_S], zr[OR_MAX_S];
  float sv[OR_MAX_S];
  for (int i = 0; i < n; ++i) { y[i] = s0[i]; sv[i] = y[i].v; }
  float prev = cond_fn(m, sv);
  int k = 0, steps = 0;
  float t = ts[0], tn = mtgp_cs_first_end(t, dt0, t_end);
  while (t < t_end && mtgp_cs_advancing(steps, t, tn) && (m->max_steps <= 0 || steps < m->max_steps)) {
    const float dt = tn - t;
    rhs(ctx, t, y, f0);
    if (euler) {
      for (int i = 0; i < n; ++i) y1[i] = od(y[i].v + f0[i].v * dt, y[i].d + f0[i].d * dt);
    } else {
      for (int i = 0; i < n; ++i) {
        acc[i] = od(mtgp_rk4_acc(0, 0.0f, f0[i].v), mtgp_rk4_acc(0, 0.0f, f0[i].d));
        f[i] = f0[i];
        zr[i] = od(0.0f, 0.0f);
      }
      for (int st = 1; st <= 3; ++st) {
        for (int i = 0; i < n; ++i) {  /* (the tangent's zero entries: JAX's jvp of the dot product) */
          yi[i] = od(mtgp_rk4_in(st, y[i].v, f[i].v, zr[i].v, dt), mtgp_rk4_in(st, y[i].d, f[i].d, zr[i].d, dt));
          zr[i] = od(mtgp_rk4_zero(st, zr[i].v, f[i].v), mtgp_rk4_zero(st, zr[i].d, f[i].d));
        }
        rhs(ctx, mtgp_rk4_time(st, t, dt), yi, f);
        for (int i = 0; i < n; ++i) acc[i] = od(mtgp_rk4_acc(st, acc[i].v, f[i].v), mtgp_rk4_acc(st, acc[i].d, f[i].d));
      }
      for (int i = 0; i < n; ++i) y1[i] = od(mtgp_rk4_out(y[i].v, acc[i].v, dt), mtgp_rk4_out(y[i].d, acc[i].d, dt));
    }
    ++steps;
    while (k < S && ts[k] <= tn) {
      const float th = mtgp_cs_rescale(t, ts[k], tn);
      for (int i = 0; i < n; ++i)
        saved[(size_t)k * n + i] =
            euler ? od(mtgp_cs_linear(y[i].v, y1[i].v, th), mtgp_cs_linear(y[i].d, y1[i].d, th))
                  : od(mtgp_cs_hermite(y[i].v, y1[i].v, f0[i].v * dt, f[i].v * dt, th),
                       mtgp_cs_hermite(y[i].d, y1[i].d, f0[i].d * dt, f[i].d * dt, th));
      ++k;
    }
    for (int i = 0; i < n; ++i) { y[i] = y1[i]; sv[i] = y[i].v; }
    t = tn;
    const float cur = cond_fn(m, sv);
    if (prev > 0.0f && cur < 0.0f) break;
    prev = cur;
    tn = mtgp_cs_next_end(t, dt0, t_end);
  }
  return k;
}

typedef struct {
  const float* cand;
  int N, nv, pt, pi;
  const OrLib* lib;
} OrSrDualCtx;

/* sr.py:85-88 in duals */
static void sr_rhs_dual(const void* ctx, float t, const ODual* s, ODual* ds) {
  const OrSrDualCtx* c = (const OrSrDualCtx*)ctx;
  (void)t;
  for (int q = 0; q < c->nv; ++q)
    ds[q] = tree_eval_dual(c->cand + (size_t)q * c->N * 4, c->N, c->lib, s, c->nv, q == c->pt ? c->pi : -1);
}

/* one rollout of one candidate: F = MSE and dF/dtheta (theta at tree pt, row pi; pt < 0: none) --
 * the fixed-step solve (fixed_dual), the MSE of the saved points (sr.py:24) in duals */
static ODual sr_rollout_dual(const OrModel* m, const float* cand, int N, const OrLib* lib, const OrRollouts* ro, int r,
                             int pt, int pi) {
  const int nv = m->n_var, S = m->n_save;
  ODual s0[OR_MAX_S];
  for (int i = 0; i < nv; ++i) s0[i] = od(ro->x0[(size_t)r * nv + i], 0.0f);
  const OrSrDualCtx ctx = {cand, N, nv, pt, pi, lib};
  ODual* saved = (ODual*)malloc(sizeof(ODual) * (size_t)S * nv);
  const int ks = fixed_dual(m, ro->ts, s0, sr_rhs_dual, &ctx, saved);
  ODual tot = od(0.0f, 0.0f);
  for (int kk = 0; kk < ks; ++kk) {
    ODual sq = od(0.0f, 0.0f);
    for (int dd = 0; dd < nv; ++dd) {
      const ODual sv = saved[(size_t)kk * nv + dd];
      const float e = sv.v - ro->ys_true[((size_t)r * S + kk) * nv + dd];
      const float de = sv.d * (2.0f * e);
      sq = dd == 0 ? od(e * e, de) : od(sq.v + e * e, sq.d + de);
    }
    tot = od(tot.v + sq.v, tot.d + sq.d);
  }
  free(saved);
  /* points after the event are +inf: the squared error is +inf (NaN stays NaN) */
  if (ks < S && mtgp_isfinite(tot.v)) tot.v = mtgp_u2f(0x7f800000u);
  return od(tot.v / (float)S, tot.d / (float)S);
}

/* sr_rollout_dual for the adaptive solve: solve_dopri5 (include/mtgp_dopri5.h) in dual numbers
 * with the step sizes, the accept / reject decisions and the event held at their primal values --
 * the derivative of the discrete solution along the step sequence the solve took, which is what
 * jax.grad gives through diffrax's DirectAdjoint: diffrax's PIDController stops the gradient of the
 * initial step size (init) and of the step-size factor (adapt_step_size), so no step size carries
 * a tangent.  The value half is solve_dopri5 + the
 * evaluator's MSE of the saved points bit for bit; the tangent half applies the same linear maps
 * (stage fma chains, dense output at the primal theta) to the tangents. */
static ODual sr_rollout_dual_dp(const OrModel* m, const float* cand, int N, const OrLib* lib, const OrRollouts* ro,
                                int r, int pt, int pi) {
  static const float A[7][6] = MTGP_DP_TABLE_A;
  static const float E[7] = MTGP_DP_TABLE_E;
  static const float CM[7] = MTGP_DP_TABLE_CMID;
  const int nv = m->n_var, S = m->n_save;
  const float* ts = ro->ts;
  const float t_end = ts[S - 1];
  ODual y[OR_MAX_S], f[7][OR_MAX_S], yi[OR_MAX_S], y1[OR_MAX_S];
  float sv[OR_MAX_S];
  ODual tot = od(0.0f, 0.0f);
#define OR_DP_RHS(in, out)                                                                          \
  for (int q = 0; q < nv; ++q)                                                                      \
    out[q] = tree_eval_dual(cand + (size_t)q * N * 4, N, lib, in, nv, q == pt ? pi : -1);
#define OR_DP_MSE(kk, val)                                                                          \
  {                                                                                                 \
    ODual sq = od(0.0f, 0.0f);                                                                      \
    for (int dd = 0; dd < nv; ++dd) {                                                               \
      const float e = (val)[dd].v - ro->ys_true[((size_t)r * S + (kk)) * nv + dd];                  \
      const float de = (val)[dd].d * (2.0f * e);                                                    \
      sq = dd == 0 ? od(e * e, de) : od(sq.v + e * e, sq.d + de);                                   \
    }                                                                                               \
    tot = od(tot.v + sq.v, tot.d + sq.d);                                                           \
  }
  for (int i = 0; i < nv; ++i) y[i] = od(ro->x0[(size_t)r * nv + i], 0.0f);
  OR_DP_MSE(0, y)
  int k = 1, steps = 0;
  float t = ts[0];
  float tnext = t + m->h;
  if (tnext > t_end) tnext = t_end;
  for (int i = 0; i < nv; ++i) sv[i] = y[i].v;
  float prev = cond_fn(m, sv);
  OR_DP_RHS(y, f[0])
  const MtgpDpPid def_pid = MTGP_DP_PID_DEFAULT;
  MtgpDpPid pid = def_pid;
  if (m->pid_custom) {
    pid.c1 = m->pid_c1; pid.c2 = m->pid_c2; pid.c3 = m->pid_c3;
    pid.safety = m->pid_safety; pid.factormin = m->pid_factormin; pid.factormax = m->pid_factormax;
  }
  MtgpDpCtl ctl = {1.0f, 1.0f, 0};
  while (t < t_end && steps < m->max_steps) {
    const float h = tnext - t;
    for (int st = 1; st <= 6; ++st) {
      for (int i = 0; i < nv; ++i) {
        float acc = 0.0f, dacc = 0.0f;
        for (int j = 0; j < st; ++j) {
          acc = mtgp_dp_term(acc, A[st][j], f[j][i].v, j == 0);
          dacc = mtgp_dp_term(dacc, A[st][j], f[j][i].d, j == 0);
        }
        yi[i] = od(MTGP_FMAF(h, acc, y[i].v), MTGP_FMAF(h, dacc, y[i].d));
        if (st == 6) y1[i] = yi[i];
      }
      OR_DP_RHS(yi, f[st])
    }
    float msum = 0.0f;
    for (int i = 0; i < nv; ++i) {
      float acc = 0.0f;
      for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], f[j][i].v, j == 0);
      const float sc = mtgp_dp_scaled(h * acc, y[i].v, y1[i].v, m->rtol, m->atol);
      msum = (i == 0) ? sc * sc : msum + sc * sc;
    }
    const float ms = msum / (float)nv;
    int keep, fail;
    const float dt = mtgp_dp_control(ms, h, m->dtmin, m->dtmax, !m->no_force_dtmin, &pid, &ctl, &keep, &fail);
    ++steps;
    int done = fail;
    if (keep) {
      const float t1 = tnext;
      while (k < S && ts[k] <= t1) {
        const float th = (ts[k] - t) / h;
        ODual sk[OR_MAX_S];
        for (int i = 0; i < nv; ++i) {
          float acc = 0.0f, dacc = 0.0f;
          for (int j = 0; j < 7; ++j) {
            acc = mtgp_dp_term(acc, CM[j], f[j][i].v, j == 0);
            dacc = mtgp_dp_term(dacc, CM[j], f[j][i].d, j == 0);
          }
          const float ymid = MTGP_FMAF(h, acc, y[i].v), dymid = MTGP_FMAF(h, dacc, y[i].d);
          sk[i] = od(mtgp_dp_interp(y[i].v, y1[i].v, ymid, h * f[0][i].v, h * f[6][i].v, th),
                     mtgp_dp_interp(y[i].d, y1[i].d, dymid, h * f[0][i].d, h * f[6][i].d, th));
        }
        OR_DP_MSE(k, sk)
        ++k;
      }
      t = t1;
      for (int i = 0; i < nv; ++i) {
        y[i] = y1[i];
        f[0][i] = f[6][i];
        sv[i] = y[i].v;
      }
      const float cur = cond_fn(m, sv);
      if (prev > 0.0f && cur < 0.0f) done = 1;
      prev = cur;
    }
    if (done) break;
    tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
  }
#undef OR_DP_RHS
#undef OR_DP_MSE
  /* unsaved points are +inf: the squared error is +inf (NaN stays NaN) */
  if (k < S && mtgp_isfinite(tot.v)) tot.v = mtgp_u2f(0x7f800000u);
  return od(tot.v / (float)S, tot.d / (float)S);
}

/* loss[P] (the evaluator's fitness, no parsimony) and grad[P, K]: prow[P, K] = t * N + i of the
 * k-th coefficient row (-1 = unused).  SR: fixed-step RK4 / Euler, or Dopri5 + PID
 * (sr_rollout_dual_dp: step sizes held at their primal values). */
int oracle_sr_grad(const OrModel* m, const float* pop, int P, int T, int N, int n_funcs, int var_start,
                   const int8_t* fn, const OrRollouts* ro, const int32_t* prow, int K, float* loss, float* grad) {
  if (m->model != 3 || N > OR_MAX_N || m->n_var > OR_MAX_S || ro->R > 64 || K < 1) return -1;
  const int R = ro->R;
#pragma omp parallel for schedule(dynamic, 1)
  for (long pk = 0; pk < (long)P * K; ++pk) {
    const int p = (int)(pk / K), kq = (int)(pk % K);
    const int row = prow[(size_t)p * K + kq];
    if (row < 0 && kq > 0) { grad[pk] = 0.0f; continue; }
    OrLib lib;
    lib.n_funcs = n_funcs;
    lib.var_start = var_start;
    lib.fn = fn;
    const float* cand = pop + (size_t)p * T * N * 4;
    float v[64], dv[64];
    for (int r = 0; r < R; ++r) {
      const int pt = row < 0 ? -1 : row / N, pi = row < 0 ? -1 : row % N;
      ODual F = m->solver == 1 ? sr_rollout_dual_dp(m, cand, N, &lib, ro, r, pt, pi)
                               : sr_rollout_dual(m, cand, N, &lib, ro, r, pt, pi);
      if (!mtgp_isfinite(F.v)) F = od(m->max_fitness, 0.0f); /* sr.py:42-43, derivative of where */
      v[r] = F.v;
      dv[r] = F.d;
    }
    const float mean = pairwise_sum(v, R) / (float)R;
    float dmean = pairwise_sum(dv, R) / (float)R;
    /* jnp.clip = minimum(maximum(x, 0), max): JAX's max/min JVP is 1/2 on a tie */
    float c = mean;
    if (mean < 0.0f) { c = 0.0f; dmean = 0.0f; }
    else if (mean == 0.0f) dmean = 0.5f * dmean;
    if (c > m->max_fitness) { c = m->max_fitness; dmean = 0.0f; }
    else if (c == m->max_fitness) dmean = 0.5f * dmean;
    if (kq == 0) loss[p] = c;
    grad[pk] = row < 0 ? 0.0f : dmean;
  }
  return 0;
}

/* ------------------------------------------------------- coefficient optimisation, control
 * The same forward-mode derivative for the dynamic (dyn.py:37-118) and static (ff.py:36-110)
 * evaluators with a fixed-step solve: dual numbers through the row-order interpreter, f_obs
 * (C@x + noise, the Acrobot angle wrap), the environment drift (include/mtgp_dual.h, the spec of
 * the tangent rules), RK4 / Euler, the Event, the save-point readout and the fitness function
 * on the full saved arrays (acrobot.py:77-84 with first_success from the values -- argmax has no
 * derivative -- harmonic_oscillator.py:71-77, reactor.py:73-78).  theta = the value entry of
 * one coefficient row (tree pt, row pi), as in oracle_sr_grad. */
static MtgpDual o2d(ODual a) { return mtgp_dl(a.v, a.d); }
static ODual d2o(MtgpDual a) { return od(a.v, a.d); }

static void ctl_f_obs_dual(const OrCtx* c, float t, const ODual* x, ODual* y) {
  const int nv = c->m->n_var, no = c->m->n_obs;
  float nz[OR_MAX_D];
  if (c->key) {
    float n[OR_MAX_D];
    mtgp_obs_normals(c->key[0], c->key[1], t, no, c->m->prng_impl, n);
    for (int j = 0; j < no; ++j) {
      float s = n[0] * c->W[0 * no + j];
      for (int i = 1; i < no; ++i) s = s + n[i] * c->W[i * no + j];
      nz[j] = s;
    }
  } else {
    for (int j = 0; j < no; ++j) nz[j] = 0.0f;
  }
  for (int i = 0; i < no; ++i) {  /* C@x: the literal index-order sum, in duals */
    MtgpDual s = mtgp_dl_cmul(i == 0 ? 1.0f : 0.0f, o2d(x[0]));
    for (int j = 1; j < nv; ++j) s = mtgp_dl_add(s, mtgp_dl_cmul(i == j ? 1.0f : 0.0f, o2d(x[j])));
    y[i] = d2o(mtgp_dl_addc(s, nz[i]));
  }
  if (c->m->env == ENV_ACROBOT) {
    y[0] = d2o(mtgp_dl_wrap_angle(o2d(y[0])));
    if (no > 1) y[1] = d2o(mtgp_dl_wrap_angle(o2d(y[1])));
  }
}

static void env_drift_dual(const OrCtx* c, const ODual* x, ODual u, ODual* dx) {
  MtgpDual xx[OR_MAX_D], d[OR_MAX_D];
  const int nv = c->m->n_var;
  for (int i = 0; i < nv; ++i) xx[i] = o2d(x[i]);
  if (c->m->env == ENV_HARMONIC) mtgp_dl_ho_drift(c->prm, xx, o2d(u), d);
  else if (c->m->env == ENV_REACTOR) mtgp_dl_reactor_drift(c->prm, xx, o2d(u), d);
  else mtgp_dl_acro_drift(c->prm, xx, o2d(u), d);
  for (int i = 0; i < nv; ++i) dx[i] = d2o(d[i]);
}

/* the readout / policy tree j on a dual data vector */
static ODual ctl_tree_dual(const OrCtx* c, int t, const ODual* data, int n_data, int pt, int pi) {
  return tree_eval_dual(c->cand + (size_t)t * c->N * 4, c->N, &c->lib, data, n_data, t == pt ? pi : -1);
}

/* dyn.py:107-118 / ff.py:104-110 in duals */
static void ctl_rhs_dual(const OrCtx* c, float t, const ODual* s, ODual* ds, int pt, int pi) {
  const OrModel* m = c->m;
  const int no = m->n_obs, nt = m->n_targets, nv = m->n_var;
  ODual y[OR_MAX_D], data[OR_MAX_D];
  ctl_f_obs_dual(c, t, s, y);
  if (m->model == 1) {
    const int na = m->state_size, nu = m->n_control, D = no + na + nu + nt;
    for (int i = 0; i < D; ++i) data[i] = od(0.0f, 0.0f);
    for (int i = 0; i < na; ++i) data[no + i] = s[nv + i];
    for (int i = 0; i < nt; ++i) data[no + na + nu + i] = od(c->target[i], 0.0f);
    ODual u[8];
    for (int j = 0; j < nu; ++j) u[j] = ctl_tree_dual(c, na + j, data, D, pt, pi);  /* [0, a, 0, tg] */
    env_drift_dual(c, s, u[0], ds);
    for (int i = 0; i < no; ++i) data[i] = y[i];
    for (int j = 0; j < nu; ++j) data[no + na + j] = u[j];
    for (int i = 0; i < na; ++i) ds[nv + i] = ctl_tree_dual(c, i, data, D, pt, pi);  /* [y, a, u, tg] */
  } else {
    for (int i = 0; i < no; ++i) data[i] = y[i];
    for (int i = 0; i < nt; ++i) data[no + i] = od(c->target[i], 0.0f);
    const ODual u = ctl_tree_dual(c, 0, data, no + nt, pt, pi);
    env_drift_dual(c, s, u, ds);
  }
}

typedef struct {
  const OrCtx* c;
  int pt, pi;
} OrCtlDualCtx;
static void ctl_rhs_dual_cb(const void* ctx, float t, const ODual* s, ODual* ds) {
  const OrCtlDualCtx* x = (const OrCtlDualCtx*)ctx;
  ctl_rhs_dual(x->c, t, s, ds, x->pt, x->pi);
}

/* solve_dopri5 of the control models in dual numbers (the coupled [x, a] state, ctl_rhs_dual at
 * the stage times t + c_i h), the step sizes, accept / reject decisions and the event held at
 * their primal values (as sr_rollout_dual_dp): saved[0..k) the dense-output save points; returns
 * k, the first unsaved index. */
static int ctl_dopri5_dual(const OrCtx* c, const OrRollouts* ro, const ODual* s0, ODual* saved, int pt, int pi) {
  static const float A[7][6] = MTGP_DP_TABLE_A;
  static const float E[7] = MTGP_DP_TABLE_E;
  static const float CM[7] = MTGP_DP_TABLE_CMID;
  const OrModel* m = c->m;
  const int n = state_dim(m), S = m->n_save;
  const float* ts = ro->ts;
  const float t_end = ts[S - 1];
  ODual y[OR_MAX_S], f[7][OR_MAX_S], yi[OR_MAX_S], y1[OR_MAX_S];
  float sv[OR_MAX_S];
  for (int i = 0; i < n; ++i) { y[i] = s0[i]; saved[i] = y[i]; sv[i] = y[i].v; }
  int k = 1, steps = 0;
  float t = ts[0];
  float tnext = t + m->h;
  if (tnext > t_end) tnext = t_end;
  float prev = cond_fn(m, sv);
  ctl_rhs_dual(c, t, y, f[0], pt, pi);
  const MtgpDpPid def_pid = MTGP_DP_PID_DEFAULT;
  MtgpDpPid pid = def_pid;
  if (m->pid_custom) {
    pid.c1 = m->pid_c1; pid.c2 = m->pid_c2; pid.c3 = m->pid_c3;
    pid.safety = m->pid_safety; pid.factormin = m->pid_factormin; pid.factormax = m->pid_factormax;
  }
  MtgpDpCtl ctl = {1.0f, 1.0f, 0};
  while (t < t_end && steps < m->max_steps) {
    const float h = tnext - t;
    for (int st = 1; st <= 6; ++st) {
      for (int i = 0; i < n; ++i) {
        float acc = 0.0f, dacc = 0.0f;
        for (int j = 0; j < st; ++j) {
          acc = mtgp_dp_term(acc, A[st][j], f[j][i].v, j == 0);
          dacc = mtgp_dp_term(dacc, A[st][j], f[j][i].d, j == 0);
        }
        yi[i] = od(MTGP_FMAF(h, acc, y[i].v), MTGP_FMAF(h, dacc, y[i].d));
        if (st == 6) y1[i] = yi[i];
      }
      ctl_rhs_dual(c, t + mtgp_dp_c(st) * h, yi, f[st], pt, pi);
    }
    float msum = 0.0f;
    for (int i = 0; i < n; ++i) {
      float acc = 0.0f;
      for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], f[j][i].v, j == 0);
      const float sc = mtgp_dp_scaled(h * acc, y[i].v, y1[i].v, m->rtol, m->atol);
      msum = (i == 0) ? sc * sc : msum + sc * sc;
    }
    const float ms = msum / (float)n;
    int keep, fail;
    const float dt = mtgp_dp_control(ms, h, m->dtmin, m->dtmax, !m->no_force_dtmin, &pid, &ctl, &keep, &fail);
    ++steps;
    int done = fail;
    if (keep) {
      const float t1 = tnext;
      while (k < S && ts[k] <= t1) {
        const float th = (ts[k] - t) / h;
        for (int i = 0; i < n; ++i) {
          float acc = 0.0f, dacc = 0.0f;
          for (int j = 0; j < 7; ++j) {
            acc = mtgp_dp_term(acc, CM[j], f[j][i].v, j == 0);
            dacc = mtgp_dp_term(dacc, CM[j], f[j][i].d, j == 0);
          }
          const float ymid = MTGP_FMAF(h, acc, y[i].v), dymid = MTGP_FMAF(h, dacc, y[i].d);
          saved[(size_t)k * n + i] =
              od(mtgp_dp_interp(y[i].v, y1[i].v, ymid, h * f[0][i].v, h * f[6][i].v, th),
                 mtgp_dp_interp(y[i].d, y1[i].d, dymid, h * f[0][i].d, h * f[6][i].d, th));
        }
        ++k;
      }
      t = t1;
      for (int i = 0; i < n; ++i) {
        y[i] = y1[i];
        f[0][i] = f[6][i];
        sv[i] = y[i].v;
      }
      const float cur = cond_fn(m, sv);
      if (prev > 0.0f && cur < 0.0f) done = 1;
      prev = cur;
    }
    if (done) break;
    tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
  }
  return k;
}

/* one rollout: F and dF / d theta (the evaluator's rollout fitness, before NaN/inf replacement) */
static ODual ctl_rollout_dual(const OrCtx* c, const OrRollouts* ro, int r, int pt, int pi) {
  const OrModel* m = c->m;
  const int n = state_dim(m), nv = m->n_var, S = m->n_save;
  ODual* saved = (ODual*)malloc(sizeof(ODual) * (size_t)S * n);
  ODual s[OR_MAX_S];
  for (int i = 0; i < n; ++i) s[i] = od(i < nv ? ro->x0[(size_t)r * nv + i] : 0.0f, 0.0f);
  int ks;
  if (m->solver == 1) {
    for (int i = 0; i < n; ++i) saved[i] = s[i];
    ks = ctl_dopri5_dual(c, ro, s, saved, pt, pi);
  } else {
    const OrCtlDualCtx ctx = {c, pt, pi};
    ks = fixed_dual(m, ro->ts, s, ctl_rhs_dual_cb, &ctx, saved);
  }
  for (int q = ks; q < S; ++q)  /* the +inf fill after the event: constants, no tangent */
    for (int i = 0; i < n; ++i) saved[(size_t)q * n + i] = od(mtgp_u2f(0x7f800000u), 0.0f);
  /* controls at the save points (dyn.py:99-101 / ff.py:96-97) */
  ODual* us = (ODual*)malloc(sizeof(ODual) * (size_t)S);
  const int no = m->n_obs, nt = m->n_targets;
  for (int q = 0; q < S; ++q) {
    const ODual* xq = saved + (size_t)q * n;
    ODual y[OR_MAX_D], data[OR_MAX_D];
    ctl_f_obs_dual(c, ro->ts[q], xq, y);
    if (m->model == 1) {
      const int na = m->state_size, nu = m->n_control, D = no + na + nu + nt;
      for (int i = 0; i < no; ++i) data[i] = y[i];
      for (int i = 0; i < na; ++i) data[no + i] = xq[nv + i];
      for (int i = 0; i < nu; ++i) data[no + na + i] = od(0.0f, 0.0f);
      for (int i = 0; i < nt; ++i) data[no + na + nu + i] = od(c->target[i], 0.0f);
      us[q] = ctl_tree_dual(c, na, data, D, pt, pi);
    } else {
      for (int i = 0; i < no; ++i) data[i] = y[i];
      for (int i = 0; i < nt; ++i) data[no + i] = od(c->target[i], 0.0f);
      us[q] = ctl_tree_dual(c, 0, data, no + nt, pt, pi);
    }
  }
  MtgpDual F = mtgp_dl(0.0f, 0.0f);
  if (m->env == ENV_HARMONIC || m->env == ENV_REACTOR) {
    const float tg = c->target[0];
    for (int q = 0; q < S; ++q) {
      const ODual* xq = saved + (size_t)q * n;
      MtgpDual cost;
      if (m->env == ENV_HARMONIC) {
        const float Q[4] = {0.5f, 0.0f, 0.0f, 0.0f}, rr = 0.5f;
        const MtgpDual e[2] = {mtgp_dl_subc(o2d(xq[0]), tg), mtgp_dl_subc(o2d(xq[1]), 0.0f)};
        const MtgpDual du = mtgp_dl_subc(o2d(us[q]), ho_u_target(c->prm, tg));
        cost = mtgp_dl_add(mtgp_dl_quad_form(e, Q, 2), mtgp_dl_mul(mtgp_dl_mulc(du, rr), du));
      } else {
        const float Q[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.01f, 0.0f, 0.0f, 0.0f, 0.0f}, rr = 0.0001f;
        const MtgpDual e[3] = {mtgp_dl_subc(o2d(xq[0]), 0.0f), mtgp_dl_subc(o2d(xq[1]), tg),
                               mtgp_dl_subc(o2d(xq[2]), 0.0f)};
        cost = mtgp_dl_add(mtgp_dl_quad_form(e, Q, 3), mtgp_dl_mul(mtgp_dl_mulc(o2d(us[q]), rr), o2d(us[q])));
      }
      F = mtgp_dl_add(F, cost);
    }
  } else {  /* acrobot.py:77-84: first_success from the values, masked control costs in duals */
    int fs = 0;
    for (int q = 0; q < S; ++q) {
      const float a1 = saved[(size_t)q * n + 0].v, a2 = saved[(size_t)q * n + 1].v;
      if (((-mtgp_cosf(a1)) - mtgp_cosf(a1 + a2)) > 1.5f) { fs = q; break; }
    }
    const float dts = ro->ts[1] - ro->ts[0];
    MtgpDual cs = mtgp_dl(0.0f, 0.0f);
    for (int q = 0; q < S; ++q) {
      const MtgpDual u = o2d(us[q]);
      const MtgpDual cost = mtgp_dl_mul(mtgp_dl_mulc(u, 0.01f), u);
      const MtgpDual masked = ((ro->ts[q] / dts) > (float)fs) ? mtgp_dl(0.0f, 0.0f) : cost;
      cs = mtgp_dl_add(cs, masked);
    }
    F = mtgp_dl_cadd((float)(fs + (fs == 0) * S), cs);
  }
  free(saved);
  free(us);
  return d2o(F);
}

int oracle_ctl_grad(const OrModel* m, const float* pop, int P, int T, int N, int n_funcs, int var_start,
                    const int8_t* fn, const OrRollouts* ro, const int32_t* prow, int K, float* loss, float* grad) {
  if ((m->model != 1 && m->model != 2) || N > OR_MAX_N || state_dim(m) > OR_MAX_S ||
      ro->R > 64 || K < 1)
    return -1;
  const int R = ro->R;
#pragma omp parallel for schedule(dynamic, 1)
  for (long pk = 0; pk < (long)P * K; ++pk) {
    const int p = (int)(pk / K), kq = (int)(pk % K);
    const int row = prow[(size_t)p * K + kq];
    if (row < 0 && kq > 0) { grad[pk] = 0.0f; continue; }
    OrCtx c = {0};
    c.m = m;
    c.cand = pop + (size_t)p * T * N * 4;
    c.N = N;
    c.lib.n_funcs = n_funcs;
    c.lib.var_start = var_start;
    c.lib.fn = fn;
    c.W = ro->obs_w;
    float v[64], dv[64];
    for (int r = 0; r < R; ++r) {
      c.target = ro->targets ? ro->targets + (size_t)r * m->n_targets : NULL;
      static const float ones[8] = {1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f};
      const int npar = m->env == ENV_HARMONIC ? 2 : (m->env == ENV_REACTOR ? 8 : 4);
      c.prm = ro->params ? ro->params + (size_t)r * npar : ones;
      c.key = ro->obs_keys ? ro->obs_keys + 2 * (size_t)r : NULL;
      ODual F = ctl_rollout_dual(&c, ro, r, row < 0 ? -1 : row / N, row < 0 ? -1 : row % N);
      if (!mtgp_isfinite(F.v)) F = od(m->max_fitness, 0.0f); /* dyn.py:49-50, derivative of where */
      v[r] = F.v;
      dv[r] = F.d;
    }
    const float mean = pairwise_sum(v, R) / (float)R;
    float dmean = pairwise_sum(dv, R) / (float)R;
    float cl = mean;
    if (mean < 0.0f) { cl = 0.0f; dmean = 0.0f; }
    else if (mean == 0.0f) dmean = 0.5f * dmean;
    if (cl > m->max_fitness) { cl = m->max_fitness; dmean = 0.0f; }
    else if (cl == m->max_fitness) dmean = 0.5f * dmean;
    if (kq == 0) loss[p] = cl;
    grad[pk] = row < 0 ? 0.0f : dmean;
  }
  return 0;
}
