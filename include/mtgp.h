/*
 * mtgp.h -- C ABI of the MI355X population-fitness evaluator for MultiTreeGP.
 *
 * Drop-in boundary.  The reference has no FFI: its hot path is the
 * Python call chain
 *     GeneticProgramming.evaluate_population(populations, data)      gp.py:403-433
 *       -> jit(shard_map(shard_eval))                                gp.py:259-269
 *         -> vmap(fitness_function.__call__(coeffs, nodes, data, tree_evaluator))
 *              dynamic_evaluate.py:37-118 / feedforward_evaluate.py:36-110 /
 *              SR_evaluator.py:30-94
 *           -> tree_evaluator = vmap_foriloop / foriloop / body_fun  gp.py:356-401
 * These entry points are what a ctypes / cffi binding of that chain needs:
 *     mtgp_flatten   replaces the per-call tree walk of body_fun/foriloop (gp.py:356-388):
 *                    it turns the [P,T,N,4] population into straight-line programs once
 *                    per generation;
 *     mtgp_eval_rk4  replaces shard_eval's vmap over individuals x rollouts of
 *                    diffeqsolve(ODETerm(_drift)) + fitness post-processing
 *                    (dyn.py:49-52, gp.py:424) with one HIP kernel launch.
 * All pointers inside the descriptor structs are DEVICE pointers owned by the caller.
 * Calls are stream-ordered and asynchronous; nothing allocates or synchronises, so a
 * caller may capture them into a hipGraph.  Errors are returned as MTGP_ERR_* codes,
 * never thrown; per-tree flatten failures land in status_out (device).
 */
#ifndef MTGP_H
#define MTGP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTGP_ABI_VERSION 20

/* ---------------------------------------------------------------- limits */
#define MTGP_MAX_FUNCS 128   /* node functions 2 + K + V (gp.py:135-199)       */
#define MTGP_MAX_NODES 256   /* max_nodes N per tree (gp.py:69)                */
#define MTGP_MAX_DATA 64     /* data-vector length D seen by a tree            */
#define MTGP_MAX_PROGRAMS 64 /* programs per individual (mtgp_schedule weights) */
#define MTGP_STACK_MAX 8     /* operand-stack slots per lane (Sethi-Ullman)    */
#define MTGP_MAX_ROLLOUTS 65536 /* rollouts R per individual (dyn.py:63 vmaps any batch) */

/* ---------------------------------------------------------------- errors */
#define MTGP_OK 0
#define MTGP_ERR_ARG -1          /* bad size / null pointer / unsupported combination */
#define MTGP_ERR_LAUNCH -2       /* hipLaunchKernel failed                             */
#define MTGP_ERR_PROG_TOO_LONG 3 /* status_out: program longer than L                  */
#define MTGP_ERR_STACK 4         /* status_out: operand stack deeper than MTGP_STACK_MAX */

/* ---------------------------------------------- node library (gp.py:132-199) */
/* Function code of every opcode of the reference's node library.  Opcode 0 is the
 * empty node (value 0.0), opcode 1 the coefficient (value column when f == 1.0 exactly,
 * gp.py:372; otherwise lambda -> 0.0, gp.py:135), operators follow in operator_list
 * order, variables in first-appearance order (gp.py:143-180). */
enum {
  MTGP_FN_ZERO = 0, /* opcode 0 / 1 through the switch: 0.0                       */
  MTGP_FN_VAR = 1,  /* lambda_leaf(opcode - var_start)             gp.py:30-31    */
  MTGP_FN_ADD = 2,  /* "+"  (x, y) -> x + y                        gp.py:27-28    */
  MTGP_FN_SUB = 3,  /* "-"  x - y                                                  */
  MTGP_FN_MUL = 4,  /* "*"  x * y                                                  */
  MTGP_FN_DIV = 5,  /* "/"  x / y   (IEEE, unprotected: SymbolicRegression.ipynb)  */
  MTGP_FN_SIN = 6,  /* "sin" f(x)                                  gp.py:24-25    */
  MTGP_FN_COS = 7,  /* "cos"                                                       */
  /* round 3: further unary operators a reference operator_list may name (gp.py:143-162
   * accepts any lambda; these follow jnp.exp / log / sqrt / tanh / abs in f32, specs in
   * mtgp_f32math.h).  Since round 4 the program JIT translates them too (shared machine-code
   * subroutines for exp / log / tanh / sqrt, abs inline), bit-identical to the interpreter. */
  MTGP_FN_EXP = 8,  /* "exp"  mtgp_expf                                            */
  MTGP_FN_LOG = 9,  /* "log"  mtgp_logf  (x < 0: NaN, 0: -inf)                     */
  MTGP_FN_SQRT = 10, /* "sqrt" IEEE sqrt (correctly rounded; x < 0: NaN)           */
  MTGP_FN_TANH = 11, /* "tanh" mtgp_tanhf                                          */
  MTGP_FN_ABS = 12   /* "abs"  |x| (sign bit cleared)                              */
};
/* unary function codes: SIN .. ABS except the binary ones */
#define MTGP_FN_IS_UNARY(fn) ((fn) == MTGP_FN_SIN || (fn) == MTGP_FN_COS || ((fn) >= MTGP_FN_EXP && (fn) <= MTGP_FN_ABS))

typedef struct {
  int32_t n_funcs;   /* 2 + K + V: lax.switch branch count (index is clamped)       */
  int32_t var_start; /* first variable opcode = 2 + K                               */
  int8_t fn[MTGP_MAX_FUNCS];
} MtgpNodeLibrary;

/* One straight-line program to emit per individual: which tree, how long the data
 * vector is, and which data slots are known to hold +0.0 (e.g. the readout during the
 * ODE solve sees zeros for y and u, dyn.py:113).  ABI v16: the evaluator's data slot s (after
 * the reference's clamp to n_data - 1, and after the zero_mask test) is placed at slot
 * s + gap when s >= gap_at (gap 0: identity) -- the control kernels keep n_var observation
 * slots, so with n_obs < n_var (C = eye(n_var)[:n_obs], control_environment_base.py:47) the
 * slots after the observations move up by n_var - n_obs. */
typedef struct {
  int32_t tree;
  int32_t n_data;
  uint64_t zero_mask;
  int32_t gap_at;
  int32_t gap;
} MtgpProgramSpec;

/* ------------------------------------------------------------ program format */
/* Accumulator machine, postorder with leaves folded into their parent, adjacent leaf
 * load + leaf operation fused into one superinstruction.
 *   op : opcode << MTGP_OP_SHIFT | aux.  aux (24 bits) = the second operand of the fused
 *        forms: VC*_f / SINV / COSV: aux = slot of V;  VV*_f: aux = slot of the right operand.
 *   imm: C forms and VC*: the f32 constant; V forms, VV* (left operand), SINV/COSV: the data
 *        slot as a u32.
 * Slots are stored as byte offsets slot * MTGP_SLOT_BYTES (the evaluator's LDS column stride),
 * so a handler addresses its operand without decoding.  Every program ends with MTGP_OP_END
 * (not counted in its length), so a program slot holds at most L - 1 instructions.  The program
 * stride L must be a multiple of 4: the evaluators fetch four instructions per scalar load.
 * Opcode values come from scripts/gen_opcodes.py (a frequency-shaped dispatch tree). */
#define MTGP_SLOT_BYTES 256u
#include "mtgp_opcodes.h"
typedef struct {
  uint32_t op;
  float imm;
} MtgpInstr;

/* -------------------------------------------------------------- the models */
enum {
  MTGP_MODEL_ACROBOT_DYNAMIC = 1, /* dynamic_evaluate.Evaluator + Acrobot  dyn.py:10-118 */
  MTGP_MODEL_ACROBOT_STATIC = 2,  /* feedforward_evaluate.Evaluator + Acrobot ff.py:10-110 */
  MTGP_MODEL_SR = 3               /* SR_evaluator.Evaluator             sr.py:9-94       */
};
/* The two control models run any of these environments (MtgpModel.env); the enum names above
 * keep their round-1 spelling: MTGP_MODEL_ACROBOT_DYNAMIC is the dynamic evaluator, whatever
 * the environment. */
#define MTGP_MODEL_DYNAMIC MTGP_MODEL_ACROBOT_DYNAMIC
#define MTGP_MODEL_STATIC MTGP_MODEL_ACROBOT_STATIC
enum {
  MTGP_ENV_ACROBOT = 0,              /* acrobot.py:7-87:  n_var 4, n_obs 4, params [R, 4] l1 l2 m1 m2 */
  MTGP_ENV_HARMONIC_OSCILLATOR = 1,  /* harmonic_oscillator.py:8-80: n_var 2, n_obs 2, n_targets 1,  */
                                     /*   params [R, 2] omega zeta                                     */
  MTGP_ENV_STIRRED_TANK_REACTOR = 2  /* reactor.py:7-81: n_var 3, n_obs 3, n_targets 1,              */
                                     /*   params [R, 8] Vol Cp dHr UA q Tf Tcf Volc                    */
};

typedef struct {
  int32_t model;
  int32_t n_var;      /* latent env state (Acrobot 4) / SR state dims            */
  int32_t state_size; /* dynamic: hidden-state trees (dyn.py:83)                 */
  int32_t n_obs;      /* Acrobot: 4                                              */
  int32_t n_control;  /* Acrobot: 1                                              */
  int32_t n_targets;  /* Acrobot: 0                                              */
  int32_t n_steps;    /* informational (ABI v18): steps of the fixed-step grid    */
  int32_t save_every; /* ignored since ABI v18 (kept for the struct layout)       */
  int32_t n_save;     /* len(ts)                                                 */
  float h;            /* dt0                                                      */
  float max_fitness;  /* 1e4 control (dyn.py:27, ff.py:27), 1e5 SR (sr.py:22)    */
  float parsimony;    /* size_parsinomy (gp.py:424)                               */
  /* program slots in the flattened table (MtgpProgramSpec order), -1 if unused   */
  int32_t prog_state;        /* first of state_size (dynamic) / n_var (SR) trees   */
  int32_t prog_readout;      /* readout / policy during the solve                  */
  int32_t prog_readout_save; /* readout at the save points (dyn.py:101)            */
  int32_t readout_save_same; /* 1: equal to prog_readout, 0: differ, -1: compare  */
  int32_t prng_impl;         /* observation-noise random-bits layout (mtgp_prng.h): */
                             /* 0 threefry original (JAX <= 0.4.x default),        */
                             /* 1 threefry partitionable (JAX >= 0.5 default)      */
  int32_t env;               /* control models: MTGP_ENV_* (0 = Acrobot)            */
  /* Solver.  MTGP_SOLVER_RK4 (BASELINE) and MTGP_SOLVER_EULER (ABI v10; diffrax.Euler, the
   * reference evaluators' default, dyn.py:11, ff.py:11, sr.py:21) run diffrax.ConstantStepSize
   * from dt0 = h over [ts[0], ts[-1]] (ABI v18, include/mtgp_cstep.h): f32 step ends accumulated
   * t += dt0 with diffrax's end clip, each step over dt = tn - t, SaveAt(ts) for ANY non-decreasing
   * ts through the solver's dense output (RK4: cubic Hermite, Euler: linear), at most max_steps
   * steps (0: no limit) -- the unsaved points are then +inf (throw=False).
   * MTGP_SOLVER_DOPRI5: diffrax.Dopri5 + PIDController(rtol, atol, dtmin, dtmax) from dt0 = h
   * with SaveAt(ts) and at most max_steps step attempts (include/mtgp_dopri5.h, the notebooks'
   * setting, e.g. SymbolicRegression.ipynb:136); n_steps / save_every are ignored.  Implemented
   * for the dynamic and static control models (every MTGP_ENV_*) and for MTGP_MODEL_SR at every
   * n_var (register-resident for n_var <= 4, the wide-state workgroup kernel up to 64). */
  int32_t solver;
  int32_t max_steps; /* steps before the solve gives up (Dopri5: accepted + rejected; 0 = no limit
                        for the fixed-step solvers)                                        */
  float rtol, atol;  /* PIDController tolerances                                         */
  float dtmin;       /* <= 0: None; else force_dtmin: steps at dtmin are always accepted */
  float dtmax;       /* <= 0: None                                                       */
  /* ABI v15: a general PIDController (mtgp_dopri5.h mtgp_dp_factor_pid).  pid_custom == 0 (a
   * zero-initialised struct): diffrax's defaults (pcoeff 0, icoeff 1, dcoeff 0, safety 0.9,
   * factormin 0.2, factormax 10).  Otherwise pid_c1 = (icoeff + pcoeff + dcoeff) / 5,
   * pid_c2 = -(pcoeff + 2 dcoeff) / 5, pid_c3 = dcoeff / 5 (error order 5), rounded to f32. */
  int32_t pid_custom;
  float pid_c1, pid_c2, pid_c3, pid_safety, pid_factormin, pid_factormax;
  int32_t no_force_dtmin; /* 1: force_dtmin=False -- dt < dtmin ends the solve (dt_min_reached) */
  /* ABI v16: Dopri5 control models in two launches.  dp_budget > 0: launch 1 runs every wave for at
   * most dp_budget step attempts and parks the waves that are not done in MtgpOutputs.dp_state /
   * dp_pending; launch 2 resumes only those (a wave runs until its slowest lane is done, so the
   * few long solves otherwise hold whole waves and SIMDs).  Results are identical either way.
   * 0: one launch. */
  int32_t dp_budget;
} MtgpModel;
enum { MTGP_SOLVER_RK4 = 0, MTGP_SOLVER_DOPRI5 = 1, MTGP_SOLVER_EULER = 2 };

typedef struct {
  const float* x0;      /* [R, n_var]                                       */
  const float* params;  /* [R, n_params] per MTGP_ENV_* (Acrobot: l1 l2 m1 m2) */
  const float* targets; /* [R, n_targets] (may be NULL when n_targets == 0)  */
  const float* ts;      /* [n_save] save times (fitness mask acrobot.py:82)  */
  const float* ys_true; /* SR: [n_save, n_var, R] ground truth, time-major   */
  int32_t R;
  const int32_t* order; /* optional [P] evaluation schedule: a permutation of  */
                        /* [0, P) from mtgp_schedule (NULL = identity).  Only   */
                        /* which individuals share a wave changes; results are  */
                        /* bit-identical and stay indexed by individual.        */
  /* Observation noise (control models, control_environment_base.py:43-48):      */
  /*   y = C@x + normal(fold_in(obs_keys[r], bitcast(t)), (n_obs,)) @ obs_w       */
  /* at every stage time t + c_i*dt of the solve and at every save time ts[k].     */
  const uint32_t* obs_keys; /* [R, 2] obs_noise_keys (dyn.py:65) or NULL = noise-free */
  const float* obs_w;       /* [n_obs, n_obs] W (acrobot.py:49: obs_noise * I;          */
                            /*  reactor.py:43: obs_noise * I * [15, 15, 0.1])          */
  /* ABI v16: lanes per individual (a lane set), a power of two >= R, or 0 = R rounded up to a
   * power of two.  lanes <= 64: a wave holds 64 / lanes individuals (a wider set than R puts
   * fewer individuals in each wave -- more waves, fewer program calls per wave; mtgp_schedule
   * and the mtgp_jit_* functions must then be given lanes in place of R).  lanes > 64 (R > 64):
   * every individual spans lanes / 64 waves, wave w running rollouts [64 w, 64 w + 64), and the
   * fitness mean is formed by a second small kernel from MtgpOutputs.rollout_fitness, which is
   * then required. */
  int32_t lanes;
  /* ABI v17, Acrobot only: the fitness mask `ts / (ts[1] - ts[0]) > first_success` (acrobot.py:82)
   * as a count table, fit_kof[f] = #{k : f32(ts[k] / (ts[1] - ts[0])) <= (float)f} for f in [0, S)
   * (the mask keeps a prefix of the save points when the ratio is non-decreasing).  NULL: the ratio
   * of save k lies in (k - 1, k + 1] for every k (ts starting at 0 on a uniform grid), which the
   * kernels' one-pass fitness assumes.  Given, the kernels keep the running cost prefix and settle
   * each rollout at prefix fit_kof[first_success]; MtgpOutputs.fit_hist is then required when some
   * f in [1, S) has 1 <= fit_kof[f] <= f (the prefix lies behind the first success). */
  const int32_t* fit_kof;
} MtgpRollouts;

/* Outputs.  Trajectories are time-major structure-of-arrays so that every save point
 * is one coalesced 256-B store per wave: xs[(k*n_var + c)*P*R + p*R + r]. */
typedef struct {
  float* fitness;         /* [P] final fitness incl. parsimony (required)     */
  float* rollout_fitness; /* [P, R] raw per-rollout fitness or NULL (required when R > 64) */
  float* xs;              /* [n_save, n_var, P*R] or NULL                     */
  float* ys;              /* [n_save, n_obs, P*R] or NULL (control models)    */
  float* us;              /* [n_save, n_control, P*R] or NULL                 */
  float* acts;            /* [n_save, state_size, P*R] or NULL (dynamic)      */
  int32_t* steps;         /* [P, R] Dopri5 step attempts (accepted + rejected) or NULL (ABI v9; */
                          /* the fixed-step RK4 kernels leave it untouched)                      */
  /* ABI v16, required when MtgpModel.dp_budget > 0 (scratch, contents undefined afterwards):   */
  float* dp_state;        /* [MTGP_DP_STATE_WORDS, waves * 64] f32, waves = mtgp_eval_waves()   */
  int32_t* dp_pending;    /* [1 + waves] int32                                                  */
  /* ABI v17 (scratch): [n_save, P*R] f32 running cost prefixes of the general Acrobot mask, or NULL */
  /* (see MtgpRollouts.fit_kof)                                                                     */
  float* fit_hist;
  /* ABI v20: trajectory layout.  MTGP_TRAJ_TIME_MAJOR (0): the rows above.  MTGP_TRAJ_LANE_MAJOR */
  /* (1): xs[((p*R + r)*n_save + k)*n_var + c] (ys / us / acts likewise) -- the reference's       */
  /* [P, R, S, c] order; adaptive (MTGP_SOLVER_DOPRI5) solves only, MTGP_ERR_ARG otherwise: their */
  /* save points are divergent, and lane-contiguous rows halve the write traffic.     */
  int32_t traj_layout;
} MtgpOutputs;
#define MTGP_TRAJ_TIME_MAJOR 0
#define MTGP_TRAJ_LANE_MAJOR 1
#define MTGP_DP_STATE_WORDS 32

/* ------------------------------------------------------------- entry points */
int mtgp_abi_version(void);

/* Build provenance (round 6): copies "sources_sha256=<hex>;..." -- the SHA-256 of the sources,
 * flags and defines the library was compiled from (__graft_entry__.sources_hash) -- into out
 * (NUL-terminated, truncated to cap - 1 bytes) and returns the full length. */
int mtgp_build_info(char* out, int32_t cap);

/* Flatten a device population f32 [P, T, N, 4] (gp.py:412 layout) into programs
 * prog_out[P, n_prog, L], lengths len_out[P, n_prog], node counts nodes_out[P]
 * (non-empty rows, gp.py:424) and per-program status_out[P, n_prog].  nodes_out is zeroed
 * by mtgp_flatten itself (stream-ordered memset) before the kernel accumulates into it. */
int mtgp_flatten(const float* population, int32_t P, int32_t T, int32_t N,
                 const MtgpNodeLibrary* lib, const MtgpProgramSpec* specs, int32_t n_prog,
                 int32_t L, MtgpInstr* prog_out, int32_t* len_out, int32_t* nodes_out,
                 int32_t* status_out, void* stream);

/* mtgp_flatten plus the per-program sizing of the program JIT (ABI v12), so the JIT build needs no
 * translation pass of its own: jit_words_out[P, n_prog] = code words of the program's
 * fall-through translation (mtgp_jit.h jit_program; < 0: untranslatable) and jit_cost_out[P,
 * n_prog] = the schedule weight mtgp_jit_cost would compute.  Either may be NULL.  jit_mode:
 * MTGP_JIT_MODE_REGS (data vector in v0-v7: control models with state_size <= 3, SR n_var <= 4) or
 * MTGP_JIT_MODE_LDS (data vector in LDS: the wide-state SR kernel, n_var 5..64, and -- round 6 --
 * the dynamic policy with state_size 4..16 under the fixed-step solvers).  population
 * must be 16-byte aligned (rows are loaded as 16-byte vectors). */
enum { MTGP_JIT_MODE_REGS = 0, MTGP_JIT_MODE_LDS = 1 };
int mtgp_flatten_ex(const float* population, int32_t P, int32_t T, int32_t N,
                    const MtgpNodeLibrary* lib, const MtgpProgramSpec* specs, int32_t n_prog,
                    int32_t L, MtgpInstr* prog_out, int32_t* len_out, int32_t* nodes_out,
                    int32_t* status_out, int32_t* jit_words_out, int32_t* jit_cost_out,
                    int32_t jit_mode, void* stream);

/* Same algorithm on the host (one tree), for tests and tooling. Returns program length
 * or a negative MTGP_ERR_* / -MTGP_ERR_PROG_TOO_LONG / -MTGP_ERR_STACK. */
int mtgp_flatten_tree_host(const float* tree, int32_t N, const MtgpNodeLibrary* lib,
                           int32_t n_data, uint64_t zero_mask, int32_t L, MtgpInstr* out,
                           int32_t* stack_need);

/* The tree_evaluator plugin (GeneticProgramming.vmap_foriloop, gp.py:390-401) batched:
 * every flattened program evaluated on M data vectors data[M, n_data] (shared by all
 * individuals) -> out[P, n_prog, M]. */
int mtgp_eval_programs(const MtgpInstr* prog, const int32_t* plen, int32_t n_prog, int32_t L,
                       int32_t P, const float* data, int32_t M, int32_t n_data, float* out,
                       void* stream);

/* Evaluation schedule (load balance).  A wave packs G = 64 / pow2ceil(R) individuals and
 * interprets their programs one after another, so its cost follows the sum of their program
 * lengths; all waves are resident at once, so the kernel takes as long as its slowest SIMD.
 * mtgp_schedule sorts individuals by cost = sum_j weights[j] * plen[p, j] (counting sort,
 * costs clamped to MTGP_SCHED_BINS - 1) and writes order_out[P] pairing the most expensive
 * with the cheapest (G >= 2), or most expensive first (G == 1).  weights: host array
 * [n_prog] (e.g. how often each program runs per step).  scratch: device int32
 * [MTGP_SCHED_SCRATCH].  Ties are ordered arbitrarily; results do not depend on the order.
 * (No reference counterpart: this is GPU scheduling.) */
#define MTGP_SCHED_BINS 4096
#define MTGP_SCHED_SCRATCH (2 * MTGP_SCHED_BINS)
int mtgp_schedule(const int32_t* plen, int32_t P, int32_t n_prog, const int32_t* weights, int32_t R,
                  int32_t* order_out, int32_t* scratch, void* stream);

/* Integrate every (individual, rollout) with fixed-step RK4 and reduce fitness. */
/* Waves of the evaluator launch for P individuals with lane set `lanes` (MtgpRollouts.lanes, or
 * the rollout count R when lanes == 0): sizes MtgpOutputs.dp_state / dp_pending. */
int mtgp_eval_waves(int32_t P, int32_t R, int32_t lanes);

int mtgp_eval_rk4(const MtgpModel* model, const MtgpInstr* prog, const int32_t* plen,
                  int32_t n_prog, int32_t L, const int32_t* nodes, int32_t P,
                  const MtgpRollouts* rollouts, const MtgpOutputs* out, void* stream);

/* ------------------------------------------------------------- program JIT */
/* The programs of a flattened population are fixed for a whole evaluation (every RK4 stage
 * of every rollout runs them), so they can be translated once into gfx950 machine code that
 * the evaluator calls directly instead of interpreting (multitreegp_amd/csrc/mtgp_jit.h; no
 * reference counterpart -- this replaces XLA's compile of the vmapped tree evaluator).
 * Code is emitted per (wave, program) unit: the code the evaluator calls to run program j for
 * all G = 64 / pow2ceil(R) individuals packed in one wave, so it depends on R and on the
 * schedule (order) the evaluation will use.
 * Results are bit-identical to the interpreter.  Usage per flattened population + schedule:
 *   mtgp_jit_units  -> number of units U = ceil(P / G) * n_prog
 *   mtgp_jit_plan   -> offsets[U + 1] (byte offset of each unit's code, last = total) and
 *                      info[2] = {0 or a negative code if some program cannot be translated
 *                      (data slot >= 8), total bytes}   (device, stream-ordered)
 *   (host sizes an executable buffer from mtgp_jit_alloc -- from info, or from an
 *    estimate when info is passed on to the evaluator, which then checks it on the device)
 *   mtgp_jit_emit   -> writes the code
 *   mtgp_eval_rk4_jit with MtgpJitCode{code, offsets}.
 * Every evaluator uses the code except Dopri5 at state_size > 3 (interpreted; pass no code); the
 * wide-state SR kernel (n_var > 4) and the dynamic policy at state_size 4..16 need it built in
 * MTGP_JIT_MODE_LDS (mtgp_flatten_ex / mtgp_jit_emit_words; the latter without role chains:
 * mtgp_jit_chain returns none for it), the others in MTGP_JIT_MODE_REGS.  The code carries no mode
 * tag: code of the other mode is undefined behaviour. */
/* Role chains (ABI v13).  A role whose programs run back to back (the state_size state
 * equations of a dynamic policy, the n_var trees of SR with n_var <= 4) can be built as ONE
 * callable chain: bit j of `next` makes unit j fall through into unit j + 1 (laid out right
 * behind it) instead of returning; bit j of `cond` makes that continuation optional (taken when
 * the evaluator asks for it: the fixed-step dynamic kernel continues the state chain into the
 * save-point readout at save points; unused by the evaluators since ABI v18).  mtgp_jit_chain gives the chain the evaluator kernels of
 * `model` call; code built with another non-zero chain is rejected (MTGP_ERR_ARG), code built
 * without one ({0, 0, 0}) is called one program at a time as before.
 * store (ABI v14): LDS store chains for the wide-state SR kernels (MTGP_JIT_MODE_LDS code): every
 * unit j writes its result into the caller's LDS output vector (slot j) and falls through into
 * unit j + 1 unless j + 1 is a multiple of `store` -- one call per wave (its `store` components)
 * and stage. */
typedef struct {
  uint32_t next;
  uint32_t cond;
  uint32_t store;
  /* ABI v18: bit j of `put` -- unit j also copies its result into data register v[put_slot]
   * before falling through, so the next units read it as a data slot.  The fixed-step dynamic
   * policy chains readout -> (u into its slot) -> state programs: one call per stage. */
  uint32_t put;
  int32_t put_slot;
} MtgpJitChain;

typedef struct {
  const void* code;         /* executable device memory from mtgp_jit_alloc           */
  const uint32_t* offsets;  /* [units + 1] from mtgp_jit_plan (same model, R, order)   */
  const int32_t* info;      /* info[2] of mtgp_jit_plan, or NULL if the host checked it */
  uint64_t capacity;        /* bytes of `code`; the kernel interprets when info says the */
                            /* plan failed or the code did not fit (no host round trip) */
  MtgpJitChain chain;       /* the chain the code was built with (ABI v13/14; {0, 0, 0}: none) */
} MtgpJitCode;

int mtgp_jit_alloc(int32_t device, size_t bytes, void** code);
int mtgp_jit_free(void* code);
int mtgp_jit_units(int32_t P, int32_t n_prog, int32_t R);
int mtgp_jit_plan(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                  const int32_t* order, uint32_t* offsets_out, int32_t* info_out, void* stream);
int mtgp_jit_emit(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                  const int32_t* order, const uint32_t* offsets, void* code, size_t code_bytes,
                  void* stream);
/* The same plan / emit from mtgp_flatten_ex's jit_words (ABI v12): the unit layout is a gather +
 * scan of the per-program sizes, and emit translates the G programs of a unit in parallel.
 * Offsets, info and code are identical to mtgp_jit_plan / mtgp_jit_emit. */
int mtgp_jit_plan_words(const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t R,
                        const int32_t* order, uint32_t* offsets_out, int32_t* info_out, void* stream);
int mtgp_jit_emit_words(const MtgpInstr* prog, const int32_t* jit_words, int32_t P, int32_t n_prog,
                        int32_t L, int32_t R, const int32_t* order, const uint32_t* offsets, void* code,
                        size_t code_bytes, int32_t jit_mode, void* stream);
/* ABI v13: the role chain the evaluator of `model` (with n_prog programs) calls, and plan / emit /
 * host emission of chained code.  chain NULL = {0, 0} = the unchained functions above. */
int mtgp_jit_chain(const MtgpModel* model, int32_t n_prog, MtgpJitChain* chain_out);
int mtgp_jit_plan_words_chain(const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t R,
                              const int32_t* order, const MtgpJitChain* chain, uint32_t* offsets_out,
                              int32_t* info_out, void* stream);
int mtgp_jit_emit_words_chain(const MtgpInstr* prog, const int32_t* jit_words, int32_t P, int32_t n_prog,
                              int32_t L, int32_t R, const int32_t* order, const MtgpJitChain* chain,
                              const uint32_t* offsets, void* code, size_t code_bytes, int32_t jit_mode,
                              void* stream);
int mtgp_jit_unit_host_chain(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                             const int32_t* order, const MtgpJitChain* chain, int32_t unit, uint32_t* out,
                             int32_t max_words, int32_t jit_mode);
/* host translation of one program (tests/tooling): number of code words, or < 0 */
int mtgp_jit_translate_host(const MtgpInstr* prog, int32_t L, uint32_t* out, int32_t max_words);
/* the same in either JIT mode (MTGP_JIT_MODE_*), for one program and for one unit */
int mtgp_jit_unit_host_ex(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                          const int32_t* order, int32_t unit, uint32_t* out, int32_t max_words,
                          int32_t jit_mode);
int mtgp_jit_translate_host_ex(const MtgpInstr* prog, int32_t L, uint32_t* out, int32_t max_words,
                               int32_t jit_mode);
/* Schedule weights for JIT code: cost_out[P*n_prog] = executed code words / 4 of each program
 * (plen where a program cannot be translated); pass it to mtgp_schedule instead of plen. */
int mtgp_jit_cost(const MtgpInstr* prog, const int32_t* plen, int32_t P, int32_t n_prog, int32_t L,
                  int32_t* cost_out, void* stream);
/* host emission of one (wave, program) unit over HOST arrays prog/order (tests/tooling), laid
 * out as if it started right after the shared sin/cos subroutines (PC-relative calls) */
int mtgp_jit_unit_host(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                       const int32_t* order, int32_t unit, uint32_t* out, int32_t max_words);
int mtgp_eval_rk4_jit(const MtgpModel* model, const MtgpInstr* prog, const int32_t* plen,
                      int32_t n_prog, int32_t L, const int32_t* nodes, int32_t P,
                      const MtgpRollouts* rollouts, const MtgpOutputs* out, const MtgpJitCode* jit,
                      void* stream);

/* ------------------------------------------------- coefficient optimisation */
/* Loss and forward-mode gradient of the SR fitness w.r.t. K parameters per individual (ABI v11),
 * the value_and_grad of GeneticProgramming.epoch (gp.py:435-452, vmap_gradients gp.py:253).
 * Replaces: jax.vmap(jax.value_and_grad(partial_ff)) over SR_evaluator.__call__ (sr.py:30-45).
 * prog: mtgp_flatten output of the PARAMETERISED population: the coefficient rows being
 *   differentiated are variable rows reading data slots n_var .. n_var + K - 1 (the host
 *   transform, multitreegp_amd/coefficients.py), so programs read data[n_var + k] = theta[p, k].
 * theta[P, K]: parameter values; nparam[P] (<= K): parameters in use per individual.
 * scratch: device float [P, K, R, 2].  loss_out[P]: the evaluator's fitness without parsimony
 *   (bit-identical to mtgp_eval_rk4's with parsimony 0); grad_out[P, K] (0 beyond nparam).
 * model: MTGP_MODEL_SR with MTGP_SOLVER_RK4, MTGP_SOLVER_EULER or (ABI v17) MTGP_SOLVER_DOPRI5,
 * n_var + K <= MTGP_MAX_DATA, R <= 64; anything else returns MTGP_ERR_ARG.  Dopri5: the adaptive
 * solve (include/mtgp_dopri5.h, rollouts->ts the save points) in dual numbers with the step sizes,
 * accept / reject decisions and the event held at their primal values. */
int mtgp_sr_grad(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                 const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* rollouts,
                 float* scratch, float* loss_out, float* grad_out, void* stream);

/* ABI v16: the same for the dynamic and static control models (dynamic_evaluate.py:37-118,
 * feedforward_evaluate.py:36-110; value_and_grad of gp.py:253 / 435-452): every MTGP_ENV_*,
 * MTGP_SOLVER_RK4, MTGP_SOLVER_EULER or (ABI v17) MTGP_SOLVER_DOPRI5 (step sizes held at their
 * primal values, as mtgp_sr_grad), observation noise included, state_size <= 3, R <= 64.
 * The programs read the reference's data vector [y(n_obs), a, u, targets] (MtgpProgramSpec gap 0)
 * followed by the K parameter slots.  Tangent rules: include/mtgp_dual.h (the environment drift,
 * f_obs, clip); the argmax step of the Acrobot fitness (acrobot.py:79) is piecewise constant.
 * ABI v19: rollouts->fit_kof (the general Acrobot cost mask, ts off the one-pass grid) is
 * differentiated too; scratch must then hold P * K * R * 2 * (1 + n_save) floats (the lanes' cost
 * prefixes follow the partials). */
int mtgp_ctl_grad(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                  const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* rollouts,
                  float* scratch, float* loss_out, float* grad_out, void* stream);

/* ABI v19: the gradient programs as dual-number machine code (multitreegp_amd/csrc/mtgp_jit_dual.h):
 * value and tangent of every program instruction in registers, operation for operation the dual
 * interpreter (results bit-identical), the coefficients theta baked in as literals -- the code is
 * emitted on the stream by the call itself (count, scan, emit: a few microseconds), no host
 * round trip.  code: executable device memory from mtgp_jit_alloc; code_bytes: its size, at
 * least MTGP_GRAD_JIT_BYTES(P, n_prog, L) suffices for any program; offsets: device uint32
 * [P * n_prog + 1]; info: device int32 [2], written by the call ([0] < 0: some program does not
 * translate, [1]: bytes the code needs).  When the code does not fit or a program does not
 * translate, the kernel interprets (same results, slower).  jit == NULL or jit->code == NULL:
 * exactly mtgp_ctl_grad. */
typedef struct {
  void* code;
  size_t code_bytes;
  uint32_t* offsets;
  int32_t* info;
} MtgpGradJit;
#define MTGP_GRAD_JIT_WORDS_PER_INSTR 64
#define MTGP_GRAD_JIT_BYTES(P, n_prog, L) \
  (65536u + (size_t)(P) * (size_t)(n_prog) * ((size_t)(L) * 4u * MTGP_GRAD_JIT_WORDS_PER_INSTR + 64u))
int mtgp_ctl_grad_jit(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                      const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* rollouts,
                      float* scratch, float* loss_out, float* grad_out, const MtgpGradJit* jit, void* stream);
/* the same for the SR gradient (mtgp_sr_grad): code for n_var <= 4 (the register-state kernels;
 * wider states interpret) */
int mtgp_sr_grad_jit(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                     const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* rollouts,
                     float* scratch, float* loss_out, float* grad_out, const MtgpGradJit* jit, void* stream);
/* host translation of one program in dual numbers (D data slots <= 8, K coefficients theta):
 * words written (out == NULL: counted), or < 0 (untranslatable / out too short) */
int mtgp_jit_dual_translate_host(const MtgpInstr* prog, int32_t L, int32_t D, const float* theta, int32_t K,
                                 uint32_t base, uint32_t* out, int32_t max_words);

/* Wall time of the calling thread's last timed mtgp_eval_rk4 kernel (ms), measured with
 * hipEvents recorded on its stream around the launch; -1 if none.  Synchronises that event.
 * The on/off switch (mtgp_set_timing) is process-wide; events are per host thread and device. */
float mtgp_last_kernel_ms(void);
/* The durations (ms) of the calling thread's last n timed launches, oldest first, into out[n]
 * (a ring of the last 1024 launches is kept): returns how many were written.  Lets a caller time
 * a whole run with one synchronisation at the end instead of one per launch. */
int mtgp_kernel_ms_history(float* out, int32_t n);
int mtgp_set_timing(int enabled);

#ifdef __cplusplus
}
#endif
#endif /* MTGP_H */
