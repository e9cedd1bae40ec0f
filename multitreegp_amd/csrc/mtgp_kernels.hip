// mtgp_kernels.hip -- MI355X (gfx950) population-fitness evaluator for MultiTreeGP.
//
// One wavefront = G = 64 / Rp individuals x Rp (R rounded up to a power of two) rollouts.
// The environment (drift, observation, RK4 update, fitness) is lane-parallel; each
// individual's tree programs are wave-uniform instruction streams, fetched with scalar loads
// (four instructions per s_load_dwordx8) and dispatched with scalar branches, while the
// per-rollout values live in VGPRs.  The data vector a tree reads and its operand stack live
// in LDS (one 64-lane column per slot, conflict-free).  The interpreter is fused into a
// fixed-step RK4 integrator: the ODE state stays in registers for the whole rollout, fitness
// is accumulated online at the save points, and only the [P] fitness (plus optional
// time-major trajectories) leaves the CU.  Individuals are mapped to waves through an
// optional schedule (MtgpRollouts.order, built by mtgp_schedule) that balances per-wave
// interpreter work.
//
// Reference path replaced: GeneticProgramming.evaluate_population -> shard_eval ->
// vmap(Evaluator.__call__) -> diffeqsolve(_drift -> vmap_foriloop)  (gp.py:259-269,
// 403-433; dynamic_evaluate.py:37-118; feedforward_evaluate.py:36-110;
// SR_evaluator.py:30-94; acrobot.py:29-87).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdlib.h>
#include <atomic>
#include <cstring>
#include <mutex>
#include <type_traits>
#include "mtgp.h"
#include "mtgp_ab.h"
#include "mtgp_f32math.h"
#include "mtgp_prng.h"
#include "mtgp_dopri5.h"
#include "mtgp_cstep.h"
#include "mtgp_flatten.h"
#include "mtgp_flatten_uniform.h"
#include "mtgp_jit.h"

// Translation units.  The library is compiled from this file several times in parallel
// (__graft_entry__.build_hip): MTGP_TU=0 holds the C ABI, the Acrobot / SR / JIT / flatten /
// schedule kernels; MTGP_TU=1 and 2 hold the HarmonicOscillator and StirredTankReactor RK4
// control kernels, MTGP_TU=3 / 4 / 5 the Dopri5 control kernels of Acrobot / HarmonicOscillator /
// StirredTankReactor, MTGP_TU=6 the Acrobot kernels of the general cost mask (EnvAcrobotMask),
// MTGP_TU=7 the fixed-step Acrobot control kernels (the C3 / C2 hot kernels: an A/B variant of
// them recompiles this unit only, scripts/build_ab.py), MTGP_TU=8 the SR kernels, MTGP_TU=9 the
// runtime-state-size Dopri5 control kernels (state_size 4 .. 16, round 6), behind one hidden C++
// entry each.  Without MTGP_TU it is one monolithic TU.
#ifndef MTGP_TU
#define MTGP_TU_MAIN 1
#define MTGP_TU_HARMONIC 1
#define MTGP_TU_REACTOR 1
#define MTGP_TU_ACRO_DOPRI5 1
#define MTGP_TU_HARMONIC_DOPRI5 1
#define MTGP_TU_REACTOR_DOPRI5 1
#define MTGP_TU_ACRO_MASK 1
#define MTGP_TU_ACRO 1
#define MTGP_TU_SR 1
#define MTGP_TU_DP_RT 1
#else
#define MTGP_TU_MAIN (MTGP_TU == 0)
#define MTGP_TU_HARMONIC (MTGP_TU == 1)
#define MTGP_TU_REACTOR (MTGP_TU == 2)
#define MTGP_TU_ACRO_DOPRI5 (MTGP_TU == 3)
#define MTGP_TU_HARMONIC_DOPRI5 (MTGP_TU == 4)
#define MTGP_TU_REACTOR_DOPRI5 (MTGP_TU == 5)
#define MTGP_TU_ACRO_MASK (MTGP_TU == 6)
#define MTGP_TU_ACRO (MTGP_TU == 7)
#define MTGP_TU_SR (MTGP_TU == 8)
#define MTGP_TU_DP_RT (MTGP_TU == 9)
#endif

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kDMax = 8;  // data slots held in LDS by the small-state kernels
constexpr int kDWide = 16;     // data slots of the runtime-state-size dynamic kernels (interpreter only)
constexpr int kNaRuntime = 8;  // k_ctl_dynamic / k_ctl_dopri5<Env, kNaRuntime, ...>: state_size 4 .. 8 at run time
constexpr int kDWide2 = 24;    // data slots of the wide runtime-state-size kernels (round 6)
constexpr int kNaWide = 16;    // k_ctl_dynamic / k_ctl_dopri5<Env, kNaWide, ...>: state_size 9 .. 16 at run time
// data slots of a dynamic-policy kernel with state-size template NA (NA <= 3: the JIT's register ABI)
constexpr int dyn_data_slots(int NA) { return NA <= 3 ? kDMax : (NA <= kNaRuntime ? kDWide : kDWide2); }
constexpr int kSMax = MTGP_STACK_MAX;
constexpr int kLdsWaveWords = (kDMax + kSMax) * kWave;  // per wave: data columns | stack columns
constexpr float kInf = __builtin_huge_valf();

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// wave votes over the active lanes as one ballot compare (the ockl __all / __any round-trip through
// a VGPR: v_cndmask + v_cmp + s_cmp per vote)
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ bool wave_all(bool p) { return __builtin_amdgcn_ballot_w64(!p) == 0; }

// --------------------------------------------------------------------------------------
// The interpreter.  `dcol` = this lane's column of the wave's LDS data vector (stride 64
// floats per slot), `st` = this lane's column of the operand stack.  `code`/`len` are
// wave-uniform, so the opcode switch compiles to a scalar branch tree and each handler is
// 1-3 vector instructions.
//
// Measured alternatives (C3, see DESIGN.md "Interpreter design record"):
//  * SIMT interpreter (every lane runs its own individual's program, branch-free select/fma
//    ALU): 1.5x slower at G = 2 -- ~35 VALU per step vs the scalar dispatch's ~4.
//  * branch-free uniform decode with SGPR select masks, data/stack in VGPRs via
//    s_set_gpr_idx: 1.9x slower (an indexed VGPR access costs ~70 cycles on gfx950,
//    scripts/micro/gpridx_cost.hip); the same with LDS data: 1.45x slower (2x the per-wave
//    instruction stream; issue, not branch latency, bounds this loop).
//  * per-instruction scalar loads (no blocks): 6-10% slower; a VGPR-lane program cache: 15%
//    slower; data vector in VGPRs behind a scalar branch tree: 2% slower.
// One instruction: the generated dispatch tree (scripts/gen_opcodes.py -> mtgp_dispatch.inc):
// range compares on the raw word w = opcode << 24 | aux, shaped by measured opcode
// frequencies; each leaf is the opcode's 1-3 instruction handler.  Expanded inline at each of
// the four block positions; END leaves the program (no per-instruction length test).
#include "mtgp_dispatch.inc"

// Programs are read through the constant address space so the wave-uniform fetch is a
// scalar load (K$), four instructions (32 B) per s_load_dwordx8.  The program stride L is a
// multiple of 4 (checked by the entry points), so a block never crosses a program slot, and
// a program's END lies inside its slot.
typedef uint32_t u8v __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) u8v* ConstBlockPtr;

__device__ __forceinline__ float run_prog(const MtgpInstr* code, const float* dcol, float* st) {
  ConstBlockPtr blk = (ConstBlockPtr)code;
  float acc = 0.0f;
  int sp = 0;
  for (;; ++blk) {
    const u8v c = *blk;
    MTGP_DISPATCH(c[0], c[1])
    MTGP_DISPATCH(c[2], c[3])
    MTGP_DISPATCH(c[4], c[5])
    MTGP_DISPATCH(c[6], c[7])
  }
done:
  return acc;
}

__device__ __forceinline__ void dset(float* dcol, int slot, float v) { dcol[slot * kWave] = v; }

// --------------------------------------------------------------------------------------
// Acrobot (acrobot.py:7-87).  Per-rollout invariant products are formed once with the same
// operations/operands as the Python expression, so the per-call result is bit-identical.
struct AcroConst {
  float m2, d1a, l1sq_lc2sq, two_l1lc2, lc2sq, l1lc2, m2lc2g, A0, B0, C0, m2l1lc2, den0;
};

__device__ __forceinline__ AcroConst acro_const(float l1, float l2, float m1, float m2) {
  AcroConst k;
  const float lc1 = 0.5f * l1, lc2 = 0.5f * l2, g = 9.81f;
  k.m2 = m2;
  k.d1a = m1 * (lc1 * lc1);
  k.l1sq_lc2sq = (l1 * l1) + (lc2 * lc2);
  k.two_l1lc2 = (2.0f * l1) * lc2;
  k.lc2sq = lc2 * lc2;
  k.l1lc2 = l1 * lc2;
  k.m2lc2g = (m2 * lc2) * g;
  k.A0 = ((-m2) * l1) * lc2;
  k.B0 = ((2.0f * m2) * l1) * lc2;
  k.C0 = ((m1 * lc1) + (m2 * l1)) * g;
  k.m2l1lc2 = (m2 * l1) * lc2;
  k.den0 = (m2 * (lc2 * lc2)) + 1.0f;
  return k;
}

// IEEE fp32 division n / d in two parts, for operands in a safe range.  The hardware sequence
// LLVM emits for `/` is v_div_scale (x2), v_rcp, a Newton step of the reciprocal, q = n r and two
// fma corrections, v_div_fmas, v_div_fixup.  When |n| and |d| lie in [2^-40, 2^40] (finite, non-zero,
// not denormal) v_div_scale scales nothing, v_div_fmas is a plain fma and v_div_fixup passes the
// quotient through, so the remaining steps below give the same correctly rounded bits; a NaN operand
// gives NaN either way.  The reciprocal part depends on d alone, so the three divisions of the
// Acrobot drift by d1 share one (two v_rcp instead of four, and no scale/fixup).  Callers test the
// range with one wave-uniform branch and fall back to `/` otherwise.
__device__ __forceinline__ float div_rcp(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_by(float n, float d, float r) {
  float q = n * r;
  q = __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
}
// |v| in [2^-40, 2^40] or NaN (NaN propagates identically through both paths)
__device__ __forceinline__ bool div_safe(float v) {
  const float a = __builtin_fabsf(v);
  return !(a < 9.094947e-13f) && !(a >= 1.0995116e12f);
}

// The drift's denominators d1 and den and the numerators d2, d2*d2 depend on the state only through
// c2 = cos(theta2) in [-1, 1]: d1 and d2 are monotone in c2 (each operation rounds monotonically),
// so their values at c2 = +-1.001 bound them, and den = den0 - d2^2 / d1 is bounded by the extreme
// quotients.  Safe for every theta2 when those bounds lie well inside [2^-40, 2^40] (true for any
// physical parameters; a NaN c2 makes everything NaN on both paths).  Per rollout, once.
__device__ __forceinline__ bool acro_div_ok(const AcroConst& k) {
  float d1b[2], d2b[2];
  for (int e = 0; e < 2; ++e) {
    const float c2 = e ? 1.001f : -1.001f;
    d1b[e] = ((k.d1a + k.m2 * (k.l1sq_lc2sq + k.two_l1lc2 * c2)) + 1.0f) + 1.0f;
    d2b[e] = k.m2 * (k.lc2sq + k.l1lc2 * c2) + 1.0f;
  }
  const float lo = 1e-9f, hi = 1e9f;  // 2^-40 .. 2^40 with ample margin for the rounding
  bool ok = true;
  for (int e = 0; e < 2; ++e) ok = ok && d1b[e] > lo && d1b[e] < hi && d2b[e] > lo && d2b[e] < hi;
  if (!ok) return false;
  const float d1lo = fminf(d1b[0], d1b[1]), d1hi = fmaxf(d1b[0], d1b[1]);
  const float d2lo = fminf(d2b[0], d2b[1]), d2hi = fmaxf(d2b[0], d2b[1]);
  const float denlo = k.den0 - (d2hi * d2hi) / d1lo * 1.001f, denhi = k.den0 - (d2lo * d2lo) / d1hi * 0.999f;
  return d2lo * d2lo > lo && d2hi * d2hi < hi && denlo > lo && denhi < hi;
}

// The fast path of mtgp_trig_pi is the spec's result for |arg| < 2^17 and for non-finite args.
// Every trig argument of the Acrobot drift and fitness is theta1, theta2, their sum or theta1 -
// pi/2 (+ theta2): when neither angle is a finite value of magnitude >= 2^15, each argument is
// either below 2^16 + 2 in magnitude or non-finite, so the fast path is exact for all of them --
// one range test per angle (on the bits: |v| in [2^15, inf) <=> slow possible) instead of a
// compare pair per trig value.
__device__ __forceinline__ bool trig_args_small(float v) {
  return (__float_as_uint(v) & 0x7fffffffu) - 0x47000000u >= 0x38800000u;
}

__device__ __forceinline__ void acro_drift(const AcroConst& k, const float x[4], float u_raw,
                                           float dx[4], bool fastdiv = false) {
  const float control = mtgp_clip1(u_raw);
  const float th1 = x[0], th2 = x[1], thd1 = x[2], thd2 = x[3];
#if MTGP_AB_NODRIFT  // diagnostic (mtgp_ab.h): no drift arithmetic at all
  dx[0] = thd1; dx[1] = thd2; dx[2] = control; dx[3] = -control;
  return;
#endif
#if MTGP_AB_NOTRIG  // diagnostic: one multiply per trig value
  const float s2 = th2 * 0.5f, c2 = th2 * 0.25f, s1 = th1 * 0.5f, ca = (th1 + th2) * 0.5f, cb = th1 * 0.25f;
#else
  // the five trig values of the drift (mtgp_sinf / mtgp_cosf bit for bit), with ONE wave-uniform
  // test for lanes that may need the slow reduction (trig_args_small)
  const float ea = (th1 + th2) - MTGP_HALF_PI_F, eb = th1 - MTGP_HALF_PI_F;
  int f0, f1, f2, f3, f4;
  float s2 = mtgp_trig_pi_fast(th2, 0, &f0), c2 = mtgp_trig_pi_fast(th2, 1, &f1);
  float s1 = mtgp_trig_pi_fast(th1, 0, &f2);
  float ca = mtgp_trig_pi_fast(ea, 1, &f3), cb = mtgp_trig_pi_fast(eb, 1, &f4);
  (void)f0; (void)f1; (void)f2; (void)f3; (void)f4;
  if (__builtin_expect(!wave_all(trig_args_small(th1) && trig_args_small(th2)), 0)) {
    s2 = mtgp_sinf(th2);
    c2 = mtgp_cosf(th2);
    s1 = mtgp_sinf(th1);
    ca = mtgp_cosf(ea);
    cb = mtgp_cosf(eb);
  }
#endif
#if MTGP_AB_NODIV  // diagnostic: the four divisions as products
#define MTGP_ACRO_DIV(a, b) ((a) * (b))
#else
#define MTGP_ACRO_DIV(a, b) ((a) / (b))
#endif
  const float d1 = ((k.d1a + k.m2 * (k.l1sq_lc2sq + k.two_l1lc2 * c2)) + 1.0f) + 1.0f;
  const float d2 = k.m2 * (k.lc2sq + k.l1lc2 * c2) + 1.0f;
  const float phi2 = k.m2lc2g * ca;
  const float phi1 = (((k.A0 * (thd2 * thd2)) * s2 - ((k.B0 * thd1) * thd2) * s1) +
                      k.C0 * cb) + phi2;
#if !MTGP_AB_NODIV && !MTGP_AB_SLOWDIV
  if (__builtin_expect(fastdiv, 1)) {  // wave-uniform: the denominators are safe (acro_div_ok)
    const float r1 = div_rcp(d1);
    const float num = ((control + div_by(d2, d1, r1) * phi1) - (k.m2l1lc2 * (thd1 * thd1)) * s2) - phi2;
    const float den = k.den0 - div_by(d2 * d2, d1, r1);
    float a2, a1;
    if (__builtin_expect(wave_all(div_safe(num)), 1)) a2 = div_by(num, den, div_rcp(den));
    else a2 = num / den;
    const float n1 = -((d2 * a2) + phi1);
    if (__builtin_expect(wave_all(div_safe(n1)), 1)) a1 = div_by(n1, d1, r1);
    else a1 = n1 / d1;
    dx[0] = thd1;
    dx[1] = thd2;
    dx[2] = a1;
    dx[3] = a2;
    return;
  }
#endif
  const float num = ((control + MTGP_ACRO_DIV(d2, d1) * phi1) - (k.m2l1lc2 * (thd1 * thd1)) * s2) - phi2;
  const float den = k.den0 - MTGP_ACRO_DIV(d2 * d2, d1);
  const float a2 = MTGP_ACRO_DIV(num, den);
  const float a1 = MTGP_ACRO_DIV(-((d2 * a2) + phi1), d1);
#undef MTGP_ACRO_DIV
  dx[0] = thd1;
  dx[1] = thd2;
  dx[2] = a1;
  dx[3] = a2;
}

// Observation noise (cbase.py:43-48): out = C@x + normal(fold_in(key, bitcast(t)), (NO,)) @ W.
// The key is per rollout (obs_noise_keys, dyn.py:65), W (acrobot.py:49: obs_noise * I;
// reactor.py:43: obs_noise * I * [15, 15, 0.1]) is shared.  C@x and the noise product are
// summed in index order exactly like the oracle.
// NV = the environment's latent size; the observation has z.no <= NV components (C =
// eye(n_var)[:n_obs], control_environment_base.py:47 / acrobot.py:48), W is [no, no].
template <int NO>
struct ObsNoise {
  uint32_t k0, k1;  // this lane's rollout key
  const float* W;   // [no, no] row-major (read with scalar loads when used: no registers held)
  int impl;         // MTGP_PRNG_* random-bits layout
  int no;           // observed components (MtgpModel.n_obs), wave-uniform
  bool diag;        // W diagonal with a non-zero diagonal: noise_j = n_j * W_jj exactly
};

template <int NO>
__device__ __forceinline__ ObsNoise<NO> obs_noise_setup(const MtgpModel& m, const MtgpRollouts& ro, int rr) {
  ObsNoise<NO> z;
  z.k0 = ro.obs_keys[2 * rr + 0];
  z.k1 = ro.obs_keys[2 * rr + 1];
  z.W = ro.obs_w;
  z.impl = m.prng_impl;
  z.no = uni(m.n_obs);
  const int no = z.no;
  bool diag = true;
#pragma unroll
  for (int i = 0; i < NO; ++i)
#pragma unroll
    for (int j = 0; j < NO; ++j)
      if (i < no && j < no) diag = diag && ((i == j) ? (z.W[i * no + j] != 0.0f) : (z.W[i * no + j] == 0.0f));
  z.diag = uni((int)diag) != 0;
  return z;
}

// normal(fold_in(key, bitcast(t)), (no,)) for a wave-uniform no <= NO (the draw depends on the
// shape): one compile-time instance per count, the rest of n[] zero
template <int NO>
__device__ __forceinline__ void obs_normals_n(uint32_t k0, uint32_t k1, float t, int no, int impl, float (&n)[NO]) {
  if (no == NO) {
    mtgp_obs_normals(k0, k1, t, NO, impl, n);
    return;
  }
  if constexpr (NO > 1) {
    float m[NO - 1];
    obs_normals_n<NO - 1>(k0, k1, t, no, impl, m);
#pragma unroll
    for (int j = 0; j < NO - 1; ++j) n[j] = m[j];
  }
  n[NO - 1] = 0.0f;
}

// noise vector normal(fold_in(key, bitcast(t)), (no,)) @ W (summed in index order).  With W
// diagonal and non-zero on the diagonal, the off-diagonal products are +-0 and the sum is
// exactly n_j * W_jj (n_j is never 0: |u| > 0 always), so the product is skipped.  Components
// j >= no (unobserved) are 0.
template <int NO>
__device__ __forceinline__ void obs_noise_vec(const ObsNoise<NO>& z, float t, float nz[NO]) {
  float n[NO];
  const int no = z.no;
  obs_normals_n<NO>(z.k0, z.k1, t, no, z.impl, n);
  if (z.diag) {
#pragma unroll
    for (int j = 0; j < NO; ++j) nz[j] = j < no ? n[j] * z.W[j * no + j] : 0.0f;
    return;
  }
#pragma unroll
  for (int j = 0; j < NO; ++j) {
    float acc = 0.0f;
    if (j < no) {
      acc = n[0] * z.W[j];
#pragma unroll
      for (int i = 1; i < NO; ++i)
        if (i < no) acc = acc + n[i] * z.W[i * no + j];
    }
    nz[j] = acc;
  }
}

// y = C@x + nz with C = eye(n_var)[:n_obs]: all NV components are formed, the programs read only
// the first n_obs (the flattener places the data slots after the observations behind all NV,
// MtgpProgramSpec.gap) and only those are stored as ys.  (C@x)_i + nz_i
// equals x_i + nz_i when every x_j is finite (the +-0 terms 0*x_j cannot change the sum; with
// nz = +0 a -0 becomes +0 either way), NaN otherwise (0*inf), then the environment's own
// observation transform (Acrobot: angle wrap, acrobot.py:29-32).
template <class Env>
__device__ __forceinline__ void ctl_obs_apply(const float x[Env::NV], const float nz[Env::NV], float y[Env::NV]) {
  constexpr int NV = Env::NV;
#if MTGP_AB_NOOBS  // diagnostic: observation = state
#pragma unroll
  for (int i = 0; i < NV; ++i) y[i] = x[i] + nz[i];
  return;
#endif
  bool fin[NV], all = true;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    fin[j] = mtgp_isfinite(x[j]);
    all = all && fin[j];
  }
  if (__builtin_expect(wave_all(all), 1)) {  // every lane's state finite (the common case): no NaN masking
#pragma unroll
    for (int i = 0; i < NV; ++i) y[i] = x[i] + nz[i];
    Env::obs_transform(y);
    return;
  }
  const float qn = mtgp_qnan();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NV; ++j)
      if (j != i) ok = ok && fin[j];
    y[i] = ok ? x[i] + nz[i] : qn;
  }
  Env::obs_transform(y);
}

template <class Env, bool NOISE>
__device__ __forceinline__ void ctl_obs(const ObsNoise<Env::NV>& z, float t, const float x[Env::NV], float y[Env::NV]) {
  float nz[Env::NV];
#pragma unroll
  for (int j = 0; j < Env::NV; ++j) nz[j] = 0.0f;
  if (NOISE) obs_noise_vec<Env::NV>(z, t, nz);
  ctl_obs_apply<Env>(x, nz, y);
}

__device__ __forceinline__ bool acro_bad(const float* s, int n) {
  bool bad = !(__builtin_fabsf(s[2]) <= MTGP_8PI_F) && !mtgp_isnan(s[2]);
  bad = bad || (!(__builtin_fabsf(s[3]) <= MTGP_18PI_F) && !mtgp_isnan(s[3]));
  for (int i = 0; i < n; ++i) bad = bad || !mtgp_isfinite(s[i]);
  return bad;
}

struct KArgs {
  MtgpModel m;
  const MtgpInstr* prog;
  const int32_t* plen;
  int32_t n_prog, L;
  const int32_t* nodes;
  int32_t P;
  MtgpRollouts ro;
  MtgpOutputs out;
  uint64_t jit_base;        // JIT code (executable device memory) or 0: interpreter only
  const uint32_t* jit_off;  // [n_waves, n_prog] byte offset of each (wave, program) unit's code
  const int32_t* jit_info;  // mtgp_jit_plan info {status, total bytes} (device) or NULL
  uint64_t jit_cap;         // bytes of the code buffer
  int32_t chain_state;      // the JIT code chains the state role (MtgpJitChain): one call per stage
  int32_t chain_save;       // ... and continues it into the save-point readout on request (s46; unused since ABI v18)
  int32_t chain_store;      // the wide-state SR code is LDS store chains: one call per wave and stage
  int32_t chain_merge;      // (ABI v18) the dynamic policy's readout chains into its state programs, u put in its slot
  uint32_t epoch;           // launch counter, never 0 (tags the fair-share progress posts)
  int32_t fair;             // fair share of the SIMDs' issue slots (FairShare; MTGP_FAIR)
  int32_t fair_dp;          // the same for the Dopri5 attempt loops (MTGP_FAIR_DP)
  int32_t fair_mode;        // 0: two priority levels; 1: the slowest wave of a SIMD above the rest (MTGP_FAIR_MODE)
  // Dopri5 in two launches (ABI v16, MtgpModel.dp_budget): launch 1 runs every wave for at most
  // dp_budget attempts and parks the lanes of waves that are not done (dp_state, word-major
  // [kDpStateWords][waves * 64]) in the list dp_pending ([0] = count, then wave ids); launch 2
  // resumes only those waves, each (mostly) alone on its SIMD.
  int32_t dp_budget, dp_pass;
  float* dp_state;
  int32_t* dp_pending;
  uint32_t dp_lanes;  // waves * 64 of the launch: the stride of a dp_state word
};

// per-lane online Acrobot fitness (acrobot.py:77-84 restated for a single pass)
struct AcroFit {
  bool settled;
  float csum, c0incl, F;
};

// A read-only per-launch table (ts) read through the constant address space: a wave-uniform index
// becomes a scalar load (scalar cache, lgkm wait) instead of a vector load with a vmcnt wait -- the
// compiler cannot prove a plain pointer unwritten by the kernel's stores.  Nothing on the device
// writes these tables, so the scalar cache sees them coherently.  (A divergent index still gets a
// vector load.)
__device__ __forceinline__ float ldc(const float* p, int i) {
  return ((const __attribute__((address_space(4))) float*)p)[i];
}
__device__ __forceinline__ bool save_incl(const float* ts, int k);
// incl (acrobot.py:82's mask at save k, save_incl) is needed only at save 0 and at a lane's first
// success: it is evaluated there (a division and three loads) instead of at every save point
__device__ __forceinline__ void acro_fit_update(AcroFit& f, int k, int S, const float* ts, float u,
                                                float x0, float x1) {
  if (f.settled) return;
  int fa, fb;
  const float x01 = x0 + x1;
  float ca = mtgp_trig_pi_fast(x0, 1, &fa), cb = mtgp_trig_pi_fast(x01, 1, &fb);
  (void)fa; (void)fb;
  if (__builtin_expect(!wave_all(trig_args_small(x0) && trig_args_small(x1)), 0)) {
    ca = mtgp_cosf(x0);
    cb = mtgp_cosf(x01);
  }
  const bool reached = ((-ca) - cb) > 1.5f;
  const float cost = (u * 0.01f) * u;
  if (k == 0) {
    f.c0incl = save_incl(ts, 0) ? cost : 0.0f;
    f.csum = cost;
    if (reached) { f.settled = true; f.F = (float)S + f.c0incl; }
  } else if (reached) {
    f.settled = true;
    f.F = (float)k + (f.csum + (save_incl(ts, k) ? cost : 0.0f));
  } else {
    f.csum = f.csum + cost;
  }
}

// The general mask (MtgpRollouts.fit_kof given: ts / (ts[1] - ts[0]) is not within one of the save
// index, e.g. ts starting at t > 0): the cost sum is the prefix of the first kof[first_success]
// costs (acrobot.py:82 keeps ratio <= first_success, a prefix of the non-decreasing ratio) summed
// left to right, the masked zeros adding nothing.  Per lane: csum = running prefix (hist row k when
// the prefix can lie behind the first success), c0incl = the prefix kof[0] (first_success 0: never
// reached, or reached at save 0), F = first success + 1 as int bits until settled (0 = none yet).
// The +inf fill after a termination never reaches (cos(inf) is NaN) but its costs (the policy on
// the fill) still count when the prefix runs past it; the last save point settles every lane.
#if MTGP_DEBUG_CHECKS
// violation counters of the debug build: [0] store_row lane offset outside its row, [1] a store
// row past the end of its array (row >= n_rows * row_len is checked by the callers' indices),
// [2] fit_hist write index outside [0, S * PR), [3] fit_hist read index outside it
static __device__ unsigned long long g_dbg_viol[4];  // one per TU (static: no host-symbol clash at link)
__device__ __forceinline__ void dbg_count(int i) { atomicAdd(&g_dbg_viol[i], 1ull); }
#endif
__device__ __forceinline__ void acro_fit_general(AcroFit& f, int k, int S, const int32_t* __restrict__ kof,
                                                 float* hist, size_t PR, int loff, bool dead, float u,
                                                 float x0, float x1) {
  if (f.settled) return;
  const float P = f.csum + (u * 0.01f) * u;  // save 0: 0 + cost = cost
  f.csum = P;
#if MTGP_DEBUG_CHECKS
  if (hist && (k < 0 || k >= S || loff < 0 || (size_t)loff >= PR)) { dbg_count(2); hist = nullptr; }
#endif
  if (hist) hist[(size_t)k * PR + loff] = P;  // read back by this lane only (below)
  if (k + 1 == kof[0]) f.c0incl = P;
  int fs1 = __float_as_int(f.F);
  if (fs1 == 0) {
    bool reached = false;
    if (!dead) {
      const float x01 = x0 + x1;
      reached = ((-mtgp_cosf(x0)) - mtgp_cosf(x01)) > 1.5f;
    }
    fs1 = reached ? k + 1 : ((dead || k == S - 1) ? 1 : 0);  // argmax of all-false = 0
  }
  if (fs1 == 0) return;
  const int fs = fs1 - 1, K = kof[fs];
  if (K > k + 1) {  // the prefix runs on past this save point
    f.F = __int_as_float(fs1);
    return;
  }
  float v = 0.0f;
  if (K > 0) {
    if (fs == 0) v = f.c0incl;
    else if (K == k + 1) v = P;
    else {
#if MTGP_DEBUG_CHECKS
      if (!hist || K - 1 < 0 || K - 1 >= S || loff < 0 || (size_t)loff >= PR) {
        dbg_count(3);
        f.settled = true;
        f.F = mtgp_qnan();
        return;
      }
#endif
      v = __hip_atomic_load(hist + (size_t)(K - 1) * PR + loff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  f.settled = true;
  f.F = (float)(fs + (fs == 0) * S) + v;
}

__device__ __forceinline__ bool save_incl(const float* ts, int k) {
  const float dts = ldc(ts, 1) - ldc(ts, 0);
  return !((ldc(ts, k) / dts) > (float)k);
}

// --------------------------------------------------------------------------------------
// Environments (control_environments/*.py).  Each is a per-lane struct: its parameters and
// target live in registers for the whole rollout; drift, observation transform, termination
// test and an online (single-pass) fitness accumulator, each restating the reference's
// expression with the same operations and operand order as the oracle (bit-identical).
//   NV          latent state size (= n_obs: C = I on this path)
//   load        per-rollout constants (initialize_parameters) and the target
//   drift       EnvironmentBase.drift(t, x, u) (autonomous: t unused by all three)
//   bad         the cond_fn_nan event (true = terminate)
//   fit_*       fitness_function over the saved points, accumulated at each save; fit_kill marks
//               a rollout whose remaining save points are the +inf fill (its fitness is then
//               fixed: Acrobot ignores them, the quadratic costs become NaN).

// Acrobot (acrobot.py:7-87)
struct EnvAcrobot {
  static constexpr int NV = 4;
  static constexpr bool kMask = false;  // the one-pass fitness (MtgpRollouts.fit_kof NULL)
  // the 4 rollout parameters stay in registers; the 12 derived products are rebuilt at each drift
  // (same operations, so bit-identical) -- holding them live cost 8 VGPRs next to the JIT call
  float l1, l2, m1, m2;
  bool fastdiv;  // wave-uniform: every lane's drift denominators are in the safe range (acro_div_ok)
  typedef AcroFit Fit;
  __device__ __forceinline__ void load(const MtgpRollouts& ro, int rr, int nt) {
    (void)nt;
    l1 = ro.params[4 * rr + 0];
    l2 = ro.params[4 * rr + 1];
    m1 = ro.params[4 * rr + 2];
    m2 = ro.params[4 * rr + 3];
    fastdiv = wave_all(acro_div_ok(acro_const(l1, l2, m1, m2)));
  }
  __device__ __forceinline__ void drift(const float x[4], float u, float dx[4]) const {
    acro_drift(acro_const(l1, l2, m1, m2), x, u, dx, fastdiv);
  }
  __device__ __forceinline__ static void obs_transform(float y[4]) {
    y[0] = mtgp_wrap_angle(y[0]);
    y[1] = mtgp_wrap_angle(y[1]);
  }
  __device__ __forceinline__ static bool bad(const float* s, int n) { return acro_bad(s, n); }
  __device__ __forceinline__ static Fit fit_init(bool active) { return Fit{!active, 0.0f, 0.0f, 0.0f}; }
  __device__ __forceinline__ void fit_update(Fit& f, int k, int S, const float* ts, float u, const float x[4]) const {
    acro_fit_update(f, k, S, ts, u, x[0], x[1]);
  }

  __device__ __forceinline__ static void fit_kill(Fit& f) { (void)f; }  // fs/cost mask ignore the fill
  __device__ __forceinline__ static float fit_final(Fit& f, int S) {
    if (!f.settled) { f.settled = true; f.F = (float)S + f.c0incl; }
    return f.F;
  }
};

// Acrobot with the general cost mask (MtgpRollouts.fit_kof): kernels of its own (translation unit
// 6, trajectory variants only: no early exit on settled lanes), so that the one-pass kernels keep
// their registers -- a run-time switch inside them held the mask's pointers live through the loop
// and cost the C3 kernel 1.3 % more VALU (SGPR spills) and 1.1 % time.
struct EnvAcrobotMask : EnvAcrobot {
  static constexpr bool kMask = true;
  // one save point (dead: a point of the +inf fill)
  __device__ __forceinline__ void fit_save(Fit& f, int k, int S, const KArgs& A, size_t PR, int loff, bool dead,
                                           float u, const float x[4]) const {
    acro_fit_general(f, k, S, A.ro.fit_kof, A.out.fit_hist, PR, loff, dead, u, x[0], x[1]);
  }
};

__device__ __forceinline__ bool any_nonfinite(const float* s, int n) {
  bool bad = false;
  for (int i = 0; i < n; ++i) bad = bad || !mtgp_isfinite(s[i]);
  return bad;
}

// (e^T Q) e with every product summed left to right over the full matrix (zeros included), the
// literal `(x - x_d).T @ Q @ (x - x_d)` of harmonic_oscillator.py:76 / reactor.py:77
template <int N>
__device__ __forceinline__ float quad_form(const float e[N], const float (&Q)[N * N]) {
  float out = 0.0f;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float v = e[0] * Q[j];
#pragma unroll
    for (int i = 1; i < N; ++i) v = v + e[i] * Q[i * N + j];
    out = (j == 0) ? v * e[0] : out + v * e[j];
  }
  return out;
}

// running sum of per-save quadratic costs (jnp.sum(costs), summed in time order)
struct QuadFit {
  bool settled;
  float F;
};

// HarmonicOscillator (harmonic_oscillator.py:8-80): dx = A x + b u, A = [[0, 1], [-omega, -zeta]],
// b = [0, 1]^T; cost (x - x_d)^T Q (x - x_d) + (u - u_d) R (u - u_d), x_d = [target, 0],
// u_d = -pinv(b) A x_d with pinv(b) = [[0, 1]] exactly, Q = [[0.5, 0], [0, 0]], R = [[0.5]].
struct EnvHarmonic {
  static constexpr int NV = 2;
  static constexpr bool kMask = false;
  float a10, a11, tg, ud;
  typedef QuadFit Fit;
  __device__ __forceinline__ void load(const MtgpRollouts& ro, int rr, int nt) {
    a10 = -ro.params[2 * rr + 0];
    a11 = -ro.params[2 * rr + 1];
    tg = ro.targets[rr * nt];
    const float M0 = (-0.0f) * 0.0f + (-1.0f) * a10, M1 = (-0.0f) * 1.0f + (-1.0f) * a11;  // -pinv(b) @ A
    ud = M0 * tg + M1 * 0.0f;
  }
  __device__ __forceinline__ void drift(const float x[2], float u, float dx[2]) const {
    dx[0] = (0.0f * x[0] + 1.0f * x[1]) + 0.0f * u;
    dx[1] = (a10 * x[0] + a11 * x[1]) + 1.0f * u;
  }
  __device__ __forceinline__ static void obs_transform(float y[2]) { (void)y; }
  __device__ __forceinline__ static bool bad(const float* s, int n) { return any_nonfinite(s, n); }
  __device__ __forceinline__ static Fit fit_init(bool active) { return Fit{!active, 0.0f}; }
  __device__ __forceinline__ void fit_update(Fit& f, int k, int S, const float* ts, float u, const float x[2]) const {
    (void)k; (void)S; (void)ts;
    const float Q[4] = {0.5f, 0.0f, 0.0f, 0.0f};
    const float e[2] = {x[0] - tg, x[1] - 0.0f};
    const float du = u - ud;
    f.F = f.F + (quad_form<2>(e, Q) + (du * 0.5f) * du);
  }
  __device__ __forceinline__ static void fit_kill(Fit& f) { f.settled = true; f.F = mtgp_qnan(); }
  __device__ __forceinline__ static float fit_final(Fit& f, int S) { (void)S; return f.F; }
};

// StirredTankReactor (reactor.py:7-81), state (Tc, T, c): k(T) = k0 exp(-Ea/R/T) with -Ea/R a
// Python float64 quotient rounded to f32, k0 = f32(7.2e10); control clipped to [0, 300]; the
// per-rollout quotients q/Vol, -dHr/Cp, UA/Vol/Cp, UA/Volc/Cp are formed once (same operations).
// Cost: x_d = [0, target, 0], Q = diag(0, 0.01, 0) (full 3x3), r = [[1e-4]].
struct EnvReactor {
  static constexpr int NV = 3;
  static constexpr bool kMask = false;
  float qV, Tf, mdHrCp, UAVCp, Volc, Tcf, UAVcCp, tg;
  typedef QuadFit Fit;
  __device__ __forceinline__ void load(const MtgpRollouts& ro, int rr, int nt) {
    const float* p = ro.params + 8 * rr;
    const float Vol = p[0], Cp = p[1], dHr = p[2], UA = p[3], q = p[4];
    Tf = p[5];
    Tcf = p[6];
    Volc = p[7];
    qV = q / Vol;
    mdHrCp = (-dHr) / Cp;
    UAVCp = (UA / Vol) / Cp;
    UAVcCp = (UA / Volc) / Cp;
    tg = ro.targets[rr * nt];
  }
  __device__ __forceinline__ void drift(const float x[3], float u, float dx[3]) const {
    const float Tc = x[0], T = x[1], c = x[2];
    const float control = mtgp_clip(u, 0.0f, 300.0f);
    const float kT = 7.2e10f * mtgp_expf((float)(-72750.0 / 8.314) / T);
    const float dc = qV * (1.0f - c) - kT * c;
    const float dT = (qV * (Tf - T) + (mdHrCp * kT) * c) + UAVCp * (Tc - T);
    const float dTc = (control / Volc) * (Tcf - Tc) + UAVcCp * (T - Tc);
    dx[0] = dTc;
    dx[1] = dT;
    dx[2] = dc;
  }
  __device__ __forceinline__ static void obs_transform(float y[3]) { (void)y; }
  __device__ __forceinline__ static bool bad(const float* s, int n) { return any_nonfinite(s, n); }
  __device__ __forceinline__ static Fit fit_init(bool active) { return Fit{!active, 0.0f}; }
  __device__ __forceinline__ void fit_update(Fit& f, int k, int S, const float* ts, float u, const float x[3]) const {
    (void)k; (void)S; (void)ts;
    const float Q[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.01f, 0.0f, 0.0f, 0.0f, 0.0f};
    const float e[3] = {x[0] - 0.0f, x[1] - tg, x[2] - 0.0f};
    f.F = f.F + (quad_form<3>(e, Q) + (u * 0.0001f) * u);
  }
  __device__ __forceinline__ static void fit_kill(Fit& f) { f.settled = true; f.F = mtgp_qnan(); }
  __device__ __forceinline__ static float fit_final(Fit& f, int S) { (void)S; return f.F; }
};

// store v at row `row` (wave-uniform element offset) + off (per lane): the 64-bit row base
// stays in SGPRs, only the 32-bit lane offset is a VGPR
// Trajectory rows are written once and never read by the kernel: non-temporal stores (`nt`), so
// the streaming output (C3: 2.3 GB, C5: 1.7 GB per launch) does not evict the JIT code and the
// rollout data from L2 -- C5's per-stage code footprint (~2 MB per XCD) is refetched every stage
// when it does (PMC: FETCH_SIZE 20 GB per launch with plain stores).
// The adaptive kernels' save points are divergent (each round writes one dword per lane into
// different rows), so their partial lines are left to L2 to merge: plain stores there
// (DP = true; non-temporal partial writes made the C3 Dopri5 kernel 44 % slower).
// Fixed-step kernels: the row is wave-uniform, so the store addresses a buffer resource at the row
// (SGPRs) plus the lane's byte offset (a VGPR) -- no per-store 64-bit VGPR address arithmetic; the
// resource's extent is the row (row_len elements), so a lane offset past it is dropped by the
// hardware instead of writing out of bounds.  off * 4 < 2^31 (checked by the entry point).

template <bool DP = false>
__device__ __forceinline__ void store_row(float* __restrict__ arr, size_t row, int off, float v, size_t row_len) {
#if MTGP_DEBUG_CHECKS
  if (off < 0 || (size_t)off >= row_len || row % row_len != 0) {
    dbg_count(0);
    return;
  }
#endif
  float* p = arr + row;
  if (!DP) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(row_len * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off * 4, 0, 2 /* nt */);
    return;
  }
  (void)row_len;
  p[off] = v;
}

// One trajectory element of an adaptive (Dopri5) kernel: save k, component c of nc, lane offset
// loff.  Time-major rows ([S][nc][P*R], store_row's plain-store form) or, with
// MtgpOutputs.traj_layout = MTGP_TRAJ_LANE_MAJOR, lane-major [P*R][S][nc] (the reference's
// [P, R, S, c] order): the save points of a Dopri5 wave are divergent, and a lane writing its own
// rows contiguously lets L2 merge its consecutive saves instead of leaving a partial line per
// store -- C3 Dopri5 write traffic 9.6 -> 4.6 GB (2.0x the trajectory bytes), kernel 20.6 -> 18.8 ms.
__device__ __forceinline__ void traj_put_dp(float* __restrict__ arr, bool lane_major, int k, int c, int nc, int loff,
                                            size_t PR, int S, float v) {
  if (lane_major) {
    const size_t at = ((size_t)loff * (size_t)S + (size_t)k) * (size_t)nc + (size_t)c;
#if MTGP_DEBUG_CHECKS
    if (loff < 0 || (size_t)loff >= PR || k < 0 || k >= S || c < 0 || c >= nc) {
      dbg_count(0);
      return;
    }
#endif
    arr[at] = v;
    return;
  }
  store_row<true>(arr, ((size_t)k * (size_t)nc + (size_t)c) * PR, loff, v, PR);
}

// --------------------------------------------------------------------------------------
// Wave layout.  A wave packs G = 64 / Rp individuals (Rp = the lane set: MtgpRollouts.lanes,
// by default R rounded up to a power of two): lane = g * Rp + r -> schedule slot q0 + g,
// rollout r; the individual at slot q is order[q] (identity without a schedule).  The
// environment (drift, observation, RK4 update, fitness) is lane-parallel and runs once for all
// G individuals; only the tree programs differ per individual, so they run once per group, each
// with a wave-uniform (scalar) instruction stream.  A half-empty wave costs as much as a full
// one on gfx950 (measured: R=32 and R=64 take the same time), so packing pays whenever the
// launch has more waves than the chip has SIMDs; below that the host widens the lane set
// (fewer individuals and program calls per wave, more waves).  A lane set wider than a wave
// (R > 64) spans W = lanes / 64 consecutive waves of one individual, wave `part` running
// rollouts [64 part, 64 part + 64); those waves share the individual's programs (and JIT unit).
struct Lane {
  int wave, lane, Rp, G, q0, g, r, p, rr;
  int W, part;  // waves per individual (1 unless R > 64) and this wave's part
  bool active;
  uint32_t ptab;  // lane gi (< G): byte offset of group gi's program block in A.prog
  uint32_t jtab;  // lane j < n_prog: JIT code offset of this wave's program-j unit
  bool jok;       // the JIT code of this launch is complete (plan status 0, fits the buffer)
};

// program-block offsets of the wave's groups, one per lane (read back with v_readlane)
__device__ __forceinline__ uint32_t prog_table(const KArgs& A, const Lane& L) {
  const int q = L.q0 + L.lane;
  const int ind = (L.lane < L.G && q < A.P) ? (A.ro.order ? A.ro.order[q] : q) : 0;
  return (uint32_t)ind * (uint32_t)A.n_prog * (uint32_t)A.L * (uint32_t)sizeof(MtgpInstr);
}

__device__ __forceinline__ int sched_ind(const KArgs& A, int q) { return A.ro.order ? A.ro.order[q] : q; }

// lanes per individual of this launch (MtgpRollouts.lanes, default R rounded up to a power of two)
__device__ __forceinline__ int lane_set(const MtgpRollouts& ro) {
  if (ro.lanes > 0) return ro.lanes;
  int Rp = 1;
  while (Rp < ro.R) Rp <<= 1;
  return Rp;
}

// wave `wv` of the launch (or lane set `wv` of a workgroup-per-lane-set kernel) -> L.q0 / g / r
__device__ __forceinline__ void lane_place(const KArgs& A, Lane& L, int wv) {
  const int set = uni(lane_set(A.ro));
  if (set <= kWave) {
    L.Rp = set;
    L.G = uni(kWave / set);
    L.W = 1;
    L.part = 0;
    L.q0 = uni(wv * L.G);
    L.g = L.lane / L.Rp;
    L.r = L.lane - L.g * L.Rp;
  } else {
    L.Rp = kWave;
    L.G = 1;
    L.W = uni(set / kWave);
    L.q0 = uni(wv / L.W);
    L.part = uni(wv - L.q0 * L.W);
    L.g = 0;
    L.r = L.part * kWave + L.lane;
  }
}

// wv < 0: this wave's own index in the launch
__device__ __forceinline__ bool lane_setup(const KArgs& A, Lane& L, int wv = -1) {
  L.wave = uni(threadIdx.x >> 6);
  L.lane = threadIdx.x & 63;
  lane_place(A, L, wv >= 0 ? wv : (int)blockIdx.x * kWavesPerBlock + L.wave);
  if (L.q0 >= A.P) return false;
  const int q = L.q0 + L.g;
  L.p = q < A.P ? sched_ind(A, q) : A.P;  // A.P marks a padding group
  L.active = (L.r < A.ro.R) && (q < A.P);
  L.rr = L.active ? L.r : 0;
  L.ptab = prog_table(A, L);
  L.jok = true;
  if (A.jit_info)  // checked on the device, so the host never waits for the plan
    L.jok = uni((int)(A.jit_info[0] == 0 && (uint64_t)(uint32_t)A.jit_info[1] <= A.jit_cap)) != 0;
  L.jtab = 0;
  if (A.jit_off && L.lane < A.n_prog) L.jtab = A.jit_off[(size_t)(L.q0 / L.G) * A.n_prog + L.lane];
  return true;
}

// number of groups of this wave that hold a real individual
__device__ __forceinline__ int groups_live(const KArgs& A, const Lane& L) {
  const int n = A.P - L.q0;
  return uni(n < L.G ? n : L.G);
}

// individual of group gi (wave-uniform)
__device__ __forceinline__ int group_ind(const KArgs& A, const Lane& L, int gi) {
  return uni(sched_ind(A, L.q0 + gi));
}

// The fixed-step solve (include/mtgp_cstep.h): diffrax.ConstantStepSize's accumulated step grid,
// wave-uniform because ts is shared by every rollout (dyn.py:63).  t, tn, dt are computed by every
// lane from the same uniform inputs; the loop and save tests go through readfirstlane so that the
// branches stay scalar.
struct CsClock {
  float t, tn, t_end, dt0;
  int steps, max_steps;
  __device__ __forceinline__ void init(const KArgs& A) {
    t = ldc(A.ro.ts, 0);
    t_end = ldc(A.ro.ts, A.m.n_save - 1);
    dt0 = A.m.h;
    tn = mtgp_cs_first_end(t, dt0, t_end);
    steps = 0;
    max_steps = A.m.max_steps;
  }
  __device__ __forceinline__ bool live() const {
    return uni((int)(t < t_end && mtgp_cs_advancing(steps, t, tn) && (max_steps <= 0 || steps < max_steps))) != 0;
  }
  __device__ __forceinline__ float dt() const { return tn - t; }
  __device__ __forceinline__ void advance() {
    ++steps;
    t = tn;
    tn = mtgp_cs_next_end(t, dt0, t_end);
  }
  // save point k is taken in this step (ts[k] <= tn; k < S checked by the caller)
  __device__ __forceinline__ bool saves(const float* ts, int k) const { return uni((int)(ldc(ts, k) <= tn)) != 0; }
};

// RK4 stage input (stage 0: s itself; stages 1..3: s + (sum_j a_ij f_j) dt over the padded tableau
// row, zero entries multiplied: mtgp_cstep.h) from f = the previous stage's derivative and acc = the
// running b-weighted sum BEFORE f's term is added (mtgp_rk4_in_acc: no zero-entry sum carried), and
// the running b-weighted sum of the stage derivatives
__device__ __forceinline__ float stage_in(int stage, float s, float f, float acc, float dt) {
  return stage == 0 ? s : mtgp_rk4_in_acc(stage, s, f, acc, dt);
}
__device__ __forceinline__ float stage_acc(int stage, float acc, float f) { return mtgp_rk4_acc(stage, acc, f); }
__device__ __forceinline__ float stage_time(int stage, float t, float dt) {
  return stage == 0 ? t : mtgp_rk4_time(stage, t, dt);
}

// The same for a whole state vector, branching on the (wave-uniform) stage once instead of
// selecting per component: the same operations, so the same bits.
template <int N>
__device__ __forceinline__ void stage_in_n(int stage, const float (&s)[N], const float (&f)[N], const float (&acc)[N],
                                           float dt, float (&out)[N]) {
  const int st = uni(stage);
  if (st == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = s[i];
  } else if (st == 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = mtgp_rk4_in_acc(1, s[i], f[i], acc[i], dt);
  } else if (st == 2) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = mtgp_rk4_in_acc(2, s[i], f[i], acc[i], dt);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = mtgp_rk4_in_acc(3, s[i], f[i], acc[i], dt);
  }
}
template <int N>
__device__ __forceinline__ void stage_acc_n(int stage, float (&acc)[N], const float (&f)[N]) {
  const int st = uni(stage);
  if (st == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = mtgp_rk4_acc(0, 0.0f, f[i]);
  } else if (st == 3) {
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = mtgp_rk4_acc(3, acc[i], f[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = mtgp_rk4_acc(1, acc[i], f[i]);
  }
}
// the state at save time th of the step [y, y1] (RK4: the Hermite cubic from the increments f0 dt,
// f3 dt; Euler: linear), +inf once the solve has ended (dead)
template <int N>
__device__ __forceinline__ void cs_dense(bool euler, bool dead, const float (&y)[N], const float (&y1)[N],
                                         const float (&f0)[N], const float (&f3)[N], float dt, float th,
                                         float (&out)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float v = euler ? mtgp_cs_linear(y[i], y1[i], th) : mtgp_cs_hermite(y[i], y1[i], f0[i] * dt, f3[i] * dt, th);
    out[i] = dead ? kInf : v;
  }
}

// --------------------------------------------------------------------------------------
// The data vector a tree reads and its operand stack.  Interpreter: one LDS column per slot
// (dcol, st).  JIT: the slots live in VGPRs v[] that the call site pins to v0-v7
// (mtgp_jit.h register ABI); the LDS columns are only filled for an interpreter fallback.
template <bool JIT>
struct DataVec {
  float* dcol;
  float* st;
  float v[kDMax];
  __device__ __forceinline__ DataVec(float* d, float* s) : dcol(d), st(s) {
#pragma unroll
    for (int k = 0; k < kDMax; ++k) v[k] = 0.0f;
  }
  __device__ __forceinline__ void put(int slot, float x) {
    if (JIT) v[slot] = x;  // (the register copy only feeds JIT calls: no dynamic index otherwise)
    if (!JIT) dcol[slot * kWave] = x;
  }
  __device__ __forceinline__ void spill() {
#pragma unroll
    for (int k = 0; k < kDMax; ++k) dcol[k * kWave] = v[k];
  }
};

// Call a JIT unit at `addr` (mtgp_jit.h ABI): data in v0-v7; a single-program role returns in
// v8, a multi-program role in v25.. ; s[32:33] collects lanes that need the interpreter (slow
// sin/cos reduction).
__device__ __forceinline__ float jit_call(uint64_t addr_, const float d[kDMax], uint64_t& flag) {
  // the target must sit in SGPRs: make its uniformity explicit to the compiler
  const uint64_t addr = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)addr_) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(addr_ >> 32)) << 32;
  float acc;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "={v8}"(acc), "+{s[32:33]}"(flag)
               : [tgt] "s"(addr), "{v0}"(d[0]), "{v1}"(d[1]), "{v2}"(d[2]), "{v3}"(d[3]), "{v4}"(d[4]),
                 "{v5}"(d[5]), "{v6}"(d[6]), "{v7}"(d[7])
               : "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v25", "s30", "s31", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41",
                 "s42", "s43", "s44", "s45", "vcc", "scc", "memory");  // (SCC: the templates' and merges' SALU ops)
  return acc;
}

// Call a role chain (mtgp_jit.h jit_unit_end, ABI v13): the chain's programs return in v26..v29
// (position order), and with cont != 0 the optional continuation (the save-point readout)
// runs too and returns in v8.
struct ChainOut {
  float v[mtgp::kJitChainMax];
  float tail;
};
__device__ __forceinline__ ChainOut jit_call_chain(uint64_t addr_, const float d[kDMax], uint64_t& flag, int cont) {
  const uint64_t addr = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)addr_) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(addr_ >> 32)) << 32;
  const int c = __builtin_amdgcn_readfirstlane(cont);
  ChainOut r;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "={v8}"(r.tail), "={v26}"(r.v[0]), "={v27}"(r.v[1]), "={v28}"(r.v[2]), "={v29}"(r.v[3]),
                 "+{s[32:33]}"(flag)
               : [tgt] "s"(addr), "{s46}"(c), "{v0}"(d[0]), "{v1}"(d[1]), "{v2}"(d[2]), "{v3}"(d[3]),
                 "{v4}"(d[4]), "{v5}"(d[5]), "{v6}"(d[6]), "{v7}"(d[7])
               : "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v25", "s30", "s31", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41",
                 "s42", "s43", "s44", "s45", "vcc", "scc", "memory");
  return r;
}

// The interpreter as an out-of-line function for the JIT kernels' fallback sites (lanes that need
// the slow sin/cos reduction, populations without usable code).  Inlined, its dispatch trees
// make the C3 kernel 190 KB of code (19 KB out of line), but the call costs more than the
// instruction fetch it saves: the call ABI spills SGPRs into VGPR lanes and a few VGPRs to
// scratch inside the stage loop.  A/B in one process (profiles/r03/v5_ab_cold.log): C3 kernel
// 2.60 ms out of line vs 2.30 inline, C2 1.06 vs 0.91, C5 7.51 vs 7.14.  Kept inline
// (MTGP_COLD_INTERP = 0, mtgp_ab.h).  The Dopri5 kernels (two waves per SIMD, 183 VGPRs) can take
// the fallback out of line too (MTGP_DP_COLD); measured on C3 Dopri5 (profiles/r03/v8_dptail.log vs
// v6): full population 21.4 vs 20.2 ms, a lone tail wave 10.6 vs 9.9 us per attempt -- inline kept.
typedef __attribute__((address_space(3))) float LdsFloat;
__device__ __attribute__((noinline)) float run_prog_cold(const MtgpInstr* code, uint32_t dcol_lds, uint32_t st_lds) {
  const float* dcol = (const float*)(LdsFloat*)(uintptr_t)dcol_lds;
  float* st = (float*)(LdsFloat*)(uintptr_t)st_lds;
  return run_prog(code, dcol, st);
}
__device__ __forceinline__ uint32_t lds_addr_of(const float* p) {
  return (uint32_t)(uintptr_t)(const LdsFloat*)p;
}

// Run program `slot` of group gi (its individual's program, wave-uniform).  COLD: out of line.
template <bool COLD = false>
__device__ __forceinline__ float run_one_interp(const KArgs& A, const Lane& L, int gi, int slot, const float* dcol,
                                                float* st) {
  const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)L.ptab, gi) +
                       (uint32_t)slot * (uint32_t)A.L * (uint32_t)sizeof(MtgpInstr);
  const MtgpInstr* code = (const MtgpInstr*)((const char*)A.prog + off);
  if (COLD) return run_prog_cold(code, lds_addr_of(dcol), lds_addr_of(st));
  return run_prog(code, dcol, st);
}

// interpreter: program `slot` of every live group on explicit LDS columns
template <bool COLD = false>
__device__ __forceinline__ float run_groups_interp(const KArgs& A, const Lane& L, int ng, int slot, const float* dcol,
                                                   float* st, float dflt) {
  float v = dflt;
  for (int gi = 0; gi < ng; ++gi) {
    const float t = run_one_interp<COLD>(A, L, gi, slot, dcol, st);
    v = (L.g == gi) ? t : v;
  }
  return v;
}

// Programs first .. first+M-1 of every live group -> out[0..M-1], each lane its own
// individual's values.  JIT: one call per program to the wave's unit (mtgp_jit.h jit_unit);
// the interpreter runs when there is no usable code or when a lane needs the slow sin/cos path.
// chained: the role's code is one chain (A.chain_state, mtgp_jit.h jit_unit_end); with save_prog
// >= 0 the chain's continuation (program save_prog, the save-point readout) runs too -> *save_v.
#if MTGP_AB_FBCOUNT  // diagnostic: JIT calls with / without slow sin/cos lanes (chain, single)
__device__ unsigned long long g_ab_fb_count[4];
#endif
template <bool JIT, int M, bool COLD = (MTGP_COLD_INTERP != 0)>
__device__ __forceinline__ void run_role(const KArgs& A, const Lane& L, int ng, int role, int first, DataVec<JIT>& D,
                                         float (&out)[M], bool chained = false, int save_prog = -1,
                                         float* save_v = nullptr, int mr = M) {
  (void)role;
  bool interp = !JIT;
  if (JIT && M <= mtgp::kJitChainMax && chained) {
    if (__builtin_expect(L.jok, 1)) {
      const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)L.jtab, first);
      uint64_t fl = 0;
#if MTGP_AB_NOPROG  // diagnostic only (A/B): no program call at all
      (void)off;
      const ChainOut r = {{0.0f, 0.0f, 0.0f, 0.0f}, 0.0f};
#else
      const ChainOut r = jit_call_chain(A.jit_base + off, D.v, fl, save_prog >= 0 ? 1 : 0);
#endif
#pragma unroll
      for (int j = 0; j < M; ++j) out[j] = r.v[j < mtgp::kJitChainMax ? j : 0];
      if (save_prog >= 0) *save_v = r.tail;
#if MTGP_AB_FBCOUNT
      if (fl != 0 && L.lane == 0) atomicAdd(&g_ab_fb_count[0], 1ull);
      if (L.lane == 0) atomicAdd(&g_ab_fb_count[1], 1ull);
#endif
      if (!MTGP_AB_NOFALLBACK && __builtin_expect(fl != 0, 0)) {  // slow sin/cos lanes: re-run the chain's
        bool spilled = false;                                      // programs for the groups concerned
        for (int gi = 0; gi < ng; ++gi) {
          if (!(fl & __ballot(L.g == gi && L.active))) continue;
          if (!spilled) { D.spill(); spilled = true; }
#pragma unroll
          for (int j = 0; j < M; ++j) {
            const float t = run_one_interp<JIT && COLD>(A, L, gi, first + j, D.dcol, D.st);
            out[j] = (L.g == gi) ? t : out[j];
          }
          if (save_prog >= 0) {
            const float t = run_one_interp<JIT && COLD>(A, L, gi, save_prog, D.dcol, D.st);
            *save_v = (L.g == gi) ? t : *save_v;
          }
        }
      }
      return;
    }
    interp = true;
    D.spill();
  } else if (JIT) {
    if (__builtin_expect(L.jok, 1)) {
#pragma unroll 1
      for (int q = 0; q < M; ++q) {
        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)L.jtab, first + q);
        uint64_t fl = 0;
#if MTGP_AB_NOPROG  // diagnostic only: the environment without any program call (A/B), never shipped
        (void)off;
        float v = 0.0f;
#else
        float v = jit_call(A.jit_base + off, D.v, fl);
#endif
#if MTGP_AB_FBCOUNT
        if (fl != 0 && L.lane == 0) atomicAdd(&g_ab_fb_count[2], 1ull);
        if (L.lane == 0) atomicAdd(&g_ab_fb_count[3], 1ull);
#endif
        if (!MTGP_AB_NOFALLBACK && __builtin_expect(fl != 0, 0)) {  // lanes that need the slow sin/cos: re-run only
          bool spilled = false;               // this program, only for the groups concerned
          for (int gi = 0; gi < ng; ++gi) {
            if (!(fl & __ballot(L.g == gi && L.active))) continue;
            if (!spilled) { D.spill(); spilled = true; }
            const float t = run_one_interp<JIT && COLD>(A, L, gi, first + q, D.dcol, D.st);
            v = (L.g == gi) ? t : v;
          }
        }
#pragma unroll
        for (int j = 0; j < M; ++j) out[j] = (q == j) ? v : out[j];
      }
    } else {
      interp = true;
    }
    if (interp) D.spill();
  }
  if (interp && !(JIT && MTGP_AB_NOINTERP)) {
#pragma unroll 1
    for (int q = 0; q < mr; ++q) {  // mr <= M: a runtime role size (state_size > 3, interpreter only)
      const float v = run_groups_interp<JIT && COLD>(A, L, ng, first + q, D.dcol, D.st, 0.0f);
#pragma unroll
      for (int j = 0; j < M; ++j) out[j] = (q == j) ? v : out[j];
    }
    if (save_prog >= 0) *save_v = run_groups_interp<JIT && COLD>(A, L, ng, save_prog, D.dcol, D.st, 0.0f);
  }
}



// Programs first .. first+mr-1 of every live group -> out[0..mr-1] from LDS-data JIT code (mtgp_jit.h
// kJitModeLds: v0 = this lane's LDS byte address of data slot 0, the interpreter's own data
// columns): the runtime-state-size control kernels (round 6), one unit call per program; the
// interpreter for lanes that need it (no template sets that flag) and for unusable code.
__device__ __forceinline__ uint32_t lds_address(const float* p);
__device__ __forceinline__ float jit_call_lds(uint64_t addr_, uint32_t lds_addr, uint64_t& flag);
template <int M>
__device__ __forceinline__ void run_role_lds(const KArgs& A, const Lane& L, int ng, int first, float* dcol, float* st,
                                             float (&out)[M], int mr = M) {
  if (__builtin_expect(L.jok, 1)) {
    const uint32_t la = lds_address(dcol);
#pragma unroll 1
    for (int q = 0; q < mr; ++q) {
      const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)L.jtab, first + q);
      uint64_t fl = 0;
      float v = jit_call_lds(A.jit_base + off, la, fl);
      if (__builtin_expect(fl != 0, 0)) {
        for (int gi = 0; gi < ng; ++gi) {
          if (!(fl & __ballot(L.g == gi && L.active))) continue;
          const float t = run_one_interp<MTGP_COLD_INTERP != 0>(A, L, gi, first + q, dcol, st);
          v = (L.g == gi) ? t : v;
        }
      }
#pragma unroll
      for (int j = 0; j < M; ++j) out[j] = (q == j) ? v : out[j];
    }
    return;
  }
#pragma unroll 1
  for (int q = 0; q < mr; ++q) {
    const float v = run_groups_interp<MTGP_COLD_INTERP != 0>(A, L, ng, first + q, dcol, st, 0.0f);
#pragma unroll
    for (int j = 0; j < M; ++j) out[j] = (q == j) ? v : out[j];
  }
}

__device__ __forceinline__ void finish_group(const KArgs& A, const Lane& L, float F) {
  const float mx = A.m.max_fitness;
  if (A.out.rollout_fitness && L.active) A.out.rollout_fitness[(size_t)L.p * A.ro.R + L.r] = F;
  if (L.W > 1) return;  // lane set over several waves: k_rollout_mean forms the fitness
  float v = L.active ? (mtgp_isfinite(F) ? F : mx) : 0.0f;
  // xor butterfly inside the group == pairwise tree in rollout order (mirrored by the oracle)
  for (int w = 1; w < L.Rp; w <<= 1) v = v + __shfl_xor(v, w, kWave);
  if (L.r == 0 && L.p < A.P) {
    float mean = v / (float)A.ro.R;
    mean = mean < 0.0f ? 0.0f : (mean > mx ? mx : mean);
    A.out.fitness[L.p] = mean + A.m.parsimony * (float)A.nodes[L.p];
  }
}

// Fitness of individuals whose lane set spans several waves (R > 64): the same sum as
// finish_group's butterfly -- per chunk of 64 rollouts the pairwise tree in rollout order (zeros
// past R), then the pairwise tree over the chunks padded to a power of two (the oracle's
// pairwise_sum) -- from the raw per-rollout fitness, then mean, clip and parsimony.  One thread
// per individual; the pairwise trees are formed with a binary-counter stack.
__global__ void __launch_bounds__(256) k_rollout_mean(const float* __restrict__ rf, int P, int R, float mx,
                                                      float parsimony, const int32_t* __restrict__ nodes,
                                                      float* __restrict__ fitness) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float* v = rf + (size_t)p * R;
  const int nch = (R + kWave - 1) / kWave;
  int np2 = 1;
  while (np2 < nch) np2 <<= 1;
  float cst[24];
  for (int c = 0; c < np2; ++c) {
    float lst[8];
    float sum = 0.0f;
    for (int l = 0; l < kWave; ++l) {
      const int r = c * kWave + l;
      float x = (c < nch && r < R) ? v[r] : 0.0f;
      if (c < nch && r < R && !mtgp_isfinite(x)) x = mx;
      int lvl = 0;
      for (; (l >> lvl) & 1; ++lvl) x = lst[lvl] + x;
      lst[lvl] = x;
      sum = x;  // after l = 63 the top of the stack holds the chunk's sum
    }
    float x = sum;
    int lvl = 0;
    for (; (c >> lvl) & 1; ++lvl) x = cst[lvl] + x;
    cst[lvl] = x;
  }
  int top = 0;
  while ((1 << top) < np2) ++top;
  float mean = cst[top] / (float)R;
  mean = mean < 0.0f ? 0.0f : (mean > mx ? mx : mean);
  fitness[p] = mean + parsimony * (float)nodes[p];
}

// --------------------------------------------------------------------------------------
// The JIT-only stage loop of the fixed-step dynamic policy (round 4).  The JIT's sin/cos/division
// templates compute every lane themselves (the spec's slow reductions included: s[32:33] is never
// set, gen_jit_templates.py), so once the launch's code is usable (Lane.jok) no lane ever needs the
// interpreter: this loop carries no interpreter code at all, its RK4 stages are unrolled (stage
// constants and branches resolved at compile time), and the kernel runs the general loop below only
// when the code is not usable.  The arithmetic is k_ctl_dynamic's, operation for operation.
template <int N>
__device__ __forceinline__ void rk_in(int st, const float (&s)[N], const float (&f)[N], const float (&acc)[N], float dt,
                                      float (&out)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = st == 0 ? s[i] : mtgp_rk4_in_acc(st, s[i], f[i], acc[i], dt);
}
template <int N>
__device__ __forceinline__ void rk_acc(int st, float (&acc)[N], const float (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) acc[i] = mtgp_rk4_acc(st, acc[i], f[i]);
}

// one JIT unit call, no fallback (the templates never request one)
__device__ __forceinline__ float jit_call_nf(uint64_t addr_, const float d[kDMax]) {
  uint64_t fl = 0;
  return jit_call(addr_, d, fl);
}
__device__ __forceinline__ ChainOut jit_call_chain_nf(uint64_t addr_, const float d[kDMax], int cont) {
  uint64_t fl = 0;
  return jit_call_chain(addr_, d, fl, cont);
}

// Fair share of a SIMD's issue slots.  The SQ issues the oldest ready wave first, so of the four
// waves a SIMD holds the oldest runs ahead and the youngest finishes long after it, alone on the
// SIMD for its last stretch (profiles/r05 wavetime: residency 0.67, durations 0.69-1.50x the mean).
// Each wave posts its step count to a per-SIMD table (HW_ID / XCC_ID) and reads the others' posts
// of one step ago; a wave more than `margin` steps ahead of the slowest lowers its priority.
// Measured (profiles/r05/v12_ab_fair.log, A/B in one process): C3 kernel 2.17 -> 1.81 ms, results
// bit-identical (priorities only reorder issue).
// Table layout (round 6): one 128-B L2 line per SIMD, 16 posts of {launch tag : 32, step : 32}.
// Every wave that reads or writes a SIMD's line runs on that SIMD, i.e. on one CU of one XCD, so
// the posts never need to leave the XCD's L2: a non-temporal vector store (write-through L1, the
// line stays in L2) and sc1 loads (bypass this CU's L1, served by L2).  The round-5 form -- agent-scope atomic
// stores, which drop the line from L2 -- sent every post and every read to memory: 105 MB of
// FETCH and 25 MB of WRITE per C3 launch (profiles/r06/v1_pmc_fair{0,3}_*.json).
static __device__ uint64_t g_fair[8 * 8 * 2 * 16 * 4 * 16];
struct FairShare {
  uint64_t* tab;
  uint64_t seen;
  uint32_t slot, tag;
  int margin, mode, level;
  __device__ void init(const KArgs& A, int setting = -1) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)) & 7u;  // HW_REG_XCC_ID
    const uint32_t key = (((xcc * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) * 4u +
                         ((hw >> 4) & 3u);
    tab = g_fair + (size_t)key * 16u;
    slot = hw & 15u;
    tag = A.epoch;
    margin = (setting < 0 ? A.fair : setting) - 1;
    mode = A.fair_mode;
    seen = 0u;
    level = 2;
    __builtin_amdgcn_s_setprio(2);
  }
  __device__ __forceinline__ void step(int lane, uint32_t st) {
    const bool valid = lane < 16 && (uint32_t)(seen >> 32) == tag && (uint32_t)lane != slot;
    int m = valid ? (int)(uint32_t)seen : 0x7fffffff;
#pragma unroll
    for (int w = 1; w < 16; w <<= 1) {
      const int o = __shfl_xor(m, w, kWave);
      m = o < m ? o : m;
    }
    const int mn = __builtin_amdgcn_readfirstlane(m);
    const int lv = mn == 0x7fffffff ? 2 : ((int)st > mn + margin ? 0 : ((mode == 1 && (int)st <= mn) ? 3 : 2));
    if (lv != level) {  // (s_setprio takes an immediate)
      if (lv == 0) __builtin_amdgcn_s_setprio(0);
      else if (lv == 2) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(3);
      level = lv;
    }
    // a non-temporal vector store: write-through L1, the line stays in L2 (a volatile store is sc0 sc1,
    // an atomic one drops the line: both sent every read of the post to memory, profiles/r06/v2_*)
    if (lane == 0) __builtin_nontemporal_store((uint64_t)tag << 32 | st, tab + slot);
    if (lane < 16) seen = __hip_atomic_load(tab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: L2
  }
};

// The fixed-step dynamic policy with usable JIT code (see above), diffrax ConstantStepSize semantics
// (include/mtgp_cstep.h): per step the NST stages at t + c_i dt, then the step's end state, the
// event test, and every save point ts[k] <= tn of the step through the dense output -- observation
// at ts[k] (dyn.py:99), the save-point readout on [y, a, 0, tar] (dyn.py:101), fitness, rows.
template <class Env, int NA, bool TRAJ, bool NOISE, int NST>
__device__ __forceinline__ void ctl_dynamic_jit(const KArgs& A, const Lane& Ln) {
  constexpr int NV = Env::NV;
  const int r = Ln.r, rr = Ln.rr;
  const bool active = Ln.active;
  const int R = A.ro.R;
  const int S = A.m.n_save;
  const float* __restrict__ ts = A.ro.ts;
  ObsNoise<NV> nzc;
  float nzv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) nzv[i] = 0.0f;
  uint32_t nzt = 0xffffffffu;  // bits of the time nzv was drawn at (a NaN pattern: none yet)
  if (NOISE) nzc = obs_noise_setup<NV>(A.m, A.ro, rr);
  constexpr int uslot = NV + NA;
  Env env;
  env.load(A.ro, rr, A.m.n_targets);
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  float dv[kDMax];
#pragma unroll
  for (int k = 0; k < kDMax; ++k) dv[k] = 0.0f;
#pragma unroll
  for (int t = 0; t < kDMax - NV - 2; ++t)
    if (t < A.m.n_targets && uslot + 1 + t < kDMax) dv[uslot + 1 + t] = A.ro.targets[rr * A.m.n_targets + t];
  // code addresses of this wave's units (wave-uniform): the readout -> state put chain, the save readout
  const uint64_t u_readout = A.jit_base + (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_readout);
  const uint64_t u_save = A.jit_base + (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_readout_save);

  float x[NV], a[NA], kx[NV], ka[NA], fx0[NV], fa0[NA], ax[NV], aa[NA];
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = A.ro.x0[rr * NV + i];
#pragma unroll
  for (int j = 0; j < NA; ++j) a[j] = ka[j] = aa[j] = fa0[j] = 0.0f;
#pragma unroll
  for (int i = 0; i < NV; ++i) kx[i] = ax[i] = fx0[i] = 0.0f;

  typename Env::Fit fit = Env::fit_init(active);
  bool dead = !active, prev_ok;
  {
    float s0[NV + NA];
#pragma unroll
    for (int i = 0; i < NV; ++i) s0[i] = x[i];
#pragma unroll
    for (int j = 0; j < NA; ++j) s0[NV + j] = a[j];
    prev_ok = !Env::bad(s0, NV + NA);
  }
  // one save point: state (xs, as) at ts[k]; fill = a point of the +inf fill after the solve ended
  auto save_point = [&](int k, const float (&xs)[NV], const float (&as)[NA], bool fill) __attribute__((always_inline)) {
    float yo[NV];
    if (NOISE) {
      const uint32_t tb = __float_as_uint(ldc(ts, k));
      if (tb != nzt) {  // (the noise of ts[k] is drawn unless the last stage was at that very time)
        obs_noise_vec<NV>(nzc, ldc(ts, k), nzv);
        nzt = tb;
      }
    }
    ctl_obs_apply<Env>(xs, nzv, yo);  // f_obs(key, (ts[k], xs[k])), dyn.py:99
#pragma unroll
    for (int i = 0; i < NV; ++i) dv[i] = yo[i];
#pragma unroll
    for (int j = 0; j < NA; ++j) dv[NV + j] = as[j];
    const float us = jit_call_nf(u_save, dv);  // readout([y, a, 0, tar]), dyn.py:101 (u folded to 0)
    if constexpr (Env::kMask) {
      if (active) env.fit_save(fit, k, S, A, PR, loff, fill, us, xs);
    } else if (!fill && !MTGP_AB_NOFIT) {
      env.fit_update(fit, k, S, ts, us, xs);
    }
    if (TRAJ && active && !MTGP_AB_NOSTORE) {
      if (A.out.xs) {
#pragma unroll
        for (int i = 0; i < NV; ++i) store_row(A.out.xs, ((size_t)k * NV + i) * PR, loff, xs[i], PR);
      }
      if (A.out.ys) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < A.m.n_obs) store_row(A.out.ys, ((size_t)k * A.m.n_obs + i) * PR, loff, yo[i], PR);
      }
      if (A.out.us) store_row(A.out.us, (size_t)k * PR, loff, us, PR);
      if (A.out.acts) {
#pragma unroll
        for (int j = 0; j < NA; ++j) store_row(A.out.acts, ((size_t)k * NA + j) * PR, loff, as[j], PR);
      }
    }
  };

  CsClock clk;
  clk.init(A);
  int k = 0;  // next save point
  const bool fair_on = uni(A.fair) != 0;
  FairShare fair;
  if (fair_on) fair.init(A);
  while (clk.live()) {
    if (fair_on) fair.step(Ln.lane, (uint32_t)clk.steps);
    const float t = clk.t, dt = clk.dt();
    // one RK stage (NST = 4) or the Euler step (NST = 1); ST is a compile-time constant.  The
    // stage input reads the b-weighted sum before f_{ST-1}'s term (mtgp_rk4_in_acc: the zero
    // tableau entries, mtgp_cstep.h), which is then added -- the same sums in the same order.
    auto stage = [&](auto st_c) {
      constexpr int ST = decltype(st_c)::value;
      float xt[NV], at[NA], y[NV];
      rk_in<NV>(ST, x, kx, ax, dt, xt);
      rk_in<NA>(ST, a, ka, aa, dt, at);
      if (NST == 4 && ST > 0) {
        rk_acc<NV>(ST - 1, ax, kx);
        rk_acc<NA>(ST - 1, aa, ka);
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) dv[NV + j] = at[j];
      if (NOISE && ST != 2) {  // stages 1 and 2 share the time t + dt/2, hence the noise draw
        const float tc = ST == 0 ? t : mtgp_rk4_time(ST, t, dt);
        obs_noise_vec<NV>(nzc, tc, nzv);
        nzt = __float_as_uint(tc);
      }
      // one call: the readout (y, u folded: reads [0, a, 0, tar]) returns u in v26, and the state
      // programs it falls into read their u slot from there ([y, a, u, tar]) -- MtgpJitChain.put
      ctl_obs_apply<Env>(xt, nzv, y);
#pragma unroll
      for (int i = 0; i < NV; ++i) dv[i] = y[i];
      const ChainOut c = jit_call_chain_nf(u_readout, dv, 0);
#pragma unroll
      for (int j = 0; j < NA; ++j) ka[j] = c.v[1 + j < mtgp::kJitChainMax ? 1 + j : 0];
      env.drift(xt, c.v[0], kx);
      if (ST == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) fx0[i] = kx[i];
#pragma unroll
        for (int j = 0; j < NA; ++j) fa0[j] = ka[j];
      }
    };
    stage(std::integral_constant<int, 0>{});
    if constexpr (NST == 4) {
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      rk_acc<NV>(3, ax, kx);
      rk_acc<NA>(3, aa, ka);
    }
    // the step's end state and the event (Event(cond_fn_nan) after the step, dyn.py:94)
    float x1[NV], a1[NA];
#pragma unroll
    for (int i = 0; i < NV; ++i) x1[i] = NST == 1 ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
#pragma unroll
    for (int j = 0; j < NA; ++j) a1[j] = NST == 1 ? a[j] + fa0[j] * dt : mtgp_rk4_out(a[j], aa[j], dt);
    bool ev = false;
    if (!dead) {
      float sn[NV + NA];
#pragma unroll
      for (int i = 0; i < NV; ++i) sn[i] = x1[i];
#pragma unroll
      for (int j = 0; j < NA; ++j) sn[NV + j] = a1[j];
      const bool ok = !Env::bad(sn, NV + NA);
      ev = prev_ok && !ok;
      prev_ok = ok;
    }
    // SaveAt(ts): every pending ts[k] <= tn through this step's dense output
    while (k < S && clk.saves(ts, k)) {
      const float th = mtgp_cs_rescale(t, ldc(ts, k), clk.tn);
      float xs[NV], as[NA];
      cs_dense<NV>(NST == 1, dead, x, x1, fx0, kx, dt, th, xs);
      cs_dense<NA>(NST == 1, dead, a, a1, fa0, ka, dt, th, as);
      save_point(k, xs, as, dead);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = x1[i];
#pragma unroll
      for (int j = 0; j < NA; ++j) a[j] = a1[j];
    }
    if (ev) {  // the solve ends: later save points are the +inf fill
      dead = true;
      if (k < S) Env::fit_kill(fit);
    }
    clk.advance();
    if (!TRAJ && wave_all(fit.settled || dead)) break;
  }
  if (k < S) {  // unsaved points (event everywhere / max_steps): +inf (throw=False)
    if (!fit.settled) Env::fit_kill(fit);
    if (TRAJ) {
      float xs[NV], as[NA];
#pragma unroll
      for (int i = 0; i < NV; ++i) xs[i] = kInf;
#pragma unroll
      for (int j = 0; j < NA; ++j) as[j] = kInf;
      for (; k < S; ++k) save_point(k, xs, as, true);
    }
  }
  finish_group(A, Ln, Env::fit_final(fit, S));
}

// --------------------------------------------------------------------------------------
// Dynamic symbolic policy (dynamic_evaluate.py:65-118) on environment Env.  NA = state_size.
// Data slots: y 0..NV-1 | a NV..NV+NA-1 | u NV+NA | targets.  Per stage the programs run in
// the order of _drift (dyn.py:107-118): readout (y, u folded to 0) -> drift -> f_obs ->
// state equations; at save points the save-time readout (dyn.py:101) is appended.
// NOISE: observation noise on; the save-point observation uses ts[k] (dyn.py:99), which is
// recomputed when it differs from the stage-0 time of that step.
#if MTGP_AB_WAVETIME
// diagnostic build only: per wave (grid order) its start / end shader clock and HW_ID / XCC_ID
constexpr int kWaveTimeMax = 1 << 15;
__device__ unsigned long long g_wave_time[kWaveTimeMax * 2];
__device__ unsigned int g_wave_hw[kWaveTimeMax * 2];
struct WaveTimer {
  unsigned long long t0;
  __device__ WaveTimer() : t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~WaveTimer() {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const int wv = (int)blockIdx.x * kWavesPerBlock + (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && wv < kWaveTimeMax) {
      g_wave_time[2 * wv] = t0;
      g_wave_time[2 * wv + 1] = t1;
      g_wave_hw[2 * wv] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
      g_wave_hw[2 * wv + 1] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    }
  }
};
#endif

template <class Env, int NA, bool TRAJ, bool NOISE, bool JIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((NA > kNaRuntime || (JIT && NA > 3)) ? 2 : 4))) k_ctl_dynamic(KArgs A) {
#if MTGP_AB_WAVETIME
  WaveTimer wave_timer;
#endif
  constexpr int NV = Env::NV;
  // NA <= 3: the state size; NA = kNaRuntime / kNaWide: state_size 4 .. 8 / 9 .. 16 at run time
  // (interpreter only: the data vector has up to kDWide / kDWide2 slots, beyond the JIT's
  // register-data ABI)
  constexpr int DM = dyn_data_slots(NA);
  __shared__ float lds[kWavesPerBlock][(DM + kSMax) * kWave];
  const int na = NA <= 3 ? NA : uni(A.m.state_size);
  Lane Ln;
  if (!lane_setup(A, Ln)) return;
  if (JIT) asm volatile("s_icache_inv");  // the JIT code was written by an earlier kernel
  if constexpr (JIT && NA <= 3) {
    if (__builtin_expect(Ln.jok && A.chain_merge, 1)) {  // usable put-chain code: the JIT-only loop
      if (A.m.solver == MTGP_SOLVER_EULER) ctl_dynamic_jit<Env, NA, TRAJ, NOISE, 1>(A, Ln);
      else ctl_dynamic_jit<Env, NA, TRAJ, NOISE, 4>(A, Ln);
      return;
    }
  }
  const int r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* dcol = &lds[Ln.wave][Ln.lane];
  float* st = &lds[Ln.wave][DM * kWave + Ln.lane];
  // NA > 3 with JIT (round 6): LDS-data code reads the interpreter's own data columns, so the
  // data vector stays in LDS (no register copy)
  constexpr bool LJ = JIT && NA > 3;
  DataVec<JIT && !LJ> D(dcol, st);

  const int S = A.m.n_save;
  ObsNoise<NV> nzc;
  float nzv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) nzv[i] = 0.0f;
  if (NOISE) nzc = obs_noise_setup<NV>(A.m, A.ro, rr);
  const int uslot = NV + na;
  Env env;
  env.load(A.ro, rr, A.m.n_targets);
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;  // element offset of this (individual, rollout) in a save row
#pragma unroll
  for (int t = 0; t < DM - NV - 2; ++t)
    if (t < A.m.n_targets && uslot + 1 + t < DM) D.put(uslot + 1 + t, A.ro.targets[rr * A.m.n_targets + t]);

  float x[NV], a[NA], kx[NV], ka[NA], fx0[NV], fa0[NA], ax[NV], aa[NA];
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = A.ro.x0[rr * NV + i];
#pragma unroll
  for (int j = 0; j < NA; ++j) a[j] = ka[j] = aa[j] = fa0[j] = 0.0f;
#pragma unroll
  for (int i = 0; i < NV; ++i) kx[i] = ax[i] = fx0[i] = 0.0f;

  typename Env::Fit fit = Env::fit_init(active);
  bool dead = !active;  // the solve has ended (event): later save points are the +inf fill
  bool prev_ok;
  {
    float s0[NV + NA];
#pragma unroll
    for (int i = 0; i < NV; ++i) s0[i] = x[i];
#pragma unroll
    for (int j = 0; j < NA; ++j) s0[NV + j] = a[j];
    prev_ok = !Env::bad(s0, NV + NA);
  }
  // one save point: the state (xs, as) at ts[k] -> f_obs(key, (ts[k], xs)) (dyn.py:99), the
  // save-point readout on [y, a, 0, tar] (dyn.py:101), fitness, rows
  auto save_point = [&](int k, const float (&xs)[NV], const float (&as)[NA], bool fill) __attribute__((always_inline)) {
    float yo[NV];
    ctl_obs<Env, NOISE>(nzc, ldc(A.ro.ts, k), xs, yo);
#pragma unroll
    for (int i = 0; i < NV; ++i) D.put(i, yo[i]);
#pragma unroll
    for (int j = 0; j < NA; ++j)
      if (j < na) D.put(NV + j, as[j]);
    D.put(uslot, 0.0f);
    float sr[1];
    if constexpr (LJ) run_role_lds<1>(A, Ln, ng, A.m.prog_readout_save, dcol, st, sr);
    else run_role<JIT, 1>(A, Ln, ng, 2, A.m.prog_readout_save, D, sr);
    const float us = sr[0];
    if constexpr (Env::kMask) {
      if (active) env.fit_save(fit, k, S, A, PR, loff, fill, us, xs);
    } else if (!fill && !MTGP_AB_NOFIT) {
      env.fit_update(fit, k, S, A.ro.ts, us, xs);
    }
    if (TRAJ && active && !MTGP_AB_NOSTORE) {
      if (A.out.xs) {
#pragma unroll
        for (int i = 0; i < NV; ++i) store_row(A.out.xs, ((size_t)k * NV + i) * PR, loff, xs[i], PR);
      }
      if (A.out.ys) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < A.m.n_obs) store_row(A.out.ys, ((size_t)k * A.m.n_obs + i) * PR, loff, yo[i], PR);
      }
      if (A.out.us) store_row(A.out.us, (size_t)k * PR, loff, us, PR);
      if (A.out.acts) {
#pragma unroll
        for (int j = 0; j < NA; ++j)
          if (j < na) store_row(A.out.acts, ((size_t)k * na + j) * PR, loff, as[j], PR);
      }
    }
  };

  const bool euler = A.m.solver == MTGP_SOLVER_EULER;  // diffrax.Euler: one stage, y + f dt
  const int n_stages = euler ? 1 : 4;
  CsClock clk;
  clk.init(A);
  int k = 0;  // next save point
  while (clk.live()) {
    const float t = clk.t, dt = clk.dt();
    // (the stage input reads the b-weighted sum before f_{stage-1}'s term -- mtgp_rk4_in_acc, the
    // zero tableau entries -- which is then added: the same sums in the same order)
#pragma unroll 1
    for (int stage = 0; stage < n_stages; ++stage) {
      float xt[NV], at[NA], y[NV];
      stage_in_n<NV>(stage, x, kx, ax, dt, xt);
      stage_in_n<NA>(stage, a, ka, aa, dt, at);
      if (stage > 0) {
        stage_acc_n<NV>(stage - 1, ax, kx);
        stage_acc_n<NA>(stage - 1, aa, ka);
      }
#pragma unroll
      for (int j = 0; j < NA; ++j)
        if (j < na) D.put(NV + j, at[j]);
      float ur[1];
      if constexpr (LJ) run_role_lds<1>(A, Ln, ng, A.m.prog_readout, dcol, st, ur);
      else run_role<JIT, 1>(A, Ln, ng, 0, A.m.prog_readout, D, ur);
      const float u = ur[0];
      env.drift(xt, u, kx);
      // stages 1 and 2 share the time t + dt/2, hence the noise draw
      if (NOISE && stage != 2) obs_noise_vec<NV>(nzc, stage_time(stage, t, dt), nzv);
      ctl_obs_apply<Env>(xt, nzv, y);
#pragma unroll
      for (int i = 0; i < NV; ++i) D.put(i, y[i]);
      D.put(uslot, u);
      if constexpr (LJ) run_role_lds<NA>(A, Ln, ng, A.m.prog_state, dcol, st, ka, na);
      else run_role<JIT, NA>(A, Ln, ng, 1, A.m.prog_state, D, ka, A.chain_state != 0, -1, nullptr, na);
      if (stage == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) fx0[i] = kx[i];
#pragma unroll
        for (int j = 0; j < NA; ++j) fa0[j] = ka[j];
      }
    }
    stage_acc_n<NV>(n_stages - 1, ax, kx);
    stage_acc_n<NA>(n_stages - 1, aa, ka);
    float x1[NV], a1[NA];
#pragma unroll
    for (int i = 0; i < NV; ++i) x1[i] = euler ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
#pragma unroll
    for (int j = 0; j < NA; ++j) a1[j] = euler ? a[j] + fa0[j] * dt : mtgp_rk4_out(a[j], aa[j], dt);
    bool ev = false;
    if (!dead) {
      float sn[NV + NA];
#pragma unroll
      for (int i = 0; i < NV; ++i) sn[i] = x1[i];
#pragma unroll
      for (int j = 0; j < NA; ++j) sn[NV + j] = a1[j];
      const bool ok = !Env::bad(sn, NV + NA);  // (slots j >= na stay 0: ka / aa start at 0)
      ev = prev_ok && !ok;
      prev_ok = ok;
    }
    while (k < S && clk.saves(A.ro.ts, k)) {  // SaveAt(ts) through this step's dense output
      const float th = mtgp_cs_rescale(t, ldc(A.ro.ts, k), clk.tn);
      float xs[NV], as[NA];
      cs_dense<NV>(euler, dead, x, x1, fx0, kx, dt, th, xs);
      cs_dense<NA>(euler, dead, a, a1, fa0, ka, dt, th, as);
      save_point(k, xs, as, dead);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = x1[i];
#pragma unroll
      for (int j = 0; j < NA; ++j) a[j] = a1[j];
    }
    if (ev) {
      dead = true;
      if (k < S) Env::fit_kill(fit);  // save points of the +inf fill follow
    }
    clk.advance();
    if (!TRAJ && wave_all(fit.settled || dead)) break;
  }
  if (k < S) {  // unsaved points (max_steps, or every lane ended): +inf (throw=False)
    if (!fit.settled) Env::fit_kill(fit);
    if (TRAJ) {
      float xs[NV], as[NA];
#pragma unroll
      for (int i = 0; i < NV; ++i) xs[i] = kInf;
#pragma unroll
      for (int j = 0; j < NA; ++j) as[j] = kInf;
      for (; k < S; ++k) save_point(k, xs, as, true);
    }
  }
  finish_group(A, Ln, Env::fit_final(fit, S));
}

// The JIT-only stage loop of the static policy (as ctl_dynamic_jit: no interpreter code, RK4 stages
// unrolled; k_ctl_static's arithmetic operation for operation).
template <class Env, bool TRAJ, bool NOISE, int NST>
__device__ __forceinline__ void ctl_static_jit(const KArgs& A, const Lane& Ln) {
  constexpr int NV = Env::NV;
  const int r = Ln.r, rr = Ln.rr;
  const bool active = Ln.active;
  const int R = A.ro.R;
  const int S = A.m.n_save;
  const float* __restrict__ ts = A.ro.ts;
  uint32_t nzt = 0xffffffffu;  // bits of the time nzv was drawn at
  ObsNoise<NV> nzc;
  float nzv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) nzv[i] = 0.0f;
  if (NOISE) nzc = obs_noise_setup<NV>(A.m, A.ro, rr);
  Env env;
  env.load(A.ro, rr, A.m.n_targets);
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  float dv[kDMax];
#pragma unroll
  for (int k = 0; k < kDMax; ++k) dv[k] = 0.0f;
#pragma unroll
  for (int t = 0; t < kDMax - NV; ++t)
    if (t < A.m.n_targets) dv[NV + t] = A.ro.targets[rr * A.m.n_targets + t];
  const uint64_t u_policy = A.jit_base + (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_readout);

  float x[NV], kx[NV], fx0[NV], ax[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = A.ro.x0[rr * NV + i];
#pragma unroll
  for (int i = 0; i < NV; ++i) kx[i] = ax[i] = fx0[i] = 0.0f;
  typename Env::Fit fit = Env::fit_init(active);
  bool dead = !active;
  bool prev_ok = !Env::bad(x, NV);
  // one save point: ys = f_obs(key, (ts[k], xs)) (ff.py:96), us = policy([ys, tar]) (ff.py:97)
  auto save_point = [&](int k, const float (&xs)[NV], bool fill) __attribute__((always_inline)) {
    float yo[NV];
    if (NOISE) {
      const uint32_t tb = __float_as_uint(ldc(ts, k));
      if (tb != nzt) {
        obs_noise_vec<NV>(nzc, ldc(ts, k), nzv);
        nzt = tb;
      }
    }
    ctl_obs_apply<Env>(xs, nzv, yo);
#pragma unroll
    for (int i = 0; i < NV; ++i) dv[i] = yo[i];
    const float us = MTGP_AB_NOSAVECALL ? dv[0] : jit_call_nf(u_policy, dv);
    if (!fill) env.fit_update(fit, k, S, ts, us, xs);
    if (TRAJ && active) {
      if (A.out.xs) {
#pragma unroll
        for (int i = 0; i < NV; ++i) store_row(A.out.xs, ((size_t)k * NV + i) * PR, loff, xs[i], PR);
      }
      if (A.out.ys) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < A.m.n_obs) store_row(A.out.ys, ((size_t)k * A.m.n_obs + i) * PR, loff, yo[i], PR);
      }
      if (A.out.us) store_row(A.out.us, (size_t)k * PR, loff, us, PR);
    }
  };

  CsClock clk;
  clk.init(A);
  int k = 0;
  const bool fair_on = uni(A.fair) != 0;
  FairShare fair;
  if (fair_on) fair.init(A);
  while (clk.live()) {
    if (fair_on) fair.step(Ln.lane, (uint32_t)clk.steps);
    const float t = clk.t, dt = clk.dt();
    // (the stage input reads the b-weighted sum before f_{ST-1}'s term -- mtgp_rk4_in_acc, the zero
    // tableau entries -- which is then added: the same sums in the same order)
    auto stage = [&](auto st_c) {
      constexpr int ST = decltype(st_c)::value;
      float xt[NV], y[NV];
      rk_in<NV>(ST, x, kx, ax, dt, xt);
      if (NST == 4 && ST > 0) rk_acc<NV>(ST - 1, ax, kx);
      if (NOISE && ST != 2) {
        const float tc = ST == 0 ? t : mtgp_rk4_time(ST, t, dt);
        obs_noise_vec<NV>(nzc, tc, nzv);
        nzt = __float_as_uint(tc);
      }
      ctl_obs_apply<Env>(xt, nzv, y);
#pragma unroll
      for (int i = 0; i < NV; ++i) dv[i] = y[i];
      const float u = jit_call_nf(u_policy, dv);  // ff.py:106-107
      env.drift(xt, u, kx);
      if (ST == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) fx0[i] = kx[i];
      }
    };
    stage(std::integral_constant<int, 0>{});
    if constexpr (NST == 4) {
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      rk_acc<NV>(3, ax, kx);
    }
    float x1[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) x1[i] = NST == 1 ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
    bool ev = false;
    if (!dead) {
      const bool ok = !Env::bad(x1, NV);
      ev = prev_ok && !ok;
      prev_ok = ok;
    }
    while (k < S && clk.saves(ts, k)) {
      float xs[NV];
      if (MTGP_AB_NOHERMITE) {
#pragma unroll
        for (int i = 0; i < NV; ++i) xs[i] = x1[i];
      } else {
        const float th = mtgp_cs_rescale(t, ldc(ts, k), clk.tn);
        cs_dense<NV>(NST == 1, dead, x, x1, fx0, kx, dt, th, xs);
      }
      save_point(k, xs, dead);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = x1[i];
    }
    if (ev) {
      dead = true;
      if (k < S) Env::fit_kill(fit);
    }
    clk.advance();
    if (!TRAJ && wave_all(fit.settled || dead)) break;
  }
  if (k < S) {
    if (!fit.settled) Env::fit_kill(fit);
    if (TRAJ) {
      float xs[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) xs[i] = kInf;
      for (; k < S; ++k) save_point(k, xs, true);
    }
  }
  finish_group(A, Ln, Env::fit_final(fit, S));
}

// --------------------------------------------------------------------------------------
// Static policy (feedforward_evaluate.py:64-110) on environment Env.  Data slots:
// y 0..NV-1 | targets.
template <class Env, bool TRAJ, bool NOISE, bool JIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_ctl_static(KArgs A) {
  constexpr int NV = Env::NV;
  __shared__ float lds[kWavesPerBlock][kLdsWaveWords];
  Lane Ln;
  if (!lane_setup(A, Ln)) return;
  if (JIT) asm volatile("s_icache_inv");  // the JIT code was written by an earlier kernel
  if constexpr (JIT && !Env::kMask) {
    if (__builtin_expect(Ln.jok, 1)) {  // usable code: the JIT-only loop
      if (A.m.solver == MTGP_SOLVER_EULER) ctl_static_jit<Env, TRAJ, NOISE, 1>(A, Ln);
      else ctl_static_jit<Env, TRAJ, NOISE, 4>(A, Ln);
      return;
    }
  }
  const int r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* dcol = &lds[Ln.wave][Ln.lane];
  float* st = &lds[Ln.wave][kDMax * kWave + Ln.lane];
  DataVec<JIT> D(dcol, st);
  const int S = A.m.n_save;
  ObsNoise<NV> nzc;
  float nzv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) nzv[i] = 0.0f;
  if (NOISE) nzc = obs_noise_setup<NV>(A.m, A.ro, rr);
  Env env;
  env.load(A.ro, rr, A.m.n_targets);
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
#pragma unroll
  for (int t = 0; t < kDMax - NV; ++t)
    if (t < A.m.n_targets) D.put(NV + t, A.ro.targets[rr * A.m.n_targets + t]);

  float x[NV], kx[NV], fx0[NV], ax[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = A.ro.x0[rr * NV + i];
#pragma unroll
  for (int i = 0; i < NV; ++i) kx[i] = ax[i] = fx0[i] = 0.0f;
  typename Env::Fit fit = Env::fit_init(active);
  bool dead = !active;
  bool prev_ok = !Env::bad(x, NV);
  // one save point: ys = f_obs(key, (ts[k], xs)) (ff.py:96), us = policy([ys, tar]) (ff.py:97)
  auto save_point = [&](int k, const float (&xs)[NV], bool fill) __attribute__((always_inline)) {
    float yo[NV];
    ctl_obs<Env, NOISE>(nzc, ldc(A.ro.ts, k), xs, yo);
#pragma unroll
    for (int i = 0; i < NV; ++i) D.put(i, yo[i]);
    float ur[1];
    run_role<JIT, 1>(A, Ln, ng, 0, A.m.prog_readout, D, ur);
    const float us = ur[0];
    if constexpr (Env::kMask) {
      if (active) env.fit_save(fit, k, S, A, PR, loff, fill, us, xs);
    } else if (!fill) {
      env.fit_update(fit, k, S, A.ro.ts, us, xs);
    }
    if (TRAJ && active) {
      if (A.out.xs) {
#pragma unroll
        for (int i = 0; i < NV; ++i) store_row(A.out.xs, ((size_t)k * NV + i) * PR, loff, xs[i], PR);
      }
      if (A.out.ys) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < A.m.n_obs) store_row(A.out.ys, ((size_t)k * A.m.n_obs + i) * PR, loff, yo[i], PR);
      }
      if (A.out.us) store_row(A.out.us, (size_t)k * PR, loff, us, PR);
    }
  };

  const bool euler = A.m.solver == MTGP_SOLVER_EULER;  // diffrax.Euler: one stage, y + f dt
  const int n_stages = euler ? 1 : 4;
  CsClock clk;
  clk.init(A);
  int k = 0;
  while (clk.live()) {
    const float t = clk.t, dt = clk.dt();
    // (the stage input reads the b-weighted sum before f_{stage-1}'s term -- mtgp_rk4_in_acc, the
    // zero tableau entries -- which is then added: the same sums in the same order)
#pragma unroll 1
    for (int stage = 0; stage < n_stages; ++stage) {
      float xt[NV], y[NV];
      stage_in_n<NV>(stage, x, kx, ax, dt, xt);
      if (stage > 0) stage_acc_n<NV>(stage - 1, ax, kx);
      // stages 1 and 2 share the time t + dt/2, hence the noise draw
      if (NOISE && stage != 2) obs_noise_vec<NV>(nzc, stage_time(stage, t, dt), nzv);
      ctl_obs_apply<Env>(xt, nzv, y);
#pragma unroll
      for (int i = 0; i < NV; ++i) D.put(i, y[i]);
      float ur[1];
      run_role<JIT, 1>(A, Ln, ng, 0, A.m.prog_readout, D, ur);  // ff.py:106-107
      env.drift(xt, ur[0], kx);
      if (stage == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) fx0[i] = kx[i];
      }
    }
    stage_acc_n<NV>(n_stages - 1, ax, kx);
    float x1[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) x1[i] = euler ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
    bool ev = false;
    if (!dead) {
      const bool ok = !Env::bad(x1, NV);
      ev = prev_ok && !ok;
      prev_ok = ok;
    }
    while (k < S && clk.saves(A.ro.ts, k)) {
      const float th = mtgp_cs_rescale(t, ldc(A.ro.ts, k), clk.tn);
      float xs[NV];
      cs_dense<NV>(euler, dead, x, x1, fx0, kx, dt, th, xs);
      save_point(k, xs, dead);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = x1[i];
    }
    if (ev) {
      dead = true;
      if (k < S) Env::fit_kill(fit);
    }
    clk.advance();
    if (!TRAJ && wave_all(fit.settled || dead)) break;
  }
  if (k < S) {
    if (!fit.settled) Env::fit_kill(fit);
    if (TRAJ) {
      float xs[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) xs[i] = kInf;
      for (; k < S; ++k) save_point(k, xs, true);
    }
  }
  finish_group(A, Ln, Env::fit_final(fit, S));
}

// Dormand-Prince stage inputs (include/mtgp_dopri5.h): sum_{j<s} a_sj f_j, the fma chain of
// mtgp_dp_term in ascending j with zero entries skipped, the tableau as compile-time constants.
// The stage loops stay rolled (one copy of the RHS and its program call sites); one wave-uniform
// switch on s selects the specialisation, and the stage derivative is filed into f[s] the same
// way.  (Reading a_sj from a table by the dynamic s and filing f[s] with selects cost ~150 VALU
// per stage: two thirds of a lone tail wave's arithmetic outside the RHS.)
template <int S, int N>
__device__ __forceinline__ void dp_stage_sum_s(const float (&f)[7][N], float (&acc)[N]) {
  constexpr float a[7][6] = MTGP_DP_TABLE_A;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < S; ++j) v = mtgp_dp_term(v, a[S][j], f[j][i], j == 0);
    acc[i] = v;
  }
}
template <int N>
__device__ __forceinline__ void dp_stage_sum(int s, const float (&f)[7][N], float (&acc)[N]) {
  switch (s) {
    case 1: dp_stage_sum_s<1, N>(f, acc); break;
    case 2: dp_stage_sum_s<2, N>(f, acc); break;
    case 3: dp_stage_sum_s<3, N>(f, acc); break;
    case 4: dp_stage_sum_s<4, N>(f, acc); break;
    case 5: dp_stage_sum_s<5, N>(f, acc); break;
    default: dp_stage_sum_s<6, N>(f, acc); break;
  }
}
template <int S, int N>
__device__ __forceinline__ void dp_file_s(float (&f)[7][N], const float (&k)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) f[S][i] = k[i];
}
template <int N>
__device__ __forceinline__ void dp_file(int s, float (&f)[7][N], const float (&k)[N]) {
  switch (s) {
    case 1: dp_file_s<1, N>(f, k); break;
    case 2: dp_file_s<2, N>(f, k); break;
    case 3: dp_file_s<3, N>(f, k); break;
    case 4: dp_file_s<4, N>(f, k); break;
    case 5: dp_file_s<5, N>(f, k); break;
    default: dp_file_s<6, N>(f, k); break;
  }
}

// the controller coefficients of model m (mtgp.h ABI v15; pid_custom == 0: diffrax's defaults)
__device__ __forceinline__ MtgpDpPid dp_pid(const MtgpModel& m) {
  if (!m.pid_custom) return MtgpDpPid MTGP_DP_PID_DEFAULT;
  return MtgpDpPid{m.pid_c1, m.pid_c2, m.pid_c3, m.pid_safety, m.pid_factormin, m.pid_factormax};
}

// --------------------------------------------------------------------------------------
// Control evaluators with adaptive Dopri5 + PIDController (the notebooks' solver,
// DynamicPolicy.ipynb:105, StaticPolicy.ipynb:102; spec include/mtgp_dopri5.h).  NA > 0: the
// dynamic evaluator (state [x, a], the RHS of dyn.py:107-118); NA == 0: the static policy
// (ff.py:104-110).  Per-lane t / step / controller state; every wave-uniform program call (the
// six FSAL stages, then one call per round of pending save points, then the +inf fill) runs for
// all lanes, and only the lanes concerned commit.  Save points: dense output of [x, a] at ts[k],
// then f_obs(ts[k], x) and the save-time readout / policy (dyn.py:99-101, ff.py:96-97).
// A lane's Dopri5 solve between the two launches (KArgs.dp_state, word-major): t, t_next, the
// controller history, flags, save index, attempts, y and the FSAL derivative f0, the fitness
// accumulator -- everything the attempt loop carries, so launch 2 continues bit for bit.
constexpr int kDpStateWords = MTGP_DP_STATE_WORDS;
template <int ND, class Fit>
struct DpParked {
  float* base;
  uint32_t stride, gl;
  static constexpr int kFitWords = (int)((sizeof(Fit) + 3) / 4);
  static_assert(7 + 2 * ND + kFitWords <= kDpStateWords - 1, "Dopri5 parked state too large");
  // the last word of lane 0's column: the wave's remaining-work estimate (launch 2's order)
  static constexpr int kEstWord = kDpStateWords - 1;
  __device__ __forceinline__ float& w(int i) const { return base[(size_t)i * stride + gl]; }
  __device__ __forceinline__ void save(float t, float tn, const MtgpDpCtl& c, bool ok, bool live, int k, int steps,
                                       const float (&y)[ND], const float (&f0)[ND], const Fit& fit) const {
    w(0) = t;
    w(1) = tn;
    w(2) = c.prev;
    w(3) = c.prev2;
    w(4) = __int_as_float((c.at_dtmin != 0) | (ok ? 2 : 0) | (live ? 4 : 0));
    w(5) = __int_as_float(k);
    w(6) = __int_as_float(steps);
#pragma unroll
    for (int i = 0; i < ND; ++i) { w(7 + i) = y[i]; w(7 + ND + i) = f0[i]; }
    uint32_t fw[kFitWords];
    __builtin_memcpy(fw, &fit, sizeof(Fit));
#pragma unroll
    for (int i = 0; i < kFitWords; ++i) w(7 + 2 * ND + i) = __uint_as_float(fw[i]);
  }
  __device__ __forceinline__ void load(float& t, float& tn, MtgpDpCtl& c, bool& ok, bool& live, int& k, int& steps,
                                       float (&y)[ND], float (&f0)[ND], Fit& fit) const {
    t = w(0);
    tn = w(1);
    c.prev = w(2);
    c.prev2 = w(3);
    const int fl = __float_as_int(w(4));
    c.at_dtmin = fl & 1;
    ok = (fl & 2) != 0;
    live = (fl & 4) != 0;
    k = __float_as_int(w(5));
    steps = __float_as_int(w(6));
#pragma unroll
    for (int i = 0; i < ND; ++i) { y[i] = w(7 + i); f0[i] = w(7 + ND + i); }
    uint32_t fw[kFitWords];
#pragma unroll
    for (int i = 0; i < kFitWords; ++i) fw[i] = __float_as_uint(w(7 + 2 * ND + i));
    __builtin_memcpy(&fit, fw, sizeof(Fit));
  }
};

// MTGP_DP_WAVES (mtgp_ab.h, 2): register budget of the Dopri5 control kernels (A/B: 2 beats 4, C3 23 vs 28 ms)
template <class Env, int NA, bool TRAJ, bool NOISE, bool JIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MTGP_DP_WAVES))) k_ctl_dopri5(KArgs A) {
  constexpr int NV = Env::NV;
  constexpr bool DYN = NA > 0;
  constexpr int NAX = DYN ? NA : 1;
  constexpr int ND = NV + NA;  // integrated state (NA > 3: the upper bound of a runtime state size)
  // NA > 3 (round 6): state_size 4 .. NA at run time, interpreter only, one launch (no parking);
  // the components past NV + na stay 0 and are left out of the error norm, the rows and the data
  constexpr bool RT = NA > 3;
  constexpr int DM = DYN ? dyn_data_slots(NA) : kDMax;
  const int na = RT ? uni(A.m.state_size) : NA;
  const int nd = NV + na;
  __shared__ float lds[kWavesPerBlock][(DM + kSMax) * kWave];
  Lane Ln;
  int wv = (int)blockIdx.x * kWavesPerBlock + (int)(threadIdx.x >> 6);
  if (A.dp_pass == 2) {  // resume a parked wave of launch 1
    if (wv >= A.dp_pending[0]) return;
    wv = uni(A.dp_pending[1 + wv]);
  }
  if (!lane_setup(A, Ln, wv)) return;
  const int r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* dcol = &lds[Ln.wave][Ln.lane];
  float* st = &lds[Ln.wave][DM * kWave + Ln.lane];
  DataVec<JIT> D(dcol, st);
  if (JIT) asm volatile("s_icache_inv");
  const int S = A.m.n_save, max_steps = A.m.max_steps;
  const float rtol = A.m.rtol, atol = A.m.atol, dtmin = A.m.dtmin, dtmax = A.m.dtmax;
  const float* __restrict__ ts = A.ro.ts;
  const float t_end = ts[S - 1];
  ObsNoise<NV> nzc;
  if (NOISE) nzc = obs_noise_setup<NV>(A.m, A.ro, rr);
  const int uslot = DYN ? NV + na : NV;  // static: targets follow y directly
  Env env;
  env.load(A.ro, rr, A.m.n_targets);
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  const int tslot = DYN ? uslot + 1 : NV;
#pragma unroll
  for (int t = 0; t < DM; ++t)
    if (t >= tslot && t - tslot < A.m.n_targets) D.put(t, A.ro.targets[rr * A.m.n_targets + (t - tslot)]);
  constexpr float E[7] = MTGP_DP_TABLE_E;
  constexpr float CM[7] = MTGP_DP_TABLE_CMID;

  // RHS at time tc of state s -> ds (dyn.py:107-118 / ff.py:104-110)
  auto rhs = [&](float tc, const float* s, float* ds) __attribute__((always_inline)) {
    float y[NV], nzv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) nzv[i] = 0.0f;
    if (NOISE) obs_noise_vec<NV>(nzc, tc, nzv);
    ctl_obs_apply<Env>(s, nzv, y);
    float ur[1];
    if (DYN) {
#pragma unroll
      for (int j = 0; j < NA; ++j)
        if (!RT || j < na) D.put(NV + j, s[NV + j]);
      run_role<JIT, 1, MTGP_DP_COLD != 0>(A, Ln, ng, 0, A.m.prog_readout, D, ur);  // reads [0, a, 0, tar]
      env.drift(s, ur[0], ds);
#pragma unroll
      for (int i = 0; i < NV; ++i) D.put(i, y[i]);
      D.put(uslot, ur[0]);
      float ka[NAX];
#pragma unroll
      for (int j = 0; j < NAX; ++j) ka[j] = 0.0f;  // (RT: the slots j >= na stay 0)
      run_role<JIT, NAX, MTGP_DP_COLD != 0>(A, Ln, ng, 1, A.m.prog_state, D, ka, DYN && !RT && A.chain_state != 0, -1,
                                            nullptr, na);
#pragma unroll
      for (int j = 0; j < NA; ++j) ds[NV + j] = ka[j];
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) D.put(i, y[i]);
      run_role<JIT, 1, MTGP_DP_COLD != 0>(A, Ln, ng, 0, A.m.prog_readout, D, ur);
      env.drift(s, ur[0], ds);
    }
  };
  // one save point of lanes with `on` (wave-uniform call): observation at ts[k], readout, fitness, rows
  typename Env::Fit fit = Env::fit_init(active);
  auto save_round = [&](bool on, int k, const float* sk, bool fill) __attribute__((always_inline)) {
    float y[NV];
    ctl_obs<Env, NOISE>(nzc, on ? ts[k] : 0.0f, sk, y);
#pragma unroll
    for (int i = 0; i < NV; ++i) D.put(i, y[i]);
    float ur[1];
    if (DYN) {
#pragma unroll
      for (int j = 0; j < NA; ++j)
        if (!RT || j < na) D.put(NV + j, sk[NV + j]);
      D.put(uslot, 0.0f);
      run_role<JIT, 1, MTGP_DP_COLD != 0>(A, Ln, ng, 2, A.m.prog_readout_save, D, ur);  // readout([y, a, 0, tar]) dyn.py:101
    } else {
      run_role<JIT, 1, MTGP_DP_COLD != 0>(A, Ln, ng, 0, A.m.prog_readout, D, ur);  // policy([y, tar]) ff.py:97
    }
    if (!on) return;
    if constexpr (Env::kMask) env.fit_save(fit, k, S, A, PR, loff, fill, ur[0], sk);
    else if (!fill) env.fit_update(fit, k, S, ts, ur[0], sk);
    if (TRAJ && active) {
      const bool lm = A.out.traj_layout == MTGP_TRAJ_LANE_MAJOR;
      if (A.out.xs) {
#pragma unroll
        for (int i = 0; i < NV; ++i) traj_put_dp(A.out.xs, lm, k, i, NV, loff, PR, S, sk[i]);
      }
      if (A.out.ys) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < A.m.n_obs) traj_put_dp(A.out.ys, lm, k, i, A.m.n_obs, loff, PR, S, y[i]);
      }
      if (A.out.us) traj_put_dp(A.out.us, lm, k, 0, 1, loff, PR, S, ur[0]);
      if (DYN && A.out.acts) {
#pragma unroll
        for (int j = 0; j < NA; ++j)
          if (!RT || j < na) traj_put_dp(A.out.acts, lm, k, j, RT ? na : NAX, loff, PR, S, sk[NV + j]);
      }
    }
  };

  float y[ND], y1[ND], f[7][ND];
  int k = 1, steps = 0;
  bool prev_ok;
  MtgpDpCtl ctl{1.0f, 1.0f, 0};
  const MtgpDpPid pid = dp_pid(A.m);
  const int force_dtmin = !A.m.no_force_dtmin;
  float t, tnext;
  bool live;
  // (RT: one launch only, the entry point rejects dp_budget; the parked state would not fit)
  DpParked<RT ? 1 : ND, typename Env::Fit> park{A.dp_state, A.dp_lanes, (uint32_t)wv * kWave + (uint32_t)Ln.lane};
  if (!RT && A.dp_pass == 2) {
    if constexpr (!RT) park.load(t, tnext, ctl, prev_ok, live, k, steps, y, f[0], fit);
  } else {
#pragma unroll
    for (int i = 0; i < NV; ++i) y[i] = A.ro.x0[rr * NV + i];
#pragma unroll
    for (int j = NV; j < ND; ++j) y[j] = 0.0f;
    save_round(active, 0, y, false);
    prev_ok = !Env::bad(y, ND);
    t = ts[0];
    tnext = t + A.m.h;
    tnext = tnext > t_end ? t_end : tnext;
    rhs(t, y, f[0]);
    live = active && t < t_end && steps < max_steps;
  }
  const int budget = A.dp_pass == 1 ? A.dp_budget : 0x7fffffff;
  const bool fair_on = uni(A.fair_dp) != 0;  // fair share of the SIMDs by attempt count (FairShare)
  FairShare fair;
  if (fair_on) fair.init(A, A.fair_dp);
  for (int iter = 0; wave_any(live); ++iter) {
    if (fair_on) fair.step(Ln.lane, (uint32_t)iter);
    if (!RT && iter == budget) {  // launch 1 of 2: park this wave (every lane), launch 2 resumes it
      if constexpr (!RT) {
        park.save(t, tnext, ctl, prev_ok, live, k, steps, y, f[0], fit);
        // the wave's remaining work, for launch 2's longest-first order (k_dp_order): its slowest
        // lane's attempts so far scaled by the time still to cover over the time covered
        const float done = t - ts[0];
        float est = !live ? 0.0f : (done > 0.0f ? (float)steps * ((t_end - t) / done) : (float)max_steps);
        est = est < (float)max_steps ? est : (float)max_steps;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) est = fmaxf(est, __shfl_xor(est, o, kWave));
        if (Ln.lane == 0) park.w(park.kEstWord) = est;
      }
      if (Ln.lane == 0) A.dp_pending[1 + atomicAdd(A.dp_pending, 1)] = wv;
      return;
    }
    const float h = tnext - t;
#pragma unroll 1
    for (int s = 1; s <= 6; ++s) {
      float yi[ND], fs[ND], acc[ND];
      dp_stage_sum<ND>(s, f, acc);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        yi[i] = MTGP_FMAF(h, acc[i], y[i]);
        y1[i] = yi[i];
      }
      rhs(t + mtgp_dp_c(s) * h, yi, fs);
      dp_file<ND>(s, f, fs);
    }
    bool keep = false, stop = false, fail = false;
    float dt = 0.0f;
    if (live) {
      float msum = 0.0f;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        if (RT && i >= nd) continue;  // (components past the runtime state size: not in the norm)
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], f[j][i], j == 0);
        const float sc = mtgp_dp_scaled(h * acc, y[i], y1[i], rtol, atol);
        msum = (i == 0) ? sc * sc : msum + sc * sc;
      }
      const float ms = msum / (float)(RT ? nd : ND);
      int kp, fl;
      dt = mtgp_dp_control(ms, h, dtmin, dtmax, force_dtmin, &pid, &ctl, &kp, &fl);
      keep = kp != 0;
      fail = fl != 0;
      ++steps;
    }
    // SaveAt(ts) through the dense output of the accepted steps, one save point per round
    bool sv = live && keep && k < S && ts[k] <= tnext;
    while (wave_any(sv)) {
      float sk[ND];
      const float th = sv ? (ts[k] - t) / h : 0.0f;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, CM[j], f[j][i], j == 0);
        const float ymid = MTGP_FMAF(h, acc, y[i]);
        sk[i] = mtgp_dp_interp(y[i], y1[i], ymid, h * f[0][i], h * f[6][i], th);
      }
      save_round(sv, k, sk, false);
      if (sv) {
        ++k;
        sv = k < S && ts[k] <= tnext;
      }
    }
    if (live) {
      if (keep) {
        t = tnext;
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          y[i] = y1[i];
          f[0][i] = f[6][i];  // FSAL
        }
        const bool ok = !Env::bad(y, ND);
        stop = prev_ok && !ok;  // Event(cond_fn_nan), dyn.py:94
        prev_ok = ok;
      }
      if (stop || fail || !(t < t_end) || steps >= max_steps || (!TRAJ && fit.settled)) live = false;
      else tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
  }
  if (active && A.out.steps) A.out.steps[loff] = steps;
  // unsaved points are +inf (throw=False); their fitness terms follow Env::fit_kill
  bool fl = active && k < S;
  if (fl && !fit.settled) Env::fit_kill(fit);  // (settled: the fitness is already final)
  if (TRAJ) {  // (EnvAcrobotMask: trajectory variants only -- the general mask counts the fill's costs)
    float sk[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) sk[i] = kInf;
    while (wave_any(fl)) {
      save_round(fl, k, sk, true);
      if (fl) fl = ++k < S;
    }
  }
  finish_group(A, Ln, Env::fit_final(fit, S));
}

// --------------------------------------------------------------------------------------
// Symbolic regression of an ODE (SR_evaluator.py:57-94): dx_i = tree_i(x); MSE vs ys_true.
template <int NV, bool TRAJ, bool JIT>
__global__ void __launch_bounds__(256) k_sr(KArgs A) {
  __shared__ float lds[kWavesPerBlock][kLdsWaveWords];
  Lane Ln;
  if (!lane_setup(A, Ln)) return;
  const int r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* dcol = &lds[Ln.wave][Ln.lane];
  float* st = &lds[Ln.wave][kDMax * kWave + Ln.lane];
  DataVec<JIT> D(dcol, st);
  if (JIT) asm volatile("s_icache_inv");  // the JIT code was written by an earlier kernel
  const int S = A.m.n_save;
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  float x[NV], kx[NV], fx0[NV], ax[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    x[i] = A.ro.x0[rr * NV + i];
    kx[i] = fx0[i] = ax[i] = 0.0f;
  }
  auto bad = [&](const float* s) {
    bool b = false;
#pragma unroll
    for (int i = 0; i < NV; ++i) b = b || !mtgp_isfinite(s[i]);
    return b;
  };
  bool dead = !active, prev_ok = !bad(x);
  float tot = 0.0f;
  // one save point: the MSE term sum_d (pred - true)^2 (sr.py:24); a point of the +inf fill makes
  // the sum +inf (NaN stays NaN), as the oracle's MSE of the saved arrays
  auto save_point = [&](int k, const float (&xs)[NV], bool fill) __attribute__((always_inline)) {
    if (fill) {
      if (mtgp_isfinite(tot)) tot = kInf;
    } else {
      float sq = 0.0f;
#pragma unroll
      for (int d = 0; d < NV; ++d) {
        const float e = xs[d] - A.ro.ys_true[((size_t)k * NV + d) * R + rr];
        sq = (d == 0) ? e * e : sq + e * e;
      }
      tot = tot + sq;
    }
    if (TRAJ && active && A.out.xs) {
#pragma unroll
      for (int d = 0; d < NV; ++d) store_row(A.out.xs, ((size_t)k * NV + d) * PR, loff, xs[d], PR);
    }
  };
  const bool euler = A.m.solver == MTGP_SOLVER_EULER;  // diffrax.Euler: one stage, y + f dt
  const int n_stages = euler ? 1 : 4;
  CsClock clk;
  clk.init(A);
  int k = 0;
  const bool fair_on = uni(A.fair) != 0;
  FairShare fair;
  if (fair_on) fair.init(A);
  while (clk.live()) {
    if (fair_on) fair.step(Ln.lane, (uint32_t)clk.steps);
    const float dt = clk.dt();
    // (the stage input reads the b-weighted sum before f_{stage-1}'s term -- mtgp_rk4_in_acc, the
    // zero tableau entries -- which is then added: the same sums in the same order)
#pragma unroll 1
    for (int stage = 0; stage < n_stages; ++stage) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        D.put(i, stage_in(stage, x[i], kx[i], ax[i], dt));
        if (stage > 0) ax[i] = stage_acc(stage - 1, ax[i], kx[i]);
      }
      run_role<JIT, NV>(A, Ln, ng, 0, A.m.prog_state, D, kx, A.chain_state != 0);
      if (stage == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) fx0[i] = kx[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) ax[i] = stage_acc(n_stages - 1, ax[i], kx[i]);
    float x1[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) x1[i] = euler ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
    bool ev = false;
    if (!dead) {
      const bool ok = !bad(x1);
      ev = prev_ok && !ok;  // the NaN event (sr.py:93-94)
      prev_ok = ok;
    }
    while (k < S && clk.saves(A.ro.ts, k)) {  // SaveAt(ts) through this step's dense output
      const float th = mtgp_cs_rescale(clk.t, ldc(A.ro.ts, k), clk.tn);
      float xs[NV];
      cs_dense<NV>(euler, dead, x, x1, fx0, kx, dt, th, xs);
      save_point(k, xs, dead);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int i = 0; i < NV; ++i) x[i] = x1[i];
    }
    if (ev) dead = true;
    clk.advance();
    if (!TRAJ && wave_all(dead)) break;  // every remaining save point adds (inf - y)^2
  }
  if (k < S) {  // unsaved points (event / max_steps): +inf
    float xs[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) xs[i] = kInf;
    if (TRAJ) {
      for (; k < S; ++k) save_point(k, xs, true);
    } else {
      save_point(k, xs, true);
    }
  }
  const float F = tot / (float)S;
  finish_group(A, Ln, F);
}

// --------------------------------------------------------------------------------------
// Symbolic regression with adaptive Dopri5 + PIDController, SaveAt(ts) by dense output and the
// NaN event (SR_evaluator.py:57-94 with the notebook's solver, SymbolicRegression.ipynb:136):
// every rule is the fp32 spec of include/mtgp_dopri5.h.  Each lane (individual, rollout) has its
// own t, step and accept/reject history; the wave iterates while any lane is still integrating
// and runs the six new stage RHS evaluations (Dopri5 is FSAL) for all lanes together, since the
// programs are shared per group.  Lanes that are done keep computing but never commit.
template <int NV, bool TRAJ, bool JIT>
__global__ void __launch_bounds__(256) k_sr_dopri5(KArgs A) {
  __shared__ float lds[kWavesPerBlock][kLdsWaveWords];
  Lane Ln;
  if (!lane_setup(A, Ln)) return;
  const int r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* dcol = &lds[Ln.wave][Ln.lane];
  float* st = &lds[Ln.wave][kDMax * kWave + Ln.lane];
  DataVec<JIT> D(dcol, st);
  if (JIT) asm volatile("s_icache_inv");
  const int S = A.m.n_save, max_steps = A.m.max_steps;
  const float rtol = A.m.rtol, atol = A.m.atol, dtmin = A.m.dtmin, dtmax = A.m.dtmax;
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  const float* __restrict__ ts = A.ro.ts;
  const float t_end = ts[S - 1];
  constexpr float E[7] = MTGP_DP_TABLE_E;
  constexpr float CM[7] = MTGP_DP_TABLE_CMID;
  float tot = 0.0f;
  // one save point: MSE term (components in index order, sr.py:24) and the trajectory row
  auto save = [&](int k, const float* v) __attribute__((always_inline)) {
    float sq = 0.0f;
#pragma unroll
    for (int d = 0; d < NV; ++d) {
      const float e = v[d] - A.ro.ys_true[((size_t)k * NV + d) * R + rr];
      sq = (d == 0) ? e * e : sq + e * e;
    }
    tot = tot + sq;
    if (TRAJ && active && A.out.xs) {
      const bool lm = A.out.traj_layout == MTGP_TRAJ_LANE_MAJOR;
#pragma unroll
      for (int d = 0; d < NV; ++d) traj_put_dp(A.out.xs, lm, k, d, NV, loff, PR, S, v[d]);
    }
  };
  auto bad = [&](const float* v) __attribute__((always_inline)) {
    bool b = false;
#pragma unroll
    for (int i = 0; i < NV; ++i) b = b || !mtgp_isfinite(v[i]);
    return b;
  };
  float y[NV], y1[NV], kx[NV], f[7][NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) y[i] = A.ro.x0[rr * NV + i];
  save(0, y);
  int k = 1, steps = 0;
  bool prev_ok = !bad(y);
  MtgpDpCtl ctl{1.0f, 1.0f, 0};
  const MtgpDpPid pid = dp_pid(A.m);
  const int force_dtmin = !A.m.no_force_dtmin;
  float t = ts[0];
  float tnext = t + A.m.h;
  tnext = tnext > t_end ? t_end : tnext;
  // FSAL seed f0 = f(t0, y0)
#pragma unroll
  for (int i = 0; i < NV; ++i) D.put(i, y[i]);
  run_role<JIT, NV, MTGP_DP_COLD != 0>(A, Ln, ng, 0, A.m.prog_state, D, kx, A.chain_state != 0);
#pragma unroll
  for (int i = 0; i < NV; ++i) f[0][i] = kx[i];
  bool live = active && t < t_end && steps < max_steps;
  while (wave_any(live)) {
    const float h = tnext - t;
#pragma unroll 1
    for (int s = 1; s <= 6; ++s) {  // stage s input y + h sum_{j<s} a_sj f_j (wave-uniform s)
      float acc[NV];
      dp_stage_sum<NV>(s, f, acc);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const float yi = MTGP_FMAF(h, acc[i], y[i]);
        y1[i] = yi;  // the stage-6 input is the step's solution
        D.put(i, yi);
      }
      run_role<JIT, NV, MTGP_DP_COLD != 0>(A, Ln, ng, 0, A.m.prog_state, D, kx, A.chain_state != 0);
      dp_file<NV>(s, f, kx);
    }
    if (live) {
      float msum = 0.0f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], f[j][i], j == 0);
        const float sc = mtgp_dp_scaled(h * acc, y[i], y1[i], rtol, atol);
        msum = (i == 0) ? sc * sc : msum + sc * sc;
      }
      const float ms = msum / (float)NV;
      int kp, fl;
      const float dt = mtgp_dp_control(ms, h, dtmin, dtmax, force_dtmin, &pid, &ctl, &kp, &fl);
      const bool keep = kp != 0;
      ++steps;
      bool stop = fl != 0;
      if (keep) {
        while (k < S && ts[k] <= tnext) {  // SaveAt(ts) through the dense output
          const float th = (ts[k] - t) / h;
          float v[NV];
#pragma unroll
          for (int i = 0; i < NV; ++i) {
            float acc = 0.0f;
#pragma unroll
            for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, CM[j], f[j][i], j == 0);
            const float ymid = MTGP_FMAF(h, acc, y[i]);
            v[i] = mtgp_dp_interp(y[i], y1[i], ymid, h * f[0][i], h * f[6][i], th);
          }
          save(k, v);
          ++k;
        }
        t = tnext;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          y[i] = y1[i];
          f[0][i] = f[6][i];  // FSAL
        }
        const bool ok = !bad(y);
        stop = stop || (prev_ok && !ok);  // Event(cond_fn_nan) (sr.py:93-94): terminate after this step
        prev_ok = ok;
      }
      if (stop || !(t < t_end) || steps >= max_steps) live = false;
      else tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
  }
  if (active && A.out.steps) A.out.steps[loff] = steps;
  if (active) {  // unsaved points are +inf (throw=False)
    float inf[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) inf[i] = kInf;
    for (; k < S; ++k) save(k, inf);
  }
  finish_group(A, Ln, tot / (float)S);
}

// --------------------------------------------------------------------------------------
// Symbolic regression with a wide state (5 <= n_var <= MTGP_MAX_DATA, BASELINE C5: the 64-dim
// "neural-ODE" SR).  One workgroup = NW = ceil(n_var / 8) waves over the same lanes (G
// individuals x Rp rollouts, like every kernel here); wave w owns components [8w, 8w + 8): it
// runs their trees, keeps x and the RK4 accumulator of those components in VGPRs, and
// publishes stage outputs through a shared, ping-ponged LDS stage vector (the data vector
// every tree reads).  The MSE (summed over components in index order, as the oracle and
// sr.py:24 do) and the termination event (any non-finite component) are reduced across the
// waves through LDS.  Per workgroup LDS: 2 x n_var columns + NW stacks + NW flag columns.
constexpr int kWideComp = 8;  // components (trees) per wave

__device__ __forceinline__ bool lane_setup_wide(const KArgs& A, Lane& L) {
  L.wave = uni(threadIdx.x >> 6);
  L.lane = threadIdx.x & 63;
  lane_place(A, L, (int)blockIdx.x);  // one workgroup per lane set
  if (L.q0 >= A.P) return false;
  const int q = L.q0 + L.g;
  L.p = q < A.P ? sched_ind(A, q) : A.P;
  L.active = (L.r < A.ro.R) && (q < A.P);
  L.rr = L.active ? L.r : 0;
  L.ptab = prog_table(A, L);
  L.jok = true;
  if (A.jit_info) L.jok = uni((int)(A.jit_info[0] == 0 && (uint64_t)(uint32_t)A.jit_info[1] <= A.jit_cap)) != 0;
  L.jtab = 0;  // lane j < n_prog: JIT unit (lane set, program j)
  if (A.jit_off && L.lane < A.n_prog) L.jtab = A.jit_off[(size_t)(L.q0 / L.G) * A.n_prog + L.lane];
  return true;
}

// Call a JIT unit in LDS-data mode (mtgp_jit.h kJitModeLds): v0 = this lane's LDS byte address of
// stage-vector slot 0; result in v8; s[32:33] collects lanes that need the interpreter.
__device__ __forceinline__ float jit_call_lds(uint64_t addr_, uint32_t lds_addr, uint64_t& flag) {
  const uint64_t addr = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)addr_) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(addr_ >> 32)) << 32;
  float acc;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "={v8}"(acc), "+{s[32:33]}"(flag)
               : [tgt] "s"(addr), "{v0}"(lds_addr)
               : "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34",
                 "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47",
                 "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "s30", "s31",
                 "s34", "s35",
                 "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "vcc", "scc", "memory");
  return acc;
}

// Call an LDS store chain (mtgp_jit.h, ABI v14): the wave's components' programs back to back, each
// result written to the output vector at v1 (slot j at + j * 256 B); the chain waits for its
// writes before returning.
__device__ __forceinline__ void jit_call_lds_store(uint64_t addr_, uint32_t lds_in, uint32_t lds_out, uint64_t& flag) {
  const uint64_t addr = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)addr_) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(addr_ >> 32)) << 32;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "+{s[32:33]}"(flag)
               : [tgt] "s"(addr), "{v0}"(lds_in), "{v1}"(lds_out)
               : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34",
                 "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47",
                 "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "s30", "s31",
                 "s34", "s35",
                 "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "vcc", "scc", "memory");
}

// LDS byte address of a pointer into shared memory
__device__ __forceinline__ uint32_t lds_address(const float* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}


// The per-save MSE (components summed in index order, sr.py:24) is needed by wave 0 only, which
// writes the fitness; the other waves skip the 64 LDS reads (every wave summing measured 0.7 %
// slower at C5, profiles/r03/v10_ab_noprog_mse.log).
template <bool TRAJ, bool JIT>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) k_sr_wide(KArgs A) {
  extern __shared__ float wl[];
  Lane Ln;
  if (!lane_setup_wide(A, Ln)) return;  // uniform over the workgroup
  if (JIT) asm volatile("s_icache_inv");  // the JIT code was written by an earlier kernel
  const int NV = A.m.n_var;
  const int NW = (NV + kWideComp - 1) / kWideComp;
  const int w = Ln.wave, lane = Ln.lane, r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* bufA = wl + lane;
  float* bufB = wl + (size_t)NV * kWave + lane;
  float* st = wl + (size_t)(2 * NV + w * kSMax) * kWave + lane;
  float* flags = wl + (size_t)(2 * NV + NW * kSMax) * kWave + lane;  // [NW] columns
  const int S = A.m.n_save;
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  const int c0 = w * kWideComp;

  // x: this wave's components of the lane's state; fx0: their stage-0 derivatives (Hermite k0 =
  // f0 dt); ax: the running b-weighted stage sum (mtgp_cstep.h)
  float x[kWideComp], ax[kWideComp], fx0[kWideComp];
#pragma unroll
  for (int t = 0; t < kWideComp; ++t) {
    x[t] = (c0 + t < NV) ? A.ro.x0[rr * NV + c0 + t] : 0.0f;
    ax[t] = fx0[t] = 0.0f;
  }
  // workgroup-wide "any component of v non-finite" for this lane (two barriers)
  auto any_bad = [&](const float (&v)[kWideComp]) {
    bool b = false;
#pragma unroll
    for (int t = 0; t < kWideComp; ++t) b = b || ((c0 + t < NV) && !mtgp_isfinite(v[t]));
    flags[w * kWave] = b ? 1.0f : 0.0f;
    __syncthreads();
    bool all = false;
    for (int v2 = 0; v2 < NW; ++v2) all = all || (flags[v2 * kWave] != 0.0f);
    __syncthreads();
    return all;
  };
  float* cur = bufA;
  float* nxt = bufB;
#pragma unroll
  for (int t = 0; t < kWideComp; ++t)
    if (c0 + t < NV) cur[(c0 + t) * kWave] = x[t];
  bool dead = !active;
  bool prev_ok = !any_bad(x);  // (its barrier also publishes cur)
  float tot = 0.0f;
  // one save point (every wave, uniform): the per-component squared errors meet in LDS (scratch
  // column buffer sq) and wave 0 sums them in index order (sr.py:24); fill: +inf, as k_sr
  // xs_of(t): component t's saved value (evaluated once per component, so the save point holds no
  // per-component array: the kernel stays within 128 VGPRs, two workgroups per CU)
  auto save_point = [&](int k, auto xs_of, bool fill, float* sq) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < kWideComp; ++t) {
      const int c = c0 + t;
      if (c < NV) {
        const float xv = xs_of(t);
        const float e = xv - A.ro.ys_true[((size_t)k * NV + c) * R + rr];
        sq[c * kWave] = e * e;
        if (TRAJ && active && A.out.xs) store_row(A.out.xs, ((size_t)k * NV + c) * PR, loff, xv, PR);
      }
    }
    __syncthreads();  // (uniform: a lane's fill flag is the same in every wave)
    if (w == 0) {  // (only wave 0 reports the fitness: finish_group)
      if (fill) {
        if (mtgp_isfinite(tot)) tot = kInf;
      } else {
        float v = sq[0];
        for (int d = 1; d < NV; ++d) v = v + sq[d * kWave];
        tot = tot + v;
      }
    }
    __syncthreads();
  };
  const bool euler = A.m.solver == MTGP_SOLVER_EULER;  // diffrax.Euler: one stage, y + f dt
  const int n_stages = euler ? 1 : 4;
  CsClock clk;
  clk.init(A);
  int k = 0;
  while (clk.live()) {  // (no FairShare: the workgroup's waves meet at a barrier every stage)
    const float dt = clk.dt();
    // (the next stage's input reads the b-weighted sum before this stage's term -- mtgp_rk4_in_acc,
    // the zero tableau entries -- which is then added: the same sums in the same order)
#pragma unroll 1
    for (int stage = 0; stage < n_stages; ++stage) {
      // trees of this wave's components on the shared stage vector; f parks in nxt
      if (JIT && Ln.jok && A.chain_store) {  // one call: this wave's components' units, results into nxt
        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_state + c0);
        uint64_t fl = 0;
#if MTGP_AB_NOPROG  // diagnostic only (A/B): the stage glue without the program calls
        (void)off;
        for (int t = 0; t < kWideComp; ++t)
          if (c0 + t < NV) nxt[(c0 + t) * kWave] = 0.0f;
#else
        jit_call_lds_store(A.jit_base + off, lds_address(cur), lds_address(nxt), fl);
#endif
        if (__builtin_expect(fl != 0, 0)) {  // lanes that need the slow sin/cos: interpret those groups
          for (int t = 0; t < kWideComp; ++t) {
            const int c = c0 + t;
            if (c >= NV) break;
            for (int gi = 0; gi < ng; ++gi) {
              if (!(fl & __ballot(Ln.g == gi && Ln.active))) continue;
              const float tv = run_one_interp<JIT && MTGP_COLD_INTERP != 0>(A, Ln, gi, A.m.prog_state + c, cur, st);
              if (Ln.g == gi) nxt[c * kWave] = tv;
            }
          }
        }
      } else if (JIT && Ln.jok) {  // one JIT unit call per component: the G groups' programs back to back
        const uint32_t la = lds_address(cur);
        for (int t = 0; t < kWideComp; ++t) {
          const int c = c0 + t;
          if (c >= NV) break;
          const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_state + c);
          uint64_t fl = 0;
          float v = jit_call_lds(A.jit_base + off, la, fl);
          if (__builtin_expect(fl != 0, 0)) {  // lanes that need the slow sin/cos: interpret those groups
            for (int gi = 0; gi < ng; ++gi) {
              if (!(fl & __ballot(Ln.g == gi && Ln.active))) continue;
              const float tv = run_one_interp<JIT && MTGP_COLD_INTERP != 0>(A, Ln, gi, A.m.prog_state + c, cur, st);
              v = (Ln.g == gi) ? tv : v;
            }
          }
          nxt[c * kWave] = v;
        }
      } else {
        for (int t = 0; t < kWideComp; ++t) {
          const int c = c0 + t;
          if (c >= NV) break;
          nxt[c * kWave] = run_groups_interp<JIT && MTGP_COLD_INTERP != 0>(A, Ln, ng, A.m.prog_state + c, cur, st, 0.0f);
        }
      }
      const bool last = stage == n_stages - 1;
#pragma unroll
      for (int t = 0; t < kWideComp; ++t) {
        const int c = c0 + t;
        if (c < NV) {
          const float kv = nxt[c * kWave];
          if (stage == 0) fx0[t] = kv;
          if (!last) nxt[c * kWave] = stage_in(stage + 1, x[t], kv, ax[t], dt);  // the next stage's input
          ax[t] = stage_acc(stage, ax[t], kv);
        }
      }
      __syncthreads();
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    // cur holds the last stage's derivatives f3 (Euler: f0); the step's end state and the event
    float x1[kWideComp];
#pragma unroll
    for (int t = 0; t < kWideComp; ++t) x1[t] = euler ? x[t] + fx0[t] * dt : mtgp_rk4_out(x[t], ax[t], dt);
    const bool bad = any_bad(x1);
    bool ev = false;
    if (!dead) {
      ev = prev_ok && bad;
      prev_ok = !bad;
    }
    while (k < S && clk.saves(A.ro.ts, k)) {  // SaveAt(ts) through this step's dense output
      const float th = mtgp_cs_rescale(clk.t, ldc(A.ro.ts, k), clk.tn);
      save_point(k, [&](int t) __attribute__((always_inline)) {  // the dense output (cs_dense), cur = f3
        const float v = euler ? mtgp_cs_linear(x[t], x1[t], th)
                              : mtgp_cs_hermite(x[t], x1[t], fx0[t] * dt, cur[(c0 + t) * kWave] * dt, th);
        return dead ? kInf : v;
      }, dead, nxt);
      ++k;
    }
    if (!dead) {
#pragma unroll
      for (int t = 0; t < kWideComp; ++t) x[t] = x1[t];
    }
    if (ev) dead = true;
#pragma unroll
    for (int t = 0; t < kWideComp; ++t)
      if (c0 + t < NV) cur[(c0 + t) * kWave] = dead ? kInf : x[t];
    __syncthreads();  // publishes cur for the next step's stage 0
    clk.advance();
    if (!TRAJ && wave_all(dead)) break;  // dead is identical in every wave: a uniform exit
  }
  if (k < S) {  // unsaved points (event / max_steps): +inf
    auto inf_of = [](int) { return kInf; };
    if (TRAJ) {
      for (; k < S; ++k) save_point(k, inf_of, true, nxt);
    } else {
      save_point(k, inf_of, true, nxt);
    }
  }
  if (w == 0) finish_group(A, Ln, tot / (float)S);
}

// --------------------------------------------------------------------------------------
// Wide-state SR (5 <= n_var <= 64) with adaptive Dopri5 + PIDController (SR_evaluator.py:57-94
// with the notebook's solver, SymbolicRegression.ipynb:136): k_sr_wide's workgroup layout (wave w
// owns components [8w, 8w + 8): their y, y1 and the seven stage derivatives stay in its VGPRs)
// with k_sr_dopri5's per-lane step control.  Every per-lane decision (error norm, accept, step
// size, event, save points) comes from quantities reduced over ALL components through LDS in
// index order, so each lane's state is identical in every wave and all barriers are uniform:
// the attempt loop, the save rounds and the +inf fill run while ANY lane needs them and commit
// per lane.  LDS: two ping-pong stage vectors + one reduction vector (n_var columns each), the
// waves' interpreter stacks and flag columns.
template <bool TRAJ, bool JIT>
__global__ void __launch_bounds__(512) k_sr_wide_dopri5(KArgs A) {
  extern __shared__ float wl[];
  Lane Ln;
  if (!lane_setup_wide(A, Ln)) return;  // uniform over the workgroup
  if (JIT) asm volatile("s_icache_inv");
  const int NV = A.m.n_var;
  const int NW = (NV + kWideComp - 1) / kWideComp;
  const int w = Ln.wave, lane = Ln.lane, r = Ln.r, rr = Ln.rr, ng = groups_live(A, Ln);
  const bool active = Ln.active;
  const int R = A.ro.R;
  float* bufs[2] = {wl + lane, wl + (size_t)NV * kWave + lane};
  float* red = wl + (size_t)2 * NV * kWave + lane;
  float* st = wl + (size_t)(3 * NV + w * kSMax) * kWave + lane;
  float* flags = wl + (size_t)(3 * NV + NW * kSMax) * kWave + lane;  // [NW] columns
  const int S = A.m.n_save, max_steps = A.m.max_steps;
  const float rtol = A.m.rtol, atol = A.m.atol, dtmin = A.m.dtmin, dtmax = A.m.dtmax;
  const size_t PR = (size_t)A.P * R;
  const int loff = Ln.p * R + r;
  const int c0 = w * kWideComp;
  const float* __restrict__ ts = A.ro.ts;
  const float t_end = ts[S - 1];
  constexpr float E[7] = MTGP_DP_TABLE_E;
  constexpr float CM[7] = MTGP_DP_TABLE_CMID;
  int buf = 0;

  // this wave's trees on stage vector `in` -> kx (the G groups' programs, JIT or interpreted)
  auto rhs = [&](const float* in, float* kx) __attribute__((always_inline)) {
    if (JIT && Ln.jok && A.chain_store) {  // one call: results into the reduction vector, read back
      const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_state + c0);
      uint64_t fl = 0;
      jit_call_lds_store(A.jit_base + off, lds_address(in), lds_address(red), fl);
#pragma unroll
      for (int t = 0; t < kWideComp; ++t) kx[t] = (c0 + t < NV) ? red[(c0 + t) * kWave] : 0.0f;
      if (__builtin_expect(fl != 0, 0)) {
        for (int t = 0; t < kWideComp; ++t) {
          const int c = c0 + t;
          if (c >= NV) break;
          for (int gi = 0; gi < ng; ++gi) {
            if (!(fl & __ballot(Ln.g == gi && Ln.active))) continue;
            const float tv = run_one_interp<JIT && MTGP_DP_COLD != 0>(A, Ln, gi, A.m.prog_state + c, in, st);
            kx[t] = (Ln.g == gi) ? tv : kx[t];
          }
        }
      }
    } else if (JIT && Ln.jok) {
      const uint32_t la = lds_address(in);
#pragma unroll
      for (int t = 0; t < kWideComp; ++t) {
        const int c = c0 + t;
        if (c >= NV) break;
        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)Ln.jtab, A.m.prog_state + c);
        uint64_t fl = 0;
        float v = jit_call_lds(A.jit_base + off, la, fl);
        if (__builtin_expect(fl != 0, 0)) {
          for (int gi = 0; gi < ng; ++gi) {
            if (!(fl & __ballot(Ln.g == gi && Ln.active))) continue;
            const float tv = run_one_interp<JIT && MTGP_DP_COLD != 0>(A, Ln, gi, A.m.prog_state + c, in, st);
            v = (Ln.g == gi) ? tv : v;
          }
        }
        kx[t] = v;
      }
    } else {
#pragma unroll
      for (int t = 0; t < kWideComp; ++t) {
        const int c = c0 + t;
        if (c >= NV) break;
        kx[t] = run_groups_interp<JIT && MTGP_DP_COLD != 0>(A, Ln, ng, A.m.prog_state + c, in, st, 0.0f);
      }
    }
  };
  // sum over all components in index order of the values this wave puts in red (uniform barriers)
  auto reduce = [&]() __attribute__((always_inline)) {
    __syncthreads();
    float s = red[0];
    for (int d = 1; d < NV; ++d) s = s + red[d * kWave];
    __syncthreads();
    return s;
  };
  auto any_bad = [&](const float* v) __attribute__((always_inline)) {
    bool b = false;
#pragma unroll
    for (int t = 0; t < kWideComp; ++t) b = b || ((c0 + t < NV) && !mtgp_isfinite(v[t]));
    flags[w * kWave] = b ? 1.0f : 0.0f;
    __syncthreads();
    bool all = false;
    for (int q = 0; q < NW; ++q) all = all || (flags[q * kWave] != 0.0f);
    __syncthreads();
    return all;
  };
  float tot = 0.0f;
  // MSE term of save point k for the lanes with `pend` (state v of this wave's components)
  auto save = [&](int k, const float* v, bool pend) __attribute__((always_inline)) {
    const int kk = k < S ? k : S - 1;
#pragma unroll
    for (int t = 0; t < kWideComp; ++t) {
      const int c = c0 + t;
      if (c < NV) {
        const float e = v[t] - A.ro.ys_true[((size_t)kk * NV + c) * R + rr];
        red[c * kWave] = e * e;
        if (TRAJ && pend && active && A.out.xs)
          traj_put_dp(A.out.xs, A.out.traj_layout == MTGP_TRAJ_LANE_MAJOR, kk, c, NV, loff, PR, S, v[t]);
      }
    }
    const float sq = reduce();
    if (pend) tot = tot + sq;
  };

  float y[kWideComp], y1[kWideComp], kx[kWideComp], f[7][kWideComp];
#pragma unroll
  for (int t = 0; t < kWideComp; ++t) {
    y[t] = (c0 + t < NV) ? A.ro.x0[rr * NV + c0 + t] : 0.0f;
    if (c0 + t < NV) bufs[0][(c0 + t) * kWave] = y[t];
  }
  save(0, y, true);  // (its barrier also publishes the stage vector)
  int k = 1, steps = 0;
  bool prev_ok = !any_bad(y);
  MtgpDpCtl ctl{1.0f, 1.0f, 0};
  const MtgpDpPid pid = dp_pid(A.m);
  const int force_dtmin = !A.m.no_force_dtmin;
  float t = ts[0];
  float tnext = t + A.m.h;
  tnext = tnext > t_end ? t_end : tnext;
  rhs(bufs[0], kx);  // FSAL seed f0 = f(t0, y0)
#pragma unroll
  for (int i = 0; i < kWideComp; ++i) f[0][i] = kx[i];
  bool live = active && t < t_end && steps < max_steps;
  while (wave_any(live)) {  // identical in every wave of the workgroup
    const float h = tnext - t;
#pragma unroll 1
    for (int s = 1; s <= 6; ++s) {
      buf ^= 1;
      float* in = bufs[buf];
      float acc[kWideComp];
      dp_stage_sum<kWideComp>(s, f, acc);
#pragma unroll
      for (int i = 0; i < kWideComp; ++i) {
        const float yi = MTGP_FMAF(h, acc[i], y[i]);
        y1[i] = yi;
        if (c0 + i < NV) in[(c0 + i) * kWave] = yi;
      }
      __syncthreads();  // the other buffer is not read again before the next barrier
      rhs(in, kx);
      dp_file<kWideComp>(s, f, kx);
    }
    // error norm: rms over all components (index order) of the scaled error estimate
#pragma unroll
    for (int i = 0; i < kWideComp; ++i) {
      float acc = 0.0f;
#pragma unroll
      for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], f[j][i], j == 0);
      const float sc = mtgp_dp_scaled(h * acc, y[i], y1[i], rtol, atol);
      if (c0 + i < NV) red[(c0 + i) * kWave] = sc * sc;
    }
    const float msum = reduce();
    const float ms = msum / (float)NV;
    MtgpDpCtl nctl = ctl;  // committed by live lanes only
    int kp, fl;
    const float dt = mtgp_dp_control(ms, h, dtmin, dtmax, force_dtmin, &pid, &nctl, &kp, &fl);
    const bool keep = kp != 0;
    const bool acc_step = live && keep;
    // SaveAt(ts) through the dense output, in rounds over the lanes that pass save points
    while (wave_any(acc_step && k < S && ts[k < S ? k : S - 1] <= tnext)) {
      const bool pend = acc_step && k < S && ts[k < S ? k : S - 1] <= tnext;
      const float th = (ts[k < S ? k : S - 1] - t) / h;
      float v[kWideComp];
#pragma unroll
      for (int i = 0; i < kWideComp; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, CM[j], f[j][i], j == 0);
        const float ymid = MTGP_FMAF(h, acc, y[i]);
        v[i] = mtgp_dp_interp(y[i], y1[i], ymid, h * f[0][i], h * f[6][i], th);
      }
      save(k, v, pend);
      if (pend) ++k;
    }
    if (acc_step) {
      t = tnext;
#pragma unroll
      for (int i = 0; i < kWideComp; ++i) {
        y[i] = y1[i];
        f[0][i] = f[6][i];  // FSAL
      }
    }
    const bool ok = !any_bad(y);
    if (live) {
      ctl = nctl;
      ++steps;
      bool stop = fl != 0;
      if (keep) {
        stop = stop || (prev_ok && !ok);  // Event(cond_fn_nan) (sr.py:93-94): terminate after this step
        prev_ok = ok;
      }
      if (stop || !(t < t_end) || steps >= max_steps) live = false;
      else tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
  }
  if (w == 0 && active && A.out.steps) A.out.steps[loff] = steps;
  float inf[kWideComp];
#pragma unroll
  for (int i = 0; i < kWideComp; ++i) inf[i] = kInf;
  while (wave_any(active && k < S)) {  // unsaved points are +inf (throw=False)
    const bool pend = active && k < S;
    save(k, inf, pend);
    if (pend) ++k;
  }
  if (w == 0) finish_group(A, Ln, tot / (float)S);
}

#if MTGP_TU_MAIN
// --------------------------------------------------------------------------------------
// tree_evaluator plugin (gp.py:390-401): every program on M shared data vectors.
// One wave per (individual, program, chunk of 64 data vectors); data vector in LDS.
__global__ void __launch_bounds__(256) k_eval_programs(const MtgpInstr* __restrict__ prog,
                                                       const int32_t* __restrict__ plen, int n_prog, int L,
                                                       int P, const float* __restrict__ data, int M,
                                                       int n_data, float* __restrict__ out) {
  extern __shared__ float dyn_lds[];
  const int wave = uni(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int chunks = (M + 63) / 64;
  const long item = (long)blockIdx.x * kWavesPerBlock + wave;
  if (item >= (long)P * n_prog * chunks) return;
  const int ch = uni((int)(item % chunks));
  const long pj = item / chunks;
  const int m = ch * 64 + lane;
  const bool active = m < M;
  float* dcol = dyn_lds + (size_t)wave * (n_data + kSMax) * kWave + lane;
  float* st = dcol + (size_t)n_data * kWave;
  for (int d = 0; d < n_data; ++d) dcol[d * kWave] = active ? data[(size_t)m * n_data + d] : 0.0f;
  const float v = run_prog(prog + (size_t)pj * L, dcol, st);
  if (active) out[(size_t)pj * M + m] = v;
}

// --------------------------------------------------------------------------------------
// Flatten: one thread per (individual, program spec), row-uniform control flow
// (mtgp_flatten_uniform.h): pass 1 resolves and sizes the rows in ascending order into an LDS
// table [row][lane], pass 2 walks the rows in descending order and writes every reachable node's
// word at its postorder position.  Rows are streamed from HBM eight at a time, the next eight in
// flight while the current ones are resolved.  Optionally the lane also sizes its program's JIT
// translation (jit_words: fall-through code words, < 0 if untranslatable; jit_cost: the schedule
// weight), so the JIT build needs no translation pass of its own before the code is emitted.
constexpr int32_t kFlatSerial = 0x7fff;  // status of a program left to k_flatten_serial

// JIT sizing of one flattened program (mtgp_flatten_ex jit_words / jit_cost)
__device__ __forceinline__ void flat_jit_size(const MtgpInstr* out, int L, int n, int32_t* jit_words_out,
                                              int32_t* jit_cost_out, size_t pj, int jit_mode) {
  if (!jit_words_out && !jit_cost_out) return;
  mtgp::JitOut o{nullptr, 0};
  const int rc = mtgp::jit_program(o, out, L, false, jit_mode);
  if (jit_words_out) jit_words_out[pj] = rc < 0 ? rc : o.n;
  if (jit_cost_out) {  // = k_jit_cost: executed words of the callable translation / 4
    const int c = rc < 0 ? rc : (o.n + 1 + o.sub);
    jit_cost_out[pj] = c > 0 ? (c + 3) / 4 : (n > 0 ? n : 0);
  }
}

// The same sizing by a whole wave (register-data mode).  In register mode the code of an
// instruction depends on its opcode alone (operands only select registers / literals), apart from
// the slot-range and stack checks, so jit_program's translation of every opcode is probed once on
// the host into JitOpTable (jit_op_table) and lane l sizes instructions l, l + 64, ... by table
// lookup (no divergent translation); a prefix sum of the stack effects gives the depth each push /
// pop sees, and the first failing instruction in program order gives the status -- within one
// instruction a slot / opcode error precedes a stack error, as in jit_program.  Identical outputs to
// flat_jit_size (tests/test_gpu_build.py compares them with the host translation).
struct JitOpTable {
  uint8_t words[64];  // code words of the opcode's translation
  uint8_t flags[64];  // kOpValid | kOpIbSlot | kOpAxSlot | kOpPush | kOpPop
  uint8_t sub[64];    // executed words of the subroutine it calls (JitOut::sub; 0: none)
};
enum : uint8_t { kOpValid = 1, kOpIbSlot = 4, kOpAxSlot = 8, kOpPush = 16, kOpPop = 32 };
static_assert(MTGP_OP_COUNT <= 64, "JitOpTable holds 64 opcodes");

JitOpTable jit_op_table() {
  JitOpTable t{};
  MtgpInstr end;
  end.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
  end.imm = 0.0f;
  for (int code = 0; code < 64; ++code) {
    if (code == MTGP_OP_END) continue;  // never sized (instructions before the END only)
    const int d = mtgp::jit_stack_delta((uint32_t)code);
    auto probe = [&](uint32_t ax, uint32_t ib, mtgp::JitOut& o) {
      MtgpInstr p[2] = {{(uint32_t)code << MTGP_OP_SHIFT | ax, 0.0f}, end};
      std::memcpy(&p[0].imm, &ib, 4);
      return mtgp::jit_program(o, p, 2, false, mtgp::kJitModeRegs, 0, mtgp::kJitPre, 0, nullptr, d < 0 ? 1 : 0);
    };
    mtgp::JitOut o{nullptr, 0};
    if (probe(0u, 0u, o) != mtgp::kJitOk) continue;  // not an opcode
    uint8_t f = kOpValid | (d > 0 ? kOpPush : 0) | (d < 0 ? kOpPop : 0);
    const uint32_t far = (uint32_t)mtgp::kJitMaxData * MTGP_SLOT_BYTES;
    mtgp::JitOut o1{nullptr, 0}, o2{nullptr, 0};
    if (probe(0u, far, o1) == mtgp::kJitErrSlot) f |= kOpIbSlot;
    if (probe(far, 0u, o2) == mtgp::kJitErrSlot) f |= kOpAxSlot;
    t.words[code] = (uint8_t)o.n;
    t.flags[code] = f;
    t.sub[code] = (uint8_t)o.sub;
  }
  return t;
}

// LP: the lanes sizing one program (the wave, or a 32-lane half of it -- k_flatten_wave's two
// programs per wave); lane = the lane within them, KI chunks of LP instructions
template <int KI, int LP = kWave>
__device__ __forceinline__ void flat_jit_size_wave(const MtgpInstr* prog, int n, const JitOpTable& T,
                                                   int32_t* jit_words_out, int32_t* jit_cost_out, size_t pj, int lane) {
  const int shift = LP == kWave ? 0 : (int)(threadIdx.x & (kWave - 1) & ~(LP - 1));  // this segment's first lane
  int words = 0, sub = 0, carry = 0, rc = 0;
  bool failed = false;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int i = k * LP + lane;
    const bool in = i < n;
    int d = 0, e = 0;
    if (in) {
      const MtgpInstr x = prog[i];
      const uint32_t code = x.op >> MTGP_OP_SHIFT;
      const uint32_t f = code < 64u ? T.flags[code] : 0u;
      uint32_t ib;
      __builtin_memcpy(&ib, &x.imm, 4);
      const int sib = (int)(ib / MTGP_SLOT_BYTES), sax = (int)((x.op & 0xffffffu) / MTGP_SLOT_BYTES);
      if (!(f & kOpValid)) e = mtgp::kJitErrOpcode;
      else if (((f & kOpIbSlot) && sib >= mtgp::kJitMaxData) || ((f & kOpAxSlot) && sax >= mtgp::kJitMaxData))
        e = mtgp::kJitErrSlot;
      d = (f & kOpPush) ? 1 : ((f & kOpPop) ? -1 : 0);
      words += code < 64u ? T.words[code] : 0;
      sub += code < 64u ? T.sub[code] : 0;
    }
    int incl = d;  // inclusive prefix sum of the stack effects over this chunk
#pragma unroll
    for (int off = 1; off < LP; off <<= 1) {
      const int v = __shfl_up(incl, off, LP);
      if (lane >= off) incl += v;
    }
    const int before = carry + incl - d;
    if (in && e == 0 && ((d > 0 && before >= MTGP_STACK_MAX) || (d < 0 && before <= 0))) e = mtgp::kJitErrStack;
    carry += __shfl(incl, LP - 1, LP);
    uint64_t bad = __ballot(in && e != 0) >> shift;
    if (LP < kWave) bad &= (1ull << LP) - 1ull;
    if (!failed && bad) {
      failed = true;
      rc = __shfl(e, __ffsll((unsigned long long)bad) - 1, LP);
    }
  }
#pragma unroll
  for (int off = LP / 2; off > 0; off >>= 1) {
    words += __shfl_xor(words, off, LP);
    sub += __shfl_xor(sub, off, LP);
  }
  if (lane == 0) {
    if (jit_words_out) jit_words_out[pj] = failed ? rc : words;
    if (jit_cost_out) {  // = flat_jit_size
      const int c = failed ? rc : (words + 1 + sub);
      jit_cost_out[pj] = c > 0 ? (c + 3) / 4 : (n > 0 ? n : 0);
    }
  }
}

// The same sizing by a whole wave in LDS-data mode (the wide-state SR kernel's code).  An
// instruction's code is its register-mode code (JitOpTable) plus, per data operand that is not
// preloaded, a load at the use (ds_read_b32 + s_waitcnt: 3 words); the program starts with the
// preloads of the first kJitPreSlots distinct slots it reads (2 words each) and one s_waitcnt.
// "First distinct": each slot's first operand position (2 i + k, ib before ax) by an LDS atomicMin,
// then a slot is preloaded iff fewer than kJitPreSlots slots occur before it.  Status as in
// jit_program: a slot >= MTGP_MAX_DATA anywhere (its preload scan runs first), else the first
// opcode / stack error in program order.  fpos: MTGP_MAX_DATA ints of this wave's LDS.
template <int KI>
__device__ __forceinline__ void flat_jit_size_wave_lds(const MtgpInstr* prog, int n, const JitOpTable& T,
                                                       int32_t* jit_words_out, int32_t* jit_cost_out, size_t pj,
                                                       int lane, int* fpos) {
  static_assert(MTGP_MAX_DATA <= kWave, "one lane per data slot");
  if (lane < MTGP_MAX_DATA) fpos[lane] = 0x7fffffff;
  __syncthreads();
  int sa[KI], sb[KI];  // this lane's data-operand slots per chunk (-1: none)
  bool far = false;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int i = k * kWave + lane;
    sa[k] = sb[k] = -1;
    if (i < n) {
      const MtgpInstr x = prog[i];
      const uint32_t code = x.op >> MTGP_OP_SHIFT;
      const uint32_t f = code < 64u ? T.flags[code] : 0u;
      uint32_t ib;
      __builtin_memcpy(&ib, &x.imm, 4);
      if (f & kOpIbSlot) sa[k] = (int)(ib / MTGP_SLOT_BYTES);
      if (f & kOpAxSlot) sb[k] = (int)((x.op & 0xffffffu) / MTGP_SLOT_BYTES);
      far = far || sa[k] >= MTGP_MAX_DATA || sb[k] >= MTGP_MAX_DATA;
      if (sa[k] >= 0 && sa[k] < MTGP_MAX_DATA) atomicMin(&fpos[sa[k]], 2 * i);
      if (sb[k] >= 0 && sb[k] < MTGP_MAX_DATA) atomicMin(&fpos[sb[k]], 2 * i + 1);
    }
  }
  __syncthreads();
  const bool slot_err = wave_any(far);
  // lane s: is slot s preloaded (fewer than kJitPreSlots slots first occur before it)
  bool pre = false;
  if (lane < MTGP_MAX_DATA) {
    const int mine = fpos[lane];
    int before = 0;
#pragma unroll 8
    for (int t = 0; t < MTGP_MAX_DATA; ++t) before += fpos[t] < mine ? 1 : 0;
    pre = mine != 0x7fffffff && before < mtgp::kJitPreSlots;
  }
  const uint64_t pre_mask = __ballot(pre);
  const int npre = __popcll(pre_mask);
  int words = 0, sub = 0, carry = 0, rc = 0;
  bool failed = false;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int i = k * kWave + lane;
    const bool in = i < n;
    int d = 0, e = 0;
    if (in) {
      const uint32_t code = prog[i].op >> MTGP_OP_SHIFT;
      const uint32_t f = code < 64u ? T.flags[code] : 0u;
      if (!(f & kOpValid)) e = mtgp::kJitErrOpcode;
      d = (f & kOpPush) ? 1 : ((f & kOpPop) ? -1 : 0);
      words += code < 64u ? T.words[code] : 0;
      if (sa[k] >= 0 && sa[k] < MTGP_MAX_DATA && !((pre_mask >> sa[k]) & 1ull)) words += 3;
      if (sb[k] >= 0 && sb[k] < MTGP_MAX_DATA && !((pre_mask >> sb[k]) & 1ull)) words += 3;
      sub += code < 64u ? T.sub[code] : 0;
    }
    int incl = d;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    const int before = carry + incl - d;
    if (in && e == 0 && ((d > 0 && before >= MTGP_STACK_MAX) || (d < 0 && before <= 0))) e = mtgp::kJitErrStack;
    carry += __shfl(incl, kWave - 1);
    const uint64_t bad = __ballot(in && e != 0);
    if (!failed && bad) {
      failed = true;
      rc = __shfl(e, __ffsll((unsigned long long)bad) - 1);
    }
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    words += __shfl_xor(words, off);
    sub += __shfl_xor(sub, off);
  }
  if (slot_err) {
    failed = true;
    rc = mtgp::kJitErrSlot;
  }
  words += npre > 0 ? 2 * mtgp::jit_preload_instrs(npre) + 1 : 0;  // paired preloads + the wait
  if (lane == 0) {
    if (jit_words_out) jit_words_out[pj] = failed ? rc : words;
    if (jit_cost_out) {  // = flat_jit_size
      const int c = failed ? rc : (words + 1 + sub);
      jit_cost_out[pj] = c > 0 ? (c + 3) / 4 : (n > 0 ? n : 0);
    }
  }
}

// The serial flatten_tree for the programs k_flatten flagged (a row reached from two parents):
// a small grid strides over all programs, so the private row table it needs is allocated for few
// waves only.
template <int NMAX>
__global__ void __launch_bounds__(64) k_flatten_serial(const float* __restrict__ pop, int P, int T, int N,
                                                       MtgpNodeLibrary lib, const MtgpProgramSpec* __restrict__ specs,
                                                       int n_prog, int L, MtgpInstr* prog_out, int32_t* len_out,
                                                       int32_t* status_out, int32_t* jit_words_out,
                                                       int32_t* jit_cost_out, int jit_mode) {
  const long total = (long)P * n_prog;
  for (long pj = (long)blockIdx.x * blockDim.x + threadIdx.x; pj < total; pj += (long)gridDim.x * blockDim.x) {
    if (status_out[pj] != kFlatSerial) continue;
    const int p = (int)(pj / n_prog), j = (int)(pj % n_prog);
    const MtgpProgramSpec sp = specs[j];
    MtgpInstr* out = prog_out + (size_t)pj * L;
    mtgp::RowInfo info[NMAX];
    const int n = mtgp::flatten_tree(pop + ((size_t)p * T + sp.tree) * N * 4, N, &lib, sp.n_data, sp.zero_mask, out,
                                     L, info, nullptr, sp.gap_at, sp.gap);
    len_out[pj] = n > 0 ? n : 0;
    status_out[pj] = n > 0 ? 0 : -n;
    flat_jit_size(out, L, n, jit_words_out, jit_cost_out, (size_t)pj, jit_mode);
  }
}

// lanes per block: the flatten is issue-latency bound (one tree per lane, few lanes in total), so
// several small waves per SIMD beat one full one

// The lane-per-program flattener is the round-1 design, kept for A/B runs only: built with
// -DMTGP_AB_FLAT_LANE=1 (MTGP_FLAT_MODE=lane then selects it); the product launches k_flatten_wave.
template <int NMAX, int TPB>
__global__ void __launch_bounds__(TPB) k_flatten(const float* __restrict__ pop, int P, int T, int N,
                                                            MtgpNodeLibrary lib,
                                                            const MtgpProgramSpec* __restrict__ specs, int n_prog,
                                                            int L, MtgpInstr* prog_out, int32_t* len_out,
                                                            int32_t* nodes_out, int32_t* status_out,
                                                            int32_t* jit_words_out, int32_t* jit_cost_out,
                                                            int jit_mode) {
  using namespace mtgp;
  __shared__ uint32_t s_w[NMAX * TPB];    // packed row record (u_pack)
  __shared__ uint32_t s_len[NMAX * TPB];  // unfused length (low 16, saturated) | fused length (high 16)
  __shared__ float s_cv[NMAX * TPB];      // folded constant
  __shared__ int32_t s_pos[NMAX * TPB];   // pass 2: first word of the node's code | push << 16
  __shared__ int8_t s_fn[MTGP_MAX_FUNCS];
  for (int k = threadIdx.x; k < MTGP_MAX_FUNCS; k += TPB) s_fn[k] = lib.fn[k];
  __syncthreads();
  const long gid = (long)blockIdx.x * TPB + threadIdx.x;
  if (gid >= (long)P * n_prog) return;
  const int lane = threadIdx.x;
  const int p = (int)(gid / n_prog), j = (int)(gid % n_prog);
  const MtgpProgramSpec sp = specs[j];
  const float4* tr = reinterpret_cast<const float4*>(pop + ((size_t)p * T + sp.tree) * N * 4);
  const size_t pj = (size_t)p * n_prog + j;
  MtgpInstr* out = prog_out + pj * L;
  const int cap = L - 1;
  const int n_funcs = lib.n_funcs, var_start = lib.var_start, n_data = sp.n_data;
  const uint64_t zmask = sp.zero_mask;
#define MTGP_UAT(i) ((i) * TPB + lane)
  // operand row jj of row i: an evaluated row (its table entry) or, for jj >= i, the original
  // value column (gp.py:366-369)
  auto operand = [&](int jj, int i, uint32_t& w, ULeaf& lf, int& len, int& flen, bool& leaf) {
    if (jj < i) {
      w = s_w[MTGP_UAT(jj)];
      const uint32_t ln = s_len[MTGP_UAT(jj)];
      len = (int)(ln & 0xffffu);
      flen = (int)(ln >> 16);
      lf.isc = u_isc(w);
      lf.v = s_cv[MTGP_UAT(jj)];
      lf.slot = u_slot(w);
      leaf = u_leaf(w);
    } else {
      w = u_pack(K_CONST, 0, 0, 1, 1, 0);
      lf.isc = true;
      lf.v = tr[jj].w;
      lf.slot = 0;
      len = flen = 1;
      leaf = true;
    }
  };
  // ---- pass 1: resolve + size (resolve_row / size_row) in row order
  int cnt = 0;  // non-empty rows of this tree (gp.py:424)
  float4 nxt[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) nxt[k] = k < N ? tr[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i0 = 0; i0 < N; i0 += 8) {
    float4 cur[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cur[k] = nxt[k];
      nxt[k] = (i0 + 8 + k < N) ? tr[i0 + 8 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k;
      if (i >= N) break;
      const float4 row = cur[k];
      cnt += row.x != 0.0f ? 1 : 0;
      uint32_t kind = K_CONST, fnc = MTGP_FN_ZERO, slot = 0, isc = 1, afirst = 1, need = 0;
      int len = 1, flen = 1;
      float cv = 0.0f;
      if (row.x == 1.0f) {  // coefficient (gp.py:372 select)
        cv = row.w;
      } else {
        int32_t f = f2i_sat(row.x);
        f = f < 0 ? 0 : (f > n_funcs - 1 ? n_funcs - 1 : f);
        const int fn = s_fn[f];
        if (fn == MTGP_FN_VAR) {
          int sl = f - var_start;
          if (sl > n_data - 1) sl = n_data - 1;
          slot = (uint32_t)(sl >= sp.gap_at ? sl + sp.gap : sl);  // MtgpProgramSpec.gap
          if (!((zmask >> sl) & 1ull)) { kind = K_VAR; isc = 0; }
        } else if (fn_arity(fn) > 0) {
          const int ar = fn_arity(fn);
          fnc = (uint32_t)fn;
          kind = ar == 1 ? K_UNARY : K_BINARY;
          uint32_t wa, wb = 0;
          ULeaf la, lb;
          lb.isc = true; lb.v = 0.0f; lb.slot = 0;
          int lena, flena, lenb = 1, flenb = 1;
          bool leafa, leafb = true;
          operand(norm_index(row.y, N), i, wa, la, lena, flena, leafa);
          if (ar == 2) operand(norm_index(row.z, N), i, wb, lb, lenb, flenb, leafb);
          if (la.isc && lb.isc) {  // constant subtree: folded with the kernel's fp32 primitives
            cv = apply_fn(fn, la.v, ar == 1 ? 0.0f : lb.v);
          } else {
            isc = 0;
            if (ar == 1) {
              if (leafa) { len = 2; flen = unary_fuses(fn) ? 1 : 2; }
              else { len = lena + 1; flen = flena + 1; need = u_need(wa); }
            } else if (leafa && leafb) {
              len = 2; flen = 1;
            } else if (leafb) {
              len = lena + 1; flen = flena + 1; need = u_need(wa);
            } else if (leafa) {
              len = lenb + 1; flen = flenb + 1; need = u_need(wb);
            } else {
              const uint32_t pa = u_need(wa), qb = u_need(wb);
              len = lena + lenb + 1;
              flen = flena + flenb + 1;
              if (pa >= qb) { afirst = 1; need = pa > qb + 1 ? pa : qb + 1; }
              else { afirst = 0; need = qb > pa + 1 ? qb : pa + 1; }
            }
          }
        }  // else: empty node (gp.py:135) -> +0.0
      }
      s_w[MTGP_UAT(i)] = u_pack(kind, fnc, slot, isc, afirst, need > 31u ? 31u : need);
      s_len[MTGP_UAT(i)] = (uint32_t)(len > 65535 ? 65535 : len) | (uint32_t)(flen > 65535 ? 65535 : flen) << 16;
      s_cv[MTGP_UAT(i)] = cv;
    }
  }
  const uint32_t wr = s_w[MTGP_UAT(N - 1)], lr = s_len[MTGP_UAT(N - 1)];
  int n;
  if ((int)u_need(wr) > MTGP_STACK_MAX) n = -MTGP_ERR_STACK;
  else if ((int)(lr & 0xffffu) > cap) n = -MTGP_ERR_PROG_TOO_LONG;
  else n = (int)(lr >> 16);
  // ---- pass 2: postorder positions top-down, one word per node
  bool shared = false;
  if (n > 0) {
    if (u_leaf(wr)) {  // the whole tree is one leaf
      ULeaf x;
      x.isc = u_isc(wr); x.v = s_cv[MTGP_UAT(N - 1)]; x.slot = u_slot(wr);
      out[0] = u_load(x, false);
    } else {
      UBits<NMAX> reach;
      reach.clear();
      reach.set(N - 1);
      s_pos[MTGP_UAT(N - 1)] = 0;
      for (int i = N - 1; i >= 0; --i) {
        if (!reach.test(i)) continue;
        const uint32_t w = s_w[MTGP_UAT(i)];
        const int pp = s_pos[MTGP_UAT(i)], pos = pp & 0xffff;
        const bool push = (pp >> 16) != 0;
        const float4 row = tr[i];
        const int fn = (int)u_fn(w);
        uint32_t wa, wb;
        ULeaf la, lb;
        int lena, flena, lenb = 1, flenb = 1;
        bool leafa, leafb = true;
        const int ja = norm_index(row.y, N);
        operand(ja, i, wa, la, lena, flena, leafa);
        int jb = 0;
        if (u_kind(w) == K_BINARY) {
          jb = norm_index(row.z, N);
          operand(jb, i, wb, lb, lenb, flenb, leafb);
        }
        auto visit = [&](int c, int cpos, bool cpush) {
          shared = shared || reach.test(c);  // a sub-DAG reached twice: emitted twice by the walk
          reach.set(c);
          s_pos[MTGP_UAT(c)] = cpos | (cpush ? 1 << 16 : 0);
        };
        MtgpInstr x;
        if (u_kind(w) == K_UNARY) {
          const MtgpInstr un = u_instr(mtgp::unary_op(fn), 0, 0.0f);
          if (leafa) {
            MtgpInstr w2[2];
            const int nw = u_unary_leaf(fn, la, push, w2);
            for (int q = 0; q < nw; ++q) out[pos + q] = w2[q];
          } else { visit(ja, pos, push); out[pos + flena] = un; }
        } else if (leafa && leafb) {
          fuse_pair(u_load(la, push), u_op_leaf(fn, 0, lb), &x);
          out[pos] = x;
        } else if (leafb) {
          visit(ja, pos, push);
          out[pos + flena] = u_op_leaf(fn, 0, lb);
        } else if (leafa) {
          visit(jb, pos, push);
          out[pos + flenb] = u_op_leaf(fn, 1, la);
        } else {
          const bool af = u_afirst(w) != 0;
          const int f1 = af ? flena : flenb, f2 = af ? flenb : flena;
          visit(af ? ja : jb, pos, push);
          visit(af ? jb : ja, pos + f1, true);
          out[pos + f1 + f2] = u_op_stack(fn, af ? 1 : 0);
        }
      }
    }
  }
#undef MTGP_UAT
  if (shared) {
    // arbitrary arrays only: the serial walk duplicates the shared subtree -- left to
    // k_flatten_serial, so that this kernel needs no private row table (scratch)
    len_out[pj] = 0;
    status_out[pj] = kFlatSerial;
  } else {
    MtgpInstr e;
    e.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
    e.imm = 0.0f;
    out[n > 0 ? n : 0] = e;
    len_out[pj] = n > 0 ? n : 0;
    status_out[pj] = n > 0 ? 0 : -n;
    flat_jit_size(out, L, n, jit_words_out, jit_cost_out, pj, jit_mode);
  }
  // node count (gp.py:424 parsimony): the individual's trees are shared out over its n_prog
  // lanes (tree t -> lane t % n_prog) and summed with integer atomics into the zeroed nodes_out
  int c = 0;
  for (int t = j; t < T; t += n_prog) c += (t == sp.tree) ? cnt : count_nodes(pop + ((size_t)p * T + t) * N * 4, N);
  if (c != 0) atomicAdd(&nodes_out[p], c);
}

// Trees per individual up to which k_flatten_wave stores node counts directly (see its end).
// (Four independent waves per flatten block with wave-level syncs measured slower: 90 vs 71 us at
// C3, a block holds its LDS and wave slots until its slowest program is done; r02/v18.)
constexpr int kFlatDirectTrees = 8;
// waves resident at once at eight per SIMD (256 CUs x 4 SIMDs x 8): the build kernels pack two or
// four programs / JIT units per wave only when one per wave would need more than one such round
constexpr long kResidentWaves = 8192;

// Flatten, one WAVE per (individual, program spec): lane l owns rows l, l + 64, ... (NMAX / 64 per
// lane), loaded with one coalesced 1-KB read per 64 rows.  The same two passes as k_flatten, but
// level-synchronous over the tree instead of serial over the rows:
//   pass 1: a row resolves (record, lengths, folded constant; mtgp_flatten_uniform.h) in the first
//     round after its operand rows (j < i) have resolved -- rounds = the height of the dependency
//     DAG, not N;
//   pass 2: a reached row emits its word at the postorder position its parent assigned and
//     assigns its children's -- rounds = the tree height.  A row reached twice (LDS atomic reach
//     counter; only in arbitrary arrays) leaves the program to k_flatten_serial.
// The tables are per wave in LDS (24 B per row), so the occupancy no longer falls with N (the
// lane-per-tree kernel needs 16 B x N per LANE).  Output = k_flatten's word for word.
// (8 waves per SIMD: the kernel is latency-bound -- one wave walks a tree level by level through
// LDS -- so occupancy is its throughput; 64 VGPRs fit without spills for NMAX <= 128)
template <int NMAX, int LP = kWave>  // LP: lanes per program (32: two programs per wave)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NMAX <= 128 ? 8 : 4)))
k_flatten_wave(const float* __restrict__ pop, int P, int T, int N,
                                                     MtgpNodeLibrary lib, const MtgpProgramSpec* __restrict__ specs,
                                                     int n_prog, int L, MtgpInstr* prog_out, int32_t* len_out,
                                                     int32_t* nodes_out, int32_t* status_out, int32_t* jit_words_out,
                                                     int32_t* jit_cost_out, int jit_mode, JitOpTable optab) {
  using namespace mtgp;
  static_assert(LP == kWave || LP == kWave / 2, "a program per wave or per half");
  constexpr int PPW = kWave / LP;  // programs per wave
  constexpr int RPL = NMAX / LP;   // rows per lane
  struct Tables {          // one program's tables (24 B per row + the program as written)
    uint32_t w[NMAX];       // packed row record (u_pack)
    uint32_t len[NMAX];     // unfused length (low 16, saturated) | fused length (high 16)
    float cv[NMAX];         // folded constant
    float val[NMAX];        // the original value column (operands j >= i, gp.py:366-369)
    int32_t pos[NMAX];      // pass 2: first word of the node's code | push << 16
    uint32_t flag[NMAX];    // pass 1: resolved; pass 2: times reached
    MtgpInstr prog[NMAX + 8];  // the program as written (read back by the JIT sizing)
  };
  __shared__ Tables s_tab[PPW];
  __shared__ int8_t s_fn[MTGP_MAX_FUNCS];
  __shared__ int s_fpos[MTGP_MAX_DATA];   // LDS-data sizing: first operand position per data slot
  const int half = LP == kWave ? 0 : (int)(threadIdx.x / LP);
  const int lane = threadIdx.x & (LP - 1);  // the lane within this program's lanes
  Tables& S = s_tab[half];  // (one base address; the tables at constant offsets from it)
  // this program's lanes' ballot (the other program's lanes masked off)
  auto seg_ballot = [&](bool x) -> uint64_t {
    if constexpr (LP == kWave) return __ballot(x);
    else return (__ballot(x) >> (half * LP)) & ((1ull << LP) - 1ull);
  };
  for (int k = threadIdx.x; k < MTGP_MAX_FUNCS; k += kWave) s_fn[k] = lib.fn[k];
  const long pj = (long)blockIdx.x * PPW + half;
  if (pj >= (long)P * n_prog) return;  // (one wave per block: the other program's lanes run on alone)
  const int p = (int)(pj / n_prog), j = (int)(pj % n_prog);
  const MtgpProgramSpec sp = specs[j];
  const float4* tr = reinterpret_cast<const float4*>(pop + ((size_t)p * T + sp.tree) * N * 4);
  MtgpInstr* out = prog_out + (size_t)pj * L;
  const int cap = L - 1;
  const int n_funcs = lib.n_funcs, var_start = lib.var_start, n_data = sp.n_data;
  const uint64_t zmask = sp.zero_mask;
  float4 row[RPL];
  int cnt = 0;  // non-empty rows of this tree (gp.py:424)
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    const int i = k * LP + lane;
    row[k] = i < N ? tr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    S.val[i] = row[k].w;
    cnt += __popcll(seg_ballot(i < N && row[k].x != 0.0f));
  }
  // Few trees (T <= kFlatDirectTrees): the individual's first program counts them all (see the end);
  // the other trees' node columns are loaded here, in flight together with this tree's rows,
  // instead of one dependent load per tree after the passes
  const bool direct = T <= kFlatDirectTrees;
  int cnt_others = 0;
  if (direct && j == 0) {
    float xo[kFlatDirectTrees][RPL];
#pragma unroll
    for (int t = 0; t < kFlatDirectTrees; ++t)
#pragma unroll
      for (int k = 0; k < RPL; ++k) {
        const int i = k * LP + lane;
        xo[t][k] = (t < T && t != sp.tree && i < N) ? pop[(((size_t)p * T + t) * N + i) * 4] : 0.0f;
      }
#pragma unroll
    for (int t = 0; t < kFlatDirectTrees; ++t)
#pragma unroll
      for (int k = 0; k < RPL; ++k) cnt_others += __popcll(seg_ballot(xo[t][k] != 0.0f));
  }
  auto operand = [&](int jj, int i, uint32_t& w, ULeaf& lf, int& len, int& flen, bool& leaf) {
    if (jj < i) {
      w = S.w[jj];
      const uint32_t ln = S.len[jj];
      len = (int)(ln & 0xffffu);
      flen = (int)(ln >> 16);
      lf.isc = u_isc(w);
      lf.v = S.cv[jj];
      lf.slot = u_slot(w);
      leaf = u_leaf(w);
    } else {
      w = u_pack(K_CONST, 0, 0, 1, 1, 0);
      lf.isc = true;
      lf.v = S.val[jj];
      lf.slot = 0;
      len = flen = 1;
      leaf = true;
    }
  };
  // ---- pass 1, round 0: leaves and empty rows resolve at once; operator rows note their operands
  int fnr[RPL], ja[RPL], jb[RPL];
  bool done[RPL];
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    const int i = k * LP + lane;
    fnr[k] = -1;
    ja[k] = jb[k] = -1;
    done[k] = true;
    if (i >= N) continue;
    uint32_t kind = K_CONST, slot = 0, isc = 1;
    float cv = 0.0f;
    if (row[k].x == 1.0f) {  // coefficient (gp.py:372 select)
      cv = row[k].w;
    } else {
      int32_t f = f2i_sat(row[k].x);
      f = f < 0 ? 0 : (f > n_funcs - 1 ? n_funcs - 1 : f);
      const int fn = s_fn[f];
      if (fn == MTGP_FN_VAR) {
        int sl = f - var_start;
        if (sl > n_data - 1) sl = n_data - 1;
        slot = (uint32_t)(sl >= sp.gap_at ? sl + sp.gap : sl);  // MtgpProgramSpec.gap
        if (!((zmask >> sl) & 1ull)) { kind = K_VAR; isc = 0; }
      } else if (fn_arity(fn) > 0) {
        fnr[k] = fn;
        ja[k] = norm_index(row[k].y, N);
        if (fn_arity(fn) == 2) jb[k] = norm_index(row[k].z, N);
        done[k] = false;
      }  // else: empty node (gp.py:135) -> +0.0
    }
    if (done[k]) {
      S.w[i] = u_pack(kind, MTGP_FN_ZERO, slot, isc, 1, 0);
      S.len[i] = 1u | 1u << 16;
      S.cv[i] = cv;
    }
    S.flag[i] = done[k] ? 1u : 0u;
  }
  // ---- pass 1, later rounds: an operator row resolves once its operand rows (j < i) have
  for (;;) {
    __syncthreads();
    bool ready[RPL], pend = false;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const int i = k * LP + lane;
      ready[k] = !done[k] && (ja[k] >= i || S.flag[ja[k]] != 0u) && (jb[k] < 0 || jb[k] >= i || S.flag[jb[k]] != 0u);
      pend = pend || (!done[k] && !ready[k]);
    }
    bool any_ready = false;
#pragma unroll
    for (int k = 0; k < RPL; ++k) any_ready = any_ready || ready[k];
    if (!wave_any(any_ready)) break;  // (a DAG: some row is always ready while any is pending)
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      if (!ready[k]) continue;
      const int i = k * LP + lane;
      const int fn = fnr[k], ar = fn_arity(fn);
      uint32_t kind = ar == 1 ? K_UNARY : K_BINARY, isc = 1, afirst = 1, need = 0;
      int len = 1, flen = 1;
      float cv = 0.0f;
      uint32_t wa, wb = 0;
      ULeaf la, lb;
      lb.isc = true; lb.v = 0.0f; lb.slot = 0;
      int lena, flena, lenb = 1, flenb = 1;
      bool leafa, leafb = true;
      operand(ja[k], i, wa, la, lena, flena, leafa);
      if (ar == 2) operand(jb[k], i, wb, lb, lenb, flenb, leafb);
      if (la.isc && lb.isc) {  // constant subtree: folded with the kernel's fp32 primitives
        cv = apply_fn(fn, la.v, ar == 1 ? 0.0f : lb.v);
      } else {
        isc = 0;
        if (ar == 1) {
          if (leafa) { len = 2; flen = unary_fuses(fn) ? 1 : 2; }
          else { len = lena + 1; flen = flena + 1; need = u_need(wa); }
        } else if (leafa && leafb) {
          len = 2; flen = 1;
        } else if (leafb) {
          len = lena + 1; flen = flena + 1; need = u_need(wa);
        } else if (leafa) {
          len = lenb + 1; flen = flenb + 1; need = u_need(wb);
        } else {
          const uint32_t pa = u_need(wa), qb = u_need(wb);
          len = lena + lenb + 1;
          flen = flena + flenb + 1;
          if (pa >= qb) { afirst = 1; need = pa > qb + 1 ? pa : qb + 1; }
          else { afirst = 0; need = qb > pa + 1 ? qb : pa + 1; }
        }
      }
      S.w[i] = u_pack(kind, (uint32_t)fn, 0, isc, afirst, need > 31u ? 31u : need);
      S.len[i] = (uint32_t)(len > 65535 ? 65535 : len) | (uint32_t)(flen > 65535 ? 65535 : flen) << 16;
      S.cv[i] = cv;
    }
    __syncthreads();  // every read of this round's flags precedes the new ones
#pragma unroll
    for (int k = 0; k < RPL; ++k)
      if (ready[k]) {
        S.flag[k * LP + lane] = 1u;
        done[k] = true;
      }
    (void)pend;
  }
  const uint32_t wr = S.w[N - 1], lr = S.len[N - 1];
  int n;
  if ((int)u_need(wr) > MTGP_STACK_MAX) n = -MTGP_ERR_STACK;
  else if ((int)(lr & 0xffffu) > cap) n = -MTGP_ERR_PROG_TOO_LONG;
  else n = (int)(lr >> 16);
  // ---- pass 2: postorder positions top-down, one word per reached node, one level per round
  // (the walk's barriers stay in wave-uniform control flow: with two programs per wave, a program
  // that does not walk takes part with no row reached)
  bool shared = false;
  const bool walk = n > 0 && !u_leaf(wr);
  if (n > 0 && u_leaf(wr) && lane == 0) {  // the whole tree is one leaf
    ULeaf x;
    x.isc = u_isc(wr); x.v = S.cv[N - 1]; x.slot = u_slot(wr);
    out[0] = S.prog[0] = u_load(x, false);
  }
  {
    if (LP == kWave ? walk : wave_any(walk)) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < RPL; ++k) S.flag[k * LP + lane] = 0u;
      __syncthreads();
      if (walk && lane == 0) {
        S.flag[N - 1] = 1u;
        S.pos[N - 1] = 0;
      }
      bool emitted[RPL];
#pragma unroll
      for (int k = 0; k < RPL; ++k) emitted[k] = false;
      for (;;) {
        __syncthreads();
        bool go[RPL], any = false;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
          const int i = k * LP + lane;
          go[k] = i < N && !emitted[k] && S.flag[i] != 0u;
          any = any || go[k];
        }
        if (!wave_any(any)) break;
        __syncthreads();  // every row's go decision precedes this round's visits
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
          if (!go[k]) continue;
          emitted[k] = true;
          const int i = k * LP + lane;
          const uint32_t w = S.w[i];
          const int pp = S.pos[i], pos = pp & 0xffff;
          const bool push = (pp >> 16) != 0;
          const int fn = (int)u_fn(w);
          uint32_t wa, wb;
          ULeaf la, lb;
          int lena, flena, lenb = 1, flenb = 1;
          bool leafa, leafb = true;
          const int ca = ja[k];
          operand(ca, i, wa, la, lena, flena, leafa);
          const int cb = u_kind(w) == K_BINARY ? jb[k] : 0;
          if (u_kind(w) == K_BINARY) operand(cb, i, wb, lb, lenb, flenb, leafb);
          auto visit = [&](int c, int cpos, bool cpush) {
            S.pos[c] = cpos | (cpush ? 1 << 16 : 0);
            shared = shared || atomicAdd(&S.flag[c], 1u) != 0u;  // a sub-DAG reached twice
          };
          MtgpInstr x;
          auto emit = [&](int at, const MtgpInstr& v) {
            out[at] = v;
            S.prog[at] = v;
          };
          if (u_kind(w) == K_UNARY) {
            const MtgpInstr un = u_instr(mtgp::unary_op(fn), 0, 0.0f);
            if (leafa) {
              MtgpInstr w2[2];
              const int nw = u_unary_leaf(fn, la, push, w2);
              emit(pos, w2[0]);  // (nw is 1 or 2; no dynamic index into w2, which would put it in scratch)
              if (nw > 1) emit(pos + 1, w2[1]);
            } else { visit(ca, pos, push); emit(pos + flena, un); }
          } else if (leafa && leafb) {
            fuse_pair(u_load(la, push), u_op_leaf(fn, 0, lb), &x);
            emit(pos, x);
          } else if (leafb) {
            visit(ca, pos, push);
            emit(pos + flena, u_op_leaf(fn, 0, lb));
          } else if (leafa) {
            visit(cb, pos, push);
            emit(pos + flenb, u_op_leaf(fn, 1, la));
          } else {
            const bool af = u_afirst(w) != 0;
            const int f1 = af ? flena : flenb, f2 = af ? flenb : flena;
            visit(af ? ca : cb, pos, push);
            visit(af ? cb : ca, pos + f1, true);
            emit(pos + f1 + f2, u_op_stack(fn, af ? 1 : 0));
          }
        }
      }
    }
  }
  shared = seg_ballot(shared) != 0ull;
  __syncthreads();  // every lane's program words (LDS copy) precede the END and the JIT sizing
  if (lane == 0) {
    if (shared) {  // arbitrary arrays only: the serial walk duplicates the shared subtree
      len_out[pj] = 0;
      status_out[pj] = kFlatSerial;
    } else {
      MtgpInstr e;
      e.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
      e.imm = 0.0f;
      out[n > 0 ? n : 0] = e;
      S.prog[n > 0 ? n : 0] = e;
      len_out[pj] = n > 0 ? n : 0;
      status_out[pj] = n > 0 ? 0 : -n;
    }
  }
  if (!shared && (jit_words_out || jit_cost_out)) {  // (shared: wave-uniform)
    constexpr int KI = (2 * NMAX + 8 + LP - 1) / LP;
    if (jit_mode == kJitModeRegs) {
      flat_jit_size_wave<KI, LP>(S.prog, n, optab, jit_words_out, jit_cost_out, pj, lane);
    } else if constexpr (LP == kWave) {  // (two programs per wave: register mode only, mtgp_flatten_ex)
      flat_jit_size_wave_lds<KI>(S.prog, n, optab, jit_words_out, jit_cost_out, pj, lane, s_fpos);
    }
  }
  // node count (gp.py:424 parsimony).  Few trees (T <= kFlatDirectTrees): the individual's first
  // program counts them all and stores the sum (no zeroing pass before the launch); many trees
  // (C5: 64): tree t is counted by program t % n_prog and summed with atomics into the zeroed
  // nodes_out, so no single wave walks the whole individual.
  if (direct && j != 0) return;
  int c = direct ? cnt + cnt_others : 0;
  for (int t = j; !direct && t < T; t += n_prog) {
    if (t == sp.tree) { c += cnt; continue; }
    const float4* tt = reinterpret_cast<const float4*>(pop + ((size_t)p * T + t) * N * 4);
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const int i = k * LP + lane;
      c += __popcll(seg_ballot(i < N && tt[i < N ? i : 0].x != 0.0f));
    }
  }
  if (lane == 0) {
    if (direct) nodes_out[p] = c;
    else if (c != 0) atomicAdd(&nodes_out[p], c);
  }
}

// --------------------------------------------------------------------------------------
// Schedule: counting sort of per-individual interpreter cost, then a slot permutation.
struct SchedW {
  int32_t w[MTGP_MAX_PROGRAMS];
};

__device__ __forceinline__ int sched_cost(const int32_t* plen, int p, int n_prog, const SchedW& W) {
  int c = 0;
  for (int j = 0; j < n_prog; ++j) c += W.w[j] * plen[(size_t)p * n_prog + j];
  return c < 0 ? 0 : (c >= MTGP_SCHED_BINS ? MTGP_SCHED_BINS - 1 : c);
}

// the same with the four programs of an individual read as one 16-byte load (n_prog == 4, plen
// 16-byte aligned; integer sums: any order gives the same cost)
__device__ __forceinline__ int sched_cost4(const int32_t* plen, int p, const SchedW& W) {
  const int4 v = reinterpret_cast<const int4*>(plen)[p];
  const int c = W.w[0] * v.x + W.w[1] * v.y + W.w[2] * v.z + W.w[3] * v.w;
  return c < 0 ? 0 : (c >= MTGP_SCHED_BINS ? MTGP_SCHED_BINS - 1 : c);
}

__global__ void __launch_bounds__(256) k_sched_hist(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                    int32_t* __restrict__ hist) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) atomicAdd(&hist[sched_cost(plen, p, n_prog, W)], 1);
}

// Exclusive scan of one value per thread over a 1024-thread block: a wave scan by shuffles and one
// barrier for the 16 wave totals (wsum: 16 ints of LDS).  Replaces a Hillis-Steele scan through
// LDS (twenty barriers).
__device__ __forceinline__ int block_excl_scan_1024(int v, int32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int inc = v;
  for (int d = 1; d < kWave; d <<= 1) {
    const int y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  int base = inc - v;
  for (int q = 0; q < 16; ++q)
    if (q < w) base += wsum[q];
  return base;
}

// exclusive scan of the histogram (one block, MTGP_SCHED_BINS / 1024 bins per thread)
__global__ void __launch_bounds__(1024) k_sched_scan(const int32_t* __restrict__ hist, int32_t* __restrict__ offs) {
  constexpr int kPer = MTGP_SCHED_BINS / 1024;
  __shared__ int32_t wsum[16];
  const int t = threadIdx.x;
  int loc[kPer], sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) { loc[i] = sum; sum += hist[t * kPer + i]; }
  const int base = block_excl_scan_1024(sum, wsum);
#pragma unroll
  for (int i = 0; i < kPer; ++i) offs[t * kPer + i] = base + loc[i];
}

// ascending rank s -> slot: G >= 2 interleaves (most expensive, cheapest, 2nd, 2nd cheapest, ...)
// so every wave holds a balanced mix; G == 1 runs the most expensive first.
__device__ __forceinline__ int sched_slot(int s, int P, int G) {
  if (G == 1) return P - 1 - s;
  const int h = P / 2;
  if (s < h) return 2 * s + 1;
  if (s >= P - h) return 2 * (P - 1 - s);
  return P - 1;  // middle element of an odd P
}

__global__ void __launch_bounds__(256) k_sched_scatter(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                       int G, int32_t* __restrict__ offs, int32_t* __restrict__ order) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  order[sched_slot(atomicAdd(&offs[sched_cost(plen, p, n_prog, W)], 1), P, G)] = p;
}

// The whole schedule in ONE block (P * n_prog <= kSchedFusedMax): histogram, exclusive scan and scatter in
// LDS (no memset, no global atomics, one launch instead of three + a fill).  Same slot formula as
// k_sched_scatter; ties are ordered arbitrarily as there.  KP > 0 (P <= 1024 * KP): every thread's
// costs are computed once, their loads issued together, and held in registers for both atomic
// passes (9.6 -> 7.7 us at P = 8192, scripts/overhead_mb.hip); KP = 0 recomputes them in strided loops.
constexpr long kSchedFusedMax = 1 << 16;  // program entries (P * n_prog): C3 32768 -> fused, C5 262144 -> 3 kernels
constexpr int kSchedRegP = 8;              // costs per thread held in registers (P <= 8192)
template <int KP>
__global__ void __launch_bounds__(1024) k_sched_fused(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                      int G, int32_t* __restrict__ order, int vec4) {
  __shared__ int32_t hist[MTGP_SCHED_BINS];
  __shared__ int32_t wsum[16];
  constexpr int kPer = MTGP_SCHED_BINS / 1024;
  constexpr int KR = KP > 0 ? KP : 1;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[i * 1024 + t] = 0;
  int c[KR];
  if constexpr (KP > 0) {
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int p = k * 1024 + t;
      c[k] = p < P ? (vec4 ? sched_cost4(plen, p, W) : sched_cost(plen, p, n_prog, W)) : -1;
    }
  }
  __syncthreads();
  if constexpr (KP > 0) {
#pragma unroll
    for (int k = 0; k < KP; ++k)
      if (c[k] >= 0) atomicAdd(&hist[c[k]], 1);
  } else {
    for (int p = t; p < P; p += 1024) atomicAdd(&hist[sched_cost(plen, p, n_prog, W)], 1);
  }
  __syncthreads();
  int loc[kPer], sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) { loc[i] = sum; sum += hist[t * kPer + i]; }
  const int base = block_excl_scan_1024(sum, wsum);
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[t * kPer + i] = base + loc[i];  // (each thread rewrites its own bins)
  __syncthreads();
  if constexpr (KP > 0) {
#pragma unroll
    for (int k = 0; k < KP; ++k)
      if (c[k] >= 0) order[sched_slot(atomicAdd(&hist[c[k]], 1), P, G)] = k * 1024 + t;
  } else {
    for (int p = t; p < P; p += 1024) order[sched_slot(atomicAdd(&hist[sched_cost(plen, p, n_prog, W)], 1), P, G)] = p;
  }
}

#endif  // MTGP_TU_MAIN

#if MTGP_TU_MAIN
// --------------------------------------------------------------------------------------
// Program JIT build (mtgp_jit.h): one unit of code per (wave, role).  Pass 1 sizes every
// unit, one block scans the sizes into byte offsets, pass 2 writes the code (vector stores)
// into executable device memory.
constexpr uint32_t kJitAlign = 64u;

struct JitUnitArgs {
  const MtgpInstr* prog;
  int n_prog, L, P, G, Rp, n_units;
  const int32_t* order;
  int mode;  // mtgp_jit.h kJitModeRegs / kJitModeLds
  uint32_t next, cond, store;  // role / LDS store chains (MtgpJitChain, mtgp_jit.h jit_unit_end)
  int pipe;                    // LDS-data units software-pipelined (mtgp_jit.h jit_lds_region)
  uint32_t put;                // MtgpJitChain.put / put_slot (ABI v18)
  int put_slot;
};

__device__ __forceinline__ int jit_unit_words(const JitUnitArgs& U, int u, uint32_t* out, uint32_t base) {
  const int wave = u / U.n_prog, j = u - wave * U.n_prog;
  return mtgp::jit_unit(U.prog, U.n_prog, U.L, U.P, U.order, U.G, U.Rp, wave, j, out, base, mtgp::kJitModeRegs,
                        U.next, U.cond, U.store, true, U.put, U.put_slot);
}

// byte span of unit u in the layout: a unit that falls through into the next one (a chain member)
// spans exactly its code, the next unit following directly; every other unit is padded so that
// it ENDS on a 64-byte line (pre = bytes of the chain members packed in front of it), so every
// unit that is called starts on one
__device__ __forceinline__ uint32_t jit_unit_span(const JitUnitArgs& U, int u, int words, uint32_t pre = 0u) {
  const int j = u % U.n_prog;
  if (mtgp::jit_unit_packed(U.next, j, U.store, U.n_prog)) return (uint32_t)words * 4u;
  return ((pre + (uint32_t)words * 4u + kJitAlign - 1u) & ~(kJitAlign - 1u)) - pre;
}

__global__ void __launch_bounds__(256) k_jit_count(JitUnitArgs U, uint32_t* __restrict__ offs,
                                                   int32_t* __restrict__ info) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= U.n_units) return;
  const int n = jit_unit_words(U, i, nullptr, 0u);
  // units start on 64-byte instruction-cache lines (measured: unaligned call targets made some
  // code shapes 2x slower, scripts/dispatch_cost.py k = 4)
  offs[i] = n > 0 ? jit_unit_span(U, i, n) : 0u;
  if (n < 0) atomicMin(&info[0], n);
}

// exclusive scan of offs[0..total) in place, offs[total] = total bytes, info[1] = total bytes
// (saturated to INT32_MAX for the host check)
// per-program JIT cost for the schedule: executed code words / 4 (>= 1; untranslatable -> plen)
__global__ void __launch_bounds__(256) k_jit_cost(const MtgpInstr* __restrict__ prog, int total, int L,
                                                  const int32_t* __restrict__ plen, int32_t* __restrict__ cost) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = mtgp::jit_cost(prog + (size_t)i * L, L);
  cost[i] = c > 0 ? (c + 3) / 4 : plen[i];
}

__global__ void __launch_bounds__(1024) k_jit_scan(uint32_t* __restrict__ offs, int total, int32_t* __restrict__ info) {
  __shared__ uint64_t part[1024];
  const int t = threadIdx.x;
  const int per = (total + 1023) / 1024;
  const int b = t * per, e = b + per < total ? b + per : total;
  uint64_t sum = 0;
  for (int i = b; i < e; ++i) sum += offs[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = part[t] - sum + mtgp::kJitTemplateBytes;  // the shared subroutines come first
  for (int i = b; i < e; ++i) {
    const uint64_t w = offs[i];
    offs[i] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
    run += w;
  }
  if (t == 1023) {
    const uint64_t tot = part[1023] + mtgp::kJitTemplateBytes;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

__global__ void __launch_bounds__(256) k_jit_emit(JitUnitArgs U, const uint32_t* __restrict__ offs,
                                                  uint32_t* __restrict__ code, uint64_t code_bytes) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= U.n_units) return;
  const uint32_t b = offs[i], e = offs[i + 1];
  if (e <= b || (uint64_t)e > code_bytes) return;  // untranslatable unit or short buffer (checked on use)
  jit_unit_words(U, i, code + b / 4, b);
}

// Unit layout from the flatten's per-program code sizes (mtgp_flatten_ex jit_words): unit
// (wave, j) = its G groups' programs + the merge words of groups 1.. (mtgp_jit.h jit_merge_words) + s_setpc (mtgp_jit.h
// jit_unit), 64-byte aligned; a grid sizes the units, one block scans the sizes into byte
// offsets.  Replaces the k_jit_count translation pass + k_jit_scan.
__device__ __forceinline__ int jit_unit_words_from(const JitUnitArgs& U, const int32_t* __restrict__ jw, int u) {
  const int wave = u / U.n_prog, j = u - wave * U.n_prog;
  int n = mtgp::jit_unit_end_words(U.next, U.cond, j, U.store, U.n_prog);  // s_setpc_b64 or the chain epilogue
  for (int g = 0; g < U.G; ++g) {
    const int q = wave * U.G + g;
    if (q >= U.P) break;
    const int ind = U.order ? U.order[q] : q;
    const int w = jw[(size_t)ind * U.n_prog + j];
    if (w < 0) return w;
    n += w + mtgp::jit_merge_words(g);
  }
  return n;
}

// pass 1, one thread per unit: its size in bytes, or 0x80000000 | -error.  A chain member's span
// needs the words of the members packed in front of it: those of this block are read from LDS
// (every thread sizes its own unit first), only members in an earlier block are sized again
// (C5's store chains run over all 64 programs of a wave: up to 63 members x 8 groups of loads
// per thread before).
__global__ void __launch_bounds__(256) k_jit_sizes(JitUnitArgs U, const int32_t* __restrict__ jw,
                                                   uint32_t* __restrict__ offs) {
  __shared__ int s_words[256];
  const int u0 = blockIdx.x * blockDim.x;
  const int u = u0 + threadIdx.x;
  const int n = u < U.n_units ? jit_unit_words_from(U, jw, u) : 0;
  s_words[threadIdx.x] = n;
  __syncthreads();
  if (u >= U.n_units) return;
  uint32_t pre = 0u;  // the chain members packed in front of this unit
  int bad = 0;
  for (int v = u - 1; v >= 0 && v / U.n_prog == u / U.n_prog && mtgp::jit_unit_packed(U.next, v % U.n_prog, U.store, U.n_prog); --v) {
    const int m = v >= u0 ? s_words[v - u0] : jit_unit_words_from(U, jw, v);
    if (m < 0) bad = m;
    else pre += (uint32_t)m * 4u;
  }
  offs[u] = (n > 0 && bad == 0) ? jit_unit_span(U, u, n, pre) : (0x80000000u | (uint32_t)(-(n < 0 ? n : bad)));
}

// pass 2, one block: exclusive scan of the sizes in place (+ the shared templates in front),
// offs[units] = total, info = {min error or 0, total bytes}.  Each thread owns a contiguous
// run of units and loads it eight entries at a time (independent loads in flight).
__global__ void __launch_bounds__(1024) k_jit_scan_sizes(uint32_t* __restrict__ offs, int total,
                                                         int32_t* __restrict__ info) {
  __shared__ uint64_t part[1024];
  __shared__ int32_t err[1024];
  const int t = threadIdx.x;
  const int per = (total + 1023) / 1024;
  const int b = t * per, e = b + per < total ? b + per : total;
  uint64_t sum = 0;
  int bad = 0;
  for (int k0 = b; k0 < e; k0 += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (k0 + k < e) ? offs[k0 + k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool isbad = (v[k] & 0x80000000u) != 0u;
      const int code = -(int)(v[k] & 0x7fffffffu);
      bad = (isbad && code < bad) ? code : bad;
      sum += isbad ? 0u : v[k];
    }
  }
  part[t] = sum;
  err[t] = bad;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan (+ min of the error codes)
    const uint64_t v = t >= d ? part[t - d] : 0;
    const int32_t m = t >= d ? err[t - d] : 0;
    __syncthreads();
    part[t] += v;
    err[t] = m < err[t] ? m : err[t];
    __syncthreads();
  }
  uint64_t run = part[t] - sum + mtgp::kJitTemplateBytes;  // the shared subroutines come first
  for (int k0 = b; k0 < e; k0 += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (k0 + k < e) ? offs[k0 + k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k0 + k >= e) break;
      const uint64_t w = (v[k] & 0x80000000u) ? 0u : v[k];
      offs[k0 + k] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
      run += w;
    }
  }
  if (t == 1023) {
    const uint64_t tot = part[1023] + mtgp::kJitTemplateBytes;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[0] = err[1023];
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

// The same scan with every thread's PER sizes held in registers (one read, one write pass),
// wave scans by shuffles and one barrier for the 16 wave totals (units <= 1024 * PER).  The sizes
// are read and the offsets written coalesced (unit k * 1024 + t by thread t) and transposed
// through LDS to the thread-contiguous runs the scan needs: a thread reading its run straight
// from global memory touches a cache line per unit, which through the one CU this block runs on
// took 16.0 us at 16384 units against 5.6 us (scripts/overhead_mb.hip).  One pad word per 64
// keeps the run reads conflict-free on the 64 LDS banks.
__device__ __forceinline__ int scan_lds_ix(int i) { return i + (i >> 6); }
template <int PER>
__global__ void __launch_bounds__(1024) k_jit_scan_sizes_reg(uint32_t* __restrict__ offs, int total,
                                                             int32_t* __restrict__ info) {
  constexpr int kUnits = 1024 * PER;
  __shared__ uint32_t s_u[kUnits + kUnits / 64];
  __shared__ uint64_t wsum[16];
  __shared__ int32_t werr[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 1024 + t;
    v[k] = i < total ? offs[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) s_u[scan_lds_ix(k * 1024 + t)] = v[k];
  __syncthreads();
  const int b = t * PER;
#pragma unroll
  for (int k = 0; k < PER; ++k) v[k] = s_u[scan_lds_ix(b + k)];  // (units >= total read as 0)
  uint64_t sum = 0;
  int bad = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const bool isbad = (v[k] & 0x80000000u) != 0u;
    const int code = -(int)(v[k] & 0x7fffffffu);
    bad = (isbad && code < bad) ? code : bad;
    sum += isbad ? 0u : v[k];
  }
  uint64_t inc = sum;  // inclusive scan over the wave
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  int e = bad;
  for (int d = 1; d < kWave; d <<= 1) {
    const int o = __shfl_xor(e, d, kWave);
    e = o < e ? o : e;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  if (lane == 0) werr[w] = e;
  __syncthreads();
  uint64_t wbase = 0;
  int err = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) wbase += wsum[q];
    err = werr[q] < err ? werr[q] : err;
  }
  uint64_t run = wbase + inc - sum + mtgp::kJitTemplateBytes;  // the shared subroutines come first
#pragma unroll
  for (int k = 0; k < PER; ++k) {  // (the sizes re-read from LDS: v is not held over the scan)
    const uint32_t x = s_u[scan_lds_ix(b + k)];
    s_u[scan_lds_ix(b + k)] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
    run += (x & 0x80000000u) ? 0u : x;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 1024 + t;
    if (i < total) offs[i] = s_u[scan_lds_ix(i)];
  }
  if (t == 1023) {
    const uint64_t tot = wbase + inc + mtgp::kJitTemplateBytes;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[0] = err;
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

// Emit with one thread per (unit, group): group g's code starts after groups 0..g-1 (sizes from
// jit_words), so the G programs of a unit are translated in parallel.
// (4 waves per SIMD: a C5 build is 4,096 waves, one round at 4 per SIMD instead of two at 3)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4)))
k_jit_emit_groups(JitUnitArgs U, const int32_t* __restrict__ jw,
                                                        const uint32_t* __restrict__ offs, uint32_t* __restrict__ code,
                                                        uint64_t code_bytes) {
  if (blockIdx.x == 0 && code_bytes >= mtgp::kJitTemplateBytes) {  // the shared subroutines
    for (int k = threadIdx.x; k < MTGP_JIT_SUB_WORDS; k += blockDim.x) code[k] = mtgp_jit_sub_blob[k];
  }
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)U.n_units * U.G) return;
  const int u = (int)(i / U.G), g = (int)(i - (long)u * U.G);
  const int wave = u / U.n_prog, j = u - wave * U.n_prog;
  const int q = wave * U.G + g;
  if (q >= U.P) return;
  const uint32_t b = offs[u], e = offs[u + 1];
  if (e <= b || (uint64_t)e > code_bytes) return;  // untranslatable unit or short buffer (checked on use)
  uint32_t start = 0;  // words before group g inside the unit
  for (int h = 0; h < g; ++h) {
    const int ind = U.order ? U.order[wave * U.G + h] : wave * U.G + h;
    start += (uint32_t)jw[(size_t)ind * U.n_prog + j] + (uint32_t)mtgp::jit_merge_words(h);
  }
  const bool last = (g == U.G - 1) || (q + 1 >= U.P);
  if (U.mode == mtgp::kJitModeLds && U.pipe && g > 0) {  // pipelined LDS units: group g's region starts after its preloads
    const int ind = U.order ? U.order[q] : q;
    const int pw = mtgp::jit_preload_words(U.prog + ((size_t)ind * U.n_prog + j) * U.L, U.L);
    if (pw < 0) return;
    start += (uint32_t)pw;
  }
  const uint32_t at = b + start * 4u;
  mtgp::jit_unit_group(U.prog, U.n_prog, U.L, U.order, U.Rp, wave * U.G, g, j, last, code + at / 4, at, U.mode,
                       U.next, U.cond, U.store, U.pipe != 0, U.put, U.put_slot);
}

// Register-data emit with one WAVE per (unit, group): as in k_flatten_wave's sizing, an
// instruction's code depends only on its opcode, the operand-stack depth before it and its byte
// address (the PC-relative sin/cos calls), so the lanes translate instructions l, l + 64, ... in
// isolation (jit_program with that depth and base) at offsets from a prefix sum of the JitOpTable
// word counts -- the same words jit_unit_group writes serially (tests/test_gpu_build.py).  Lane 0
// writes the group's frame (the v25 keep, the lane-group select, the unit end).
template <int KI>
__global__ void __launch_bounds__(256) k_jit_emit_waves(JitUnitArgs U, const int32_t* __restrict__ jw,
                                                        const uint32_t* __restrict__ offs, uint32_t* __restrict__ code,
                                                        uint64_t code_bytes, JitOpTable optab) {
  if (blockIdx.x == 0 && code_bytes >= mtgp::kJitTemplateBytes) {  // the shared subroutines
    for (int k = threadIdx.x; k < MTGP_JIT_SUB_WORDS; k += blockDim.x) code[k] = mtgp_jit_sub_blob[k];
  }
  const int lane = threadIdx.x & (kWave - 1);
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) / kWave;  // (wave-uniform)
  if (i >= (long)U.n_units * U.G) return;
  const int u = (int)(i / U.G), g = (int)(i - (long)u * U.G);
  const int wave = u / U.n_prog, j = u - wave * U.n_prog;
  const int remap = mtgp::jit_put_remap(U.next, U.put, j);  // (put chains: slot put_slot read from v26 + pos)
  const int q = wave * U.G + g;
  if (q >= U.P) return;
  const uint32_t b = offs[u], e = offs[u + 1];
  if (e <= b || (uint64_t)e > code_bytes) return;  // untranslatable unit or short buffer (checked on use)
  uint32_t start = 0;  // words before group g inside the unit
  for (int h = 0; h < g; ++h) {
    const int ind = U.order ? U.order[wave * U.G + h] : wave * U.G + h;
    start += (uint32_t)jw[(size_t)ind * U.n_prog + j] + (uint32_t)mtgp::jit_merge_words(h);
  }
  const bool last = (g == U.G - 1) || (q + 1 >= U.P);
  const uint32_t at = b + start * 4u;  // byte address of the group's first word
  uint32_t* out = code + at / 4;
  const int ind = U.order ? U.order[q] : q;
  const MtgpInstr* prog = U.prog + ((size_t)ind * U.n_prog + j) * U.L;
  const int pre = mtgp::jit_merge_keep(g) ? 1 : 0;  // v_mov v25, v8
  MtgpInstr end;
  end.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
  end.imm = 0.0f;
  int woff = 0, sp = 0;  // words and stack depth before this chunk
  bool ended = false;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    if (ended) break;  // (wave-uniform)
    const int ii = k * kWave + lane;
    const MtgpInstr x = ii < U.L ? prog[ii] : end;
    const uint32_t c = x.op >> MTGP_OP_SHIFT;
    const uint64_t ends = __ballot(c == (uint32_t)MTGP_OP_END);
    const int first_end = ends ? __ffsll((unsigned long long)ends) - 1 : kWave;
    const bool in = lane < first_end;
    const uint32_t f = (in && c < 64u) ? optab.flags[c] : 0u;
    const int w = (in && c < 64u) ? optab.words[c] : 0;
    const int d = (f & kOpPush) ? 1 : ((f & kOpPop) ? -1 : 0);
    int wi = w, di = d;  // inclusive prefix sums over the chunk
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int vw = __shfl_up(wi, off), vd = __shfl_up(di, off);
      if (lane >= off) { wi += vw; di += vd; }
    }
    if (in) {
      const MtgpInstr t[2] = {x, end};
      mtgp::JitOut o{out + pre + woff + (wi - w), 0};
      o.base = at + (uint32_t)(pre + woff + (wi - w)) * 4u;
      (void)mtgp::jit_program(o, t, 2, false, mtgp::kJitModeRegs, 0, mtgp::kJitPre, 0, nullptr, sp + di - d,
                              nullptr, 0, remap < 0 ? -1 : U.put_slot, remap);
    }
    woff += __shfl(wi, kWave - 1);
    sp += __shfl(di, kWave - 1);
    ended = ends != 0ull;
  }
  if (lane == 0) {
    mtgp::JitOut o{out, 0};
    o.base = at;
    if (mtgp::jit_merge_keep(g)) o.movv(mtgp::kJitKeep, mtgp::kJitAcc);
    o.n = pre + woff;
    if (g > 0) mtgp::jit_merge_tail(o, g, U.Rp, last);
    if (last) mtgp::jit_unit_end(o, U.next, U.cond, j, U.store, U.n_prog);
  }
}

// The same emit with 64 / LP (unit, group) pairs per wave, LP lanes each (chunks of LP
// instructions, prefix sums within the LP lanes; "halves" below for any LP).  The register-mode
// programs are short, so a whole wave per pair left most of it idle and C3's 32,768 waves ran in
// four rounds at full occupancy: 40.3 us one pair per wave, 28.2 two, 20.0 four (LP = 16, the
// default; profiles/r06/v21_*, v25_*).  The same words as k_jit_emit_waves (tests/test_gpu_build.py).
template <int KI, int LP = kWave / 2>  // KI chunks of LP instructions; LP lanes per pair
__global__ void __launch_bounds__(256) k_jit_emit_halves(JitUnitArgs U, const int32_t* __restrict__ jw,
                                                         const uint32_t* __restrict__ offs, uint32_t* __restrict__ code,
                                                         uint64_t code_bytes, JitOpTable optab) {
  constexpr int kHalf = LP;  // (a "half": the LP lanes of one pair)
  constexpr int PPW = kWave / LP;
  if (blockIdx.x == 0 && code_bytes >= mtgp::kJitTemplateBytes) {  // the shared subroutines
    for (int k = threadIdx.x; k < MTGP_JIT_SUB_WORDS; k += blockDim.x) code[k] = mtgp_jit_sub_blob[k];
  }
  const int lane = threadIdx.x & (kWave - 1), hl = lane & (kHalf - 1), half = lane / kHalf;
  const long i = (((long)blockIdx.x * blockDim.x + threadIdx.x) / kWave) * PPW + half;  // (half-uniform)
  bool live = i < (long)U.n_units * U.G;
  int u = 0, g = 0, wave = 0, j = 0, q = 0;
  if (live) {
    u = (int)(i / U.G);
    g = (int)(i - (long)u * U.G);
    wave = u / U.n_prog;
    j = u - wave * U.n_prog;
    q = wave * U.G + g;
    live = q < U.P;
  }
  uint32_t b = 0u;
  if (live) {
    b = offs[u];
    const uint32_t e = offs[u + 1];
    live = !(e <= b || (uint64_t)e > code_bytes);  // untranslatable unit or short buffer (checked on use)
  }
  const int remap = live ? mtgp::jit_put_remap(U.next, U.put, j) : -1;
  uint32_t start = 0;  // words before group g inside the unit
  for (int h = 0; live && h < g; ++h) {
    const int ind = U.order ? U.order[wave * U.G + h] : wave * U.G + h;
    start += (uint32_t)jw[(size_t)ind * U.n_prog + j] + (uint32_t)mtgp::jit_merge_words(h);
  }
  const bool last = (g == U.G - 1) || (q + 1 >= U.P);
  const uint32_t at = b + start * 4u;  // byte address of the group's first word
  uint32_t* out = code + at / 4;
  const int ind = live ? (U.order ? U.order[q] : q) : 0;
  const MtgpInstr* prog = U.prog + ((size_t)ind * U.n_prog + j) * U.L;
  const int pre = mtgp::jit_merge_keep(g) ? 1 : 0;  // v_mov v25, v8
  MtgpInstr end;
  end.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
  end.imm = 0.0f;
  int woff = 0, sp = 0;  // words and stack depth before this chunk
  bool ended = !live;    // (half-uniform)
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    if (__ballot(!ended) == 0ull) break;  // (wave-uniform: both halves done)
    const int ii = k * kHalf + hl;
    const MtgpInstr x = (!ended && ii < U.L) ? prog[ii] : end;
    const uint32_t c = x.op >> MTGP_OP_SHIFT;
    const uint32_t ends = (uint32_t)((__ballot(c == (uint32_t)MTGP_OP_END) >> (half * kHalf)) & ((1ull << kHalf) - 1ull));
    const int first_end = ends ? __ffs(ends) - 1 : kHalf;
    const bool in = !ended && hl < first_end;
    const uint32_t f = (in && c < 64u) ? optab.flags[c] : 0u;
    const int w = (in && c < 64u) ? optab.words[c] : 0;
    const int d = (f & kOpPush) ? 1 : ((f & kOpPop) ? -1 : 0);
    int wi = w, di = d;  // inclusive prefix sums over the chunk (within the half)
#pragma unroll
    for (int off = 1; off < kHalf; off <<= 1) {
      const int vw = __shfl_up(wi, off, kHalf), vd = __shfl_up(di, off, kHalf);
      if (hl >= off) { wi += vw; di += vd; }
    }
    if (in) {
      const MtgpInstr t[2] = {x, end};
      mtgp::JitOut o{out + pre + woff + (wi - w), 0};
      o.base = at + (uint32_t)(pre + woff + (wi - w)) * 4u;
      (void)mtgp::jit_program(o, t, 2, false, mtgp::kJitModeRegs, 0, mtgp::kJitPre, 0, nullptr, sp + di - d,
                              nullptr, 0, remap < 0 ? -1 : U.put_slot, remap);
    }
    woff += __shfl(wi, kHalf - 1, kHalf);
    sp += __shfl(di, kHalf - 1, kHalf);
    ended = ended || ends != 0u;
  }
  if (live && hl == 0) {
    mtgp::JitOut o{out, 0};
    o.base = at;
    if (mtgp::jit_merge_keep(g)) o.movv(mtgp::kJitKeep, mtgp::kJitAcc);
    o.n = pre + woff;
    if (g > 0) mtgp::jit_merge_tail(o, g, U.Rp, last);
    if (last) mtgp::jit_unit_end(o, U.next, U.cond, j, U.store, U.n_prog);
  }
}

// LDS-data emit with one WAVE per (unit, group) (the wide-state SR kernel's pipelined units,
// mtgp_jit.h jit_lds_region): the lanes first find the preload tables of the group's program and
// of the next group's (the first kJitPreSlots distinct data slots in order of first use: per slot
// its first operand position by an LDS atomicMin, its rank = the slots first used before it, as
// flat_jit_size_wave_lds sizes them), write the preloads (a lane per slot), then translate the body
// instructions l, l + 64, ... in isolation (jit_program part 3 with the table, the stack depth and
// byte address from prefix sums: table words + 3 per operand loaded at its use).  Lane 0 writes
// the frame (the v25 keep, the wait for the group's own preloads, the select, the unit end).
// The same words as k_jit_emit_groups' serial jit_unit_group (tests/test_gpu_build.py).
constexpr int kEmitLdsWaves = 4;  // waves per block
template <int KI>
__global__ void __launch_bounds__(kEmitLdsWaves * kWave) k_jit_emit_waves_lds(JitUnitArgs U, const int32_t* __restrict__ jw,
                                                                             const uint32_t* __restrict__ offs,
                                                                             uint32_t* __restrict__ code,
                                                                             uint64_t code_bytes, JitOpTable optab) {
  static_assert(MTGP_MAX_DATA <= kWave, "one lane per data slot");
  __shared__ int s_first[kEmitLdsWaves][MTGP_MAX_DATA];
  if (blockIdx.x == 0 && code_bytes >= mtgp::kJitTemplateBytes) {  // the shared subroutines
    for (int k = threadIdx.x; k < MTGP_JIT_SUB_WORDS; k += blockDim.x) code[k] = mtgp_jit_sub_blob[k];
  }
  const int lane = threadIdx.x & (kWave - 1), wib = threadIdx.x >> 6;
  int* fpos = s_first[wib];
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) / kWave;  // (wave-uniform)
  if (i >= (long)U.n_units * U.G) return;
  const int u = (int)(i / U.G), g = (int)(i - (long)u * U.G);
  const int wave = u / U.n_prog, j = u - wave * U.n_prog;
  const int q = wave * U.G + g;
  if (q >= U.P) return;
  const uint32_t b = offs[u], e = offs[u + 1];
  if (e <= b || (uint64_t)e > code_bytes) return;  // untranslatable unit or short buffer (checked on use)
  const bool last = (g == U.G - 1) || (q + 1 >= U.P);
  MtgpInstr end;
  end.op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
  end.imm = 0.0f;
  // the preload table of program p: pre_slot(r) = the slot of rank r (r < npre), via the lanes
  // (lane s: slot s's rank, or -1 when it is not preloaded)
  auto table = [&](const MtgpInstr* p, int& npre) -> int {
    fpos[lane] = 0x7fffffff;  // (lane < MTGP_MAX_DATA == kWave)
    __builtin_amdgcn_wave_barrier();
    bool ended = false;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      if (ended) break;  // (wave-uniform)
      const int ii = k * kWave + lane;
      const MtgpInstr x = ii < U.L ? p[ii] : end;
      const uint32_t c = x.op >> MTGP_OP_SHIFT;
      const uint64_t ends = __ballot(c == (uint32_t)MTGP_OP_END);
      const int first_end = ends ? __ffsll((unsigned long long)ends) - 1 : kWave;
      if (lane < first_end) {
        const uint32_t f = c < 64u ? optab.flags[c] : 0u;
        uint32_t ib;
        __builtin_memcpy(&ib, &x.imm, 4);
        const int sa = (f & kOpIbSlot) ? (int)(ib / MTGP_SLOT_BYTES) : -1;
        const int sb = (f & kOpAxSlot) ? (int)((x.op & 0xffffffu) / MTGP_SLOT_BYTES) : -1;
        if (sa >= 0 && sa < MTGP_MAX_DATA) atomicMin(&fpos[sa], 2 * ii);
        if (sb >= 0 && sb < MTGP_MAX_DATA) atomicMin(&fpos[sb], 2 * ii + 1);
      }
      ended = ends != 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    const int mine = fpos[lane];
    int before = 0;
#pragma unroll 8
    for (int t = 0; t < MTGP_MAX_DATA; ++t) before += fpos[t] < mine ? 1 : 0;
    const bool pre = mine != 0x7fffffff && before < mtgp::kJitPreSlots;
    npre = __popcll(__ballot(pre));
    __builtin_amdgcn_wave_barrier();
    return pre ? before : -1;
  };
  const int ind = U.order ? U.order[q] : q;
  const MtgpInstr* prog = U.prog + ((size_t)ind * U.n_prog + j) * U.L;
  const MtgpInstr* nprog = nullptr;
  if (!last) nprog = U.prog + ((size_t)(U.order ? U.order[q + 1] : q + 1) * U.n_prog + j) * U.L;
  int npre = 0, np1 = 0;
  const int rank = table(prog, npre);
  // the body's table in every lane: pre_tab[r] = the slot of rank r
  int pre_tab[mtgp::kJitPreSlots];
#pragma unroll
  for (int r = 0; r < mtgp::kJitPreSlots; ++r) {
    const uint64_t m = __ballot(rank == r);
    pre_tab[r] = m ? __ffsll((unsigned long long)m) - 1 : 0;
  }
  const int nrank = nprog ? table(nprog, np1) : -1;
  int nxt_tab[mtgp::kJitPreSlots];  // the next program's table (its preload pairs)
#pragma unroll
  for (int r = 0; r < mtgp::kJitPreSlots; ++r) {
    const uint64_t m = __ballot(nrank == r);
    nxt_tab[r] = m ? __ffsll((unsigned long long)m) - 1 : 0;
  }
  // preload instruction of rank r (even): a pair with rank r + 1, or the odd last one alone
  auto preload = [&](uint32_t* at, int r, int n, const int* tab, int base_reg) {
    if (r & 1) return;
    at[r] = r + 1 < n ? (mtgp::kDsRead2St64B32 | (uint32_t)tab[r + 1] << 8 | (uint32_t)tab[r])
                      : (mtgp::kDsReadB32 | (uint32_t)(tab[r] * (int)MTGP_SLOT_BYTES));
    at[r + 1] = (uint32_t)(base_reg + r) << 24 | (uint32_t)mtgp::kJitLdsAddr;
  };
  // group g's region (jit_lds_region): [P_0 (g = 0)] [P_(g+1)] [keep (g = 1)] [wait] [body] [select] [end]
  uint32_t start = 0;  // words before group g inside the unit
  for (int h = 0; h < g; ++h) {
    const int ih = U.order ? U.order[wave * U.G + h] : wave * U.G + h;
    start += (uint32_t)jw[(size_t)ih * U.n_prog + j] + (uint32_t)mtgp::jit_merge_words(h);
  }
  if (g > 0) start += 2u * (uint32_t)mtgp::jit_preload_instrs(npre);  // its preloads sit in group g-1's region
  const uint32_t at = b + start * 4u;
  uint32_t* out = code + at / 4;
  const int set = mtgp::jit_pre_set(g), nset = mtgp::jit_pre_set(g + 1);
  int w0 = 0;  // words written before the body
  if (g == 0) {
    if (lane < npre) preload(out, lane, npre, pre_tab, set);
    w0 += 2 * mtgp::jit_preload_instrs(npre);
  }
  if (lane < np1) preload(out + w0, lane, np1, nxt_tab, nset);
  w0 += 2 * mtgp::jit_preload_instrs(np1);
  const int keep = mtgp::jit_merge_keep(g) ? 1 : 0;
  const int wait = npre > 0 ? 1 : 0;
  const int body0 = w0 + keep + wait;
  int woff = 0, sp = 0;  // words and stack depth before this chunk
  bool ended = false;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    if (ended) break;  // (wave-uniform)
    const int ii = k * kWave + lane;
    const MtgpInstr x = ii < U.L ? prog[ii] : end;
    const uint32_t c = x.op >> MTGP_OP_SHIFT;
    const uint64_t ends = __ballot(c == (uint32_t)MTGP_OP_END);
    const int first_end = ends ? __ffsll((unsigned long long)ends) - 1 : kWave;
    const bool in = lane < first_end;
    const uint32_t f = (in && c < 64u) ? optab.flags[c] : 0u;
    int w = (in && c < 64u) ? optab.words[c] : 0;
    if (in) {  // + a ds_read / s_waitcnt (3 words) per data operand that is not preloaded
      uint32_t ib;
      __builtin_memcpy(&ib, &x.imm, 4);
      const int sa = (f & kOpIbSlot) ? (int)(ib / MTGP_SLOT_BYTES) : -1;
      const int sb = (f & kOpAxSlot) ? (int)((x.op & 0xffffffu) / MTGP_SLOT_BYTES) : -1;
      bool pa = false, pb = false;
#pragma unroll
      for (int r = 0; r < mtgp::kJitPreSlots; ++r) {
        pa = pa || (r < npre && pre_tab[r] == sa);
        pb = pb || (r < npre && pre_tab[r] == sb);
      }
      w += (sa >= 0 && !pa ? 3 : 0) + (sb >= 0 && !pb ? 3 : 0);
    }
    const int d = (f & kOpPush) ? 1 : ((f & kOpPop) ? -1 : 0);
    int wi = w, di = d;  // inclusive prefix sums over the chunk
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int vw = __shfl_up(wi, off), vd = __shfl_up(di, off);
      if (lane >= off) { wi += vw; di += vd; }
    }
    if (in) {
      const MtgpInstr t[2] = {x, end};
      mtgp::JitOut o{out + body0 + woff + (wi - w), 0};
      o.base = at + (uint32_t)(body0 + woff + (wi - w)) * 4u;
      (void)mtgp::jit_program(o, t, 2, false, mtgp::kJitModeLds, 3, set, 0, nullptr, sp + di - d, pre_tab, npre);
    }
    woff += __shfl(wi, kWave - 1);
    sp += __shfl(di, kWave - 1);
    ended = ends != 0ull;
  }
  if (lane == 0) {
    mtgp::JitOut o{out, 0};
    o.base = at;
    o.n = w0;
    if (keep) o.movv(mtgp::kJitKeep, mtgp::kJitAcc);
    if (wait) o.w(mtgp::jit_wait_lgkm(mtgp::jit_preload_instrs(np1)));
    o.n = body0 + woff;
    if (g > 0) mtgp::jit_merge_tail(o, g, U.Rp, last);
    if (last) mtgp::jit_unit_end(o, U.next, U.cond, j, U.store, U.n_prog);
  }
}

// the shared subroutines (sin, cos, exp, log, tanh, sqrt) at the start of the code buffer
__global__ void __launch_bounds__(256) k_jit_templates(uint32_t* __restrict__ code, uint64_t code_bytes) {
  if (code_bytes < mtgp::kJitTemplateBytes) return;
  for (int i = threadIdx.x; i < MTGP_JIT_SUB_WORDS; i += blockDim.x) code[i] = mtgp_jit_sub_blob[i];
}

bool jit_unit_args(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R, const int32_t* order,
                   JitUnitArgs& U) {
  // R: the lane set (MtgpRollouts.lanes) or the rollout count; a set wider than a wave holds one
  // individual, whose waves share its units
  if (!prog || P < 0 || n_prog <= 0 || n_prog > MTGP_MAX_PROGRAMS || L <= 0 || R <= 0 || R > MTGP_MAX_ROLLOUTS)
    return false;
  int Rp = 1;
  while (Rp < R) Rp <<= 1;
  if (Rp > kWave) Rp = kWave;
  U.prog = prog;
  U.n_prog = n_prog;
  U.L = L;
  U.P = P;
  U.Rp = Rp;
  U.G = kWave / Rp;
  U.order = order;
  U.mode = mtgp::kJitModeRegs;
  U.next = U.cond = U.store = U.put = 0u;
  U.put_slot = 0;
  U.pipe = 1;
  const long waves = ((long)P + U.G - 1) / U.G;
  if (waves * n_prog > INT32_MAX - 1) return false;
  U.n_units = (int)(waves * n_prog);
  return true;
}

// The role chain the evaluator kernels of `m` call (mtgp.h MtgpJitChain): the state role's
// programs prog_state .. prog_state + M - 1 (M = state_size for the dynamic policy, n_var for
// register-resident SR) as one chain when M >= 2, continued into the save-point readout when the
// fixed-step dynamic kernel can use it (the readout_save program right after the state programs).
MtgpJitChain jit_chain_for(const MtgpModel& m, int n_prog) {
  MtgpJitChain c{0u, 0u, 0u, 0u, 0};
  int first = m.prog_state, M = 0;
  const int lim = n_prog < 32 ? n_prog : 32;
  if (m.model == MTGP_MODEL_SR) {
    if (m.n_var > 4) {  // the wide-state kernels: one LDS store chain per wave (its kWideComp components)
      if (m.prog_state == 0 && n_prog >= m.n_var) c.store = (uint32_t)kWideComp;
      return c;
    }
    M = m.n_var;
  } else if (m.model == MTGP_MODEL_DYNAMIC) {
    if (m.state_size > 3) return c;  // runtime state size: LDS-data code, one unit per program (round 6)
    M = m.state_size;
    // fixed step (ABI v18): readout -> u into its data slot -> state programs, one call per stage
    // (the readout reads [0, a, 0, tar] with y and u folded, so y may already sit in its slots)
    const int uslot = m.n_var + m.state_size;
    if (m.solver != MTGP_SOLVER_DOPRI5 && m.state_size >= 1 && m.prog_readout >= 0 && m.prog_readout + 1 == first &&
        1 + M <= mtgp::kJitChainMax && first + M <= lim && uslot < kDMax) {
      for (int k = 0; k < M; ++k) c.next |= 1u << (m.prog_readout + k);
      c.put = 1u << m.prog_readout;
      c.put_slot = uslot;
      return c;
    }
  } else {
    return c;
  }
  if (M < 2 || M > mtgp::kJitChainMax || first < 0 || first + M > lim) return c;
  for (int k = 0; k + 1 < M; ++k) c.next |= 1u << (first + k);
  return c;
}

// a chain's put is a data register of the register-data ABI (v0-v7)
static bool jit_chain_put_ok(const MtgpJitChain& c) { return c.put == 0u || (c.put_slot >= 0 && c.put_slot < kDMax); }

// Executable device memory for the JIT (HSA pool allocation with the executable flag on the
// coarse-grained pool of the agent that backs HIP device `dev`, matched by PCI location).
struct JitAgentQuery {
  uint32_t domain, bdf;
  bool found;
  hsa_agent_t agent;
  hsa_amd_memory_pool_t pool;
  bool have_pool;
};

hsa_status_t jit_find_agent(hsa_agent_t a, void* data) {
  JitAgentQuery* q = (JitAgentQuery*)data;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if ((bdf >> 3) == (q->bdf >> 3) && dom == q->domain) {
    q->agent = a;
    q->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t jit_find_pool(hsa_amd_memory_pool_t p, void* data) {
  JitAgentQuery* q = (JitAgentQuery*)data;
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) {
    q->pool = p;
    q->have_pool = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

#endif  // MTGP_TU_MAIN

// Kernel timing (mtgp_set_timing / mtgp_last_kernel_ms / mtgp_kernel_ms_history): the switch is
// process-wide; the event pairs (a ring of the last kTimingRing launches, so a caller can read the
// durations of a whole run after one synchronisation instead of stalling the queue every launch)
// are per host thread and re-created when the thread moves to another device, so concurrent callers
// on different threads / streams / devices never share events.
std::atomic<bool> g_timing{false};
constexpr int kTimingRing = 1024;
struct TimingState {
  hipEvent_t ev0[kTimingRing] = {}, ev1[kTimingRing] = {};
  int device = -1;
  long long count = 0;  // timed launches recorded on `device`
  void reset(int dev) {
    for (int i = 0; i < kTimingRing; ++i)
      if (ev0[i]) { (void)hipEventDestroy(ev0[i]); (void)hipEventDestroy(ev1[i]); ev0[i] = ev1[i] = nullptr; }
    device = dev;
    count = 0;
  }
};
thread_local TimingState t_timing;

float timing_ms(const TimingState& ts, long long i) {
  const int k = (int)(i % kTimingRing);
  float ms = -1.0f;
  (void)hipEventElapsedTime(&ms, ts.ev0[k], ts.ev1[k]);
  return ms;
}

template <class F>
int launch_timed(F&& launch, hipStream_t s) {
  const bool timing = g_timing.load(std::memory_order_relaxed);
  TimingState& ts = t_timing;
  int k = 0;
  if (timing) {
    int dev = -1;
    (void)hipGetDevice(&dev);
    if (ts.device != dev) ts.reset(dev);
    k = (int)(ts.count % kTimingRing);
    if (!ts.ev0[k]) { (void)hipEventCreate(&ts.ev0[k]); (void)hipEventCreate(&ts.ev1[k]); }
    (void)hipEventRecord(ts.ev0[k], s);
  }
  launch();
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  if (timing) { (void)hipEventRecord(ts.ev1[k], s); ++ts.count; }
  return MTGP_OK;
}

}  // namespace

// the eight (TRAJ, NOISE, JIT) variants of one control kernel; an Env with kMask (EnvAcrobotMask)
// has the four TRAJ variants only (the caller passes traj = true)
template <class E, int... N>
constexpr bool kTrajOnly = E::kMask;
#define MTGP_CTL_VARIANTS(KERNEL, ...)                                                                   \
  do {                                                                                                  \
    if (jit) {                                                                                          \
      if (noise) {                                                                                      \
        if (traj) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, true, true>), grid, block, 0, s, A);    \
        else if constexpr (!kTrajOnly<__VA_ARGS__>)                                                     \
          hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, true, true>), grid, block, 0, s, A);           \
      } else {                                                                                          \
        if (traj) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, false, true>), grid, block, 0, s, A);   \
        else if constexpr (!kTrajOnly<__VA_ARGS__>)                                                     \
          hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, false, true>), grid, block, 0, s, A);          \
      }                                                                                                 \
    } else if (noise) {                                                                                 \
      if (traj) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, true, false>), grid, block, 0, s, A);     \
      else if constexpr (!kTrajOnly<__VA_ARGS__>)                                                       \
        hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, true, false>), grid, block, 0, s, A);            \
    } else {                                                                                            \
      if (traj) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, false, false>), grid, block, 0, s, A);    \
      else if constexpr (!kTrajOnly<__VA_ARGS__>)                                                       \
        hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, false, false>), grid, block, 0, s, A);           \
    }                                                                                                   \
  } while (0)

template <class Env, int NA>
int launch_dyn(const KArgs& A, bool jit, bool noise, bool traj, dim3 grid, dim3 block, hipStream_t s) {
  // (NA > 3, state_size 4 .. kNaWide: the data vector lives in LDS -- interpreter, or LDS-data JIT
  // code, round 6)
  return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_dynamic, Env, NA); }, s);
}

// Launch 2's order (round 6): the parked waves longest-first by their remaining-work estimate
// (DpParked::kEstWord of lane 0), so the hardware dispatches the waves that bound the kernel's tail
// before the short ones (longest-processing-time order).  One workgroup, a counting sort over 256
// log-scale buckets in LDS (order inside a bucket arbitrary: results do not depend on the order);
// more than kDpOrderMax parked waves keep the order they parked in.
constexpr int kDpOrderMax = 8192;
static __global__ void __launch_bounds__(1024) k_dp_order(int32_t* pending, const float* state, uint32_t stride) {
  __shared__ int hist[256];
  __shared__ int ids[kDpOrderMax];
  __shared__ unsigned char keys[kDpOrderMax];
  const int n = pending[0];
  if (n <= 1 || n > kDpOrderMax) return;
  for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int id = pending[1 + i];
    const float est = state[(size_t)(kDpStateWords - 1) * stride + (size_t)id * kWave];
    const float q = est > 0.0f ? 16.0f * __log2f(est + 1.0f) : 0.0f;  // 1/16-octave buckets
    const int key = 255 - (q >= 255.0f ? 255 : (int)q);               // longest first
    ids[i] = id;
    keys[i] = (unsigned char)key;
    atomicAdd(&hist[key], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < 256; ++b) {
      const int c = hist[b];
      hist[b] = acc;
      acc += c;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) pending[1 + atomicAdd(&hist[keys[i]], 1)] = ids[i];
}

// adaptive Dopri5 at a runtime state size (NA = kNaRuntime / kNaWide): interpreter variants only;
// the non-mask environments' kernels live in TU 9 (their register allocation dominates a build)
__attribute__((visibility("hidden"))) int mtgp_tu_launch_dp_rt(const void* A, int env, bool wide, bool noise, bool traj,
                                                                unsigned grid, unsigned block, hipStream_t s);
template <class Env, int NA>
int launch_dp_rt(const KArgs& A, bool noise, bool traj, dim3 grid, dim3 block, hipStream_t s) {
  return launch_timed([&] {
    if (noise) {
      if (traj) hipLaunchKernelGGL((k_ctl_dopri5<Env, NA, true, true, false>), grid, block, 0, s, A);
      else if constexpr (!Env::kMask) hipLaunchKernelGGL((k_ctl_dopri5<Env, NA, false, true, false>), grid, block, 0, s, A);
    } else if (traj) {
      hipLaunchKernelGGL((k_ctl_dopri5<Env, NA, true, false, false>), grid, block, 0, s, A);
    } else if constexpr (!Env::kMask) {
      hipLaunchKernelGGL((k_ctl_dopri5<Env, NA, false, false, false>), grid, block, 0, s, A);
    }
  }, s);
}

// adaptive Dopri5 variants (k_ctl_dopri5): static = NA 0
template <class Env>
int launch_ctl_dp(const KArgs& A, const MtgpModel* model, bool jit, bool noise, bool traj, dim3 grid, dim3 block,
                  hipStream_t s) {
  if (model->model == MTGP_MODEL_STATIC) return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_dopri5, Env, 0); }, s);
  switch (model->state_size) {
    case 1: return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_dopri5, Env, 1); }, s);
    case 2: return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_dopri5, Env, 2); }, s);
    case 3: return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_dopri5, Env, 3); }, s);
    default:  // runtime state size (round 6): interpreter only, one launch
      if (jit || model->state_size < 4 || model->state_size > kNaWide) return MTGP_ERR_ARG;
      if constexpr (Env::kMask) {  // (the cost-mask kernels stay in their own TU)
        return model->state_size > kNaRuntime ? launch_dp_rt<Env, kNaWide>(A, noise, traj, grid, block, s)
                                              : launch_dp_rt<Env, kNaRuntime>(A, noise, traj, grid, block, s);
      } else {
        const int env = std::is_same<Env, EnvAcrobot>::value ? 0 : std::is_same<Env, EnvHarmonic>::value ? 1 : 2;
        return mtgp_tu_launch_dp_rt(&A, env, model->state_size > kNaRuntime, noise, traj, grid.x, block.x, s);
      }
  }
}
// every environment's Dopri5 kernels live in their own translation unit (MTGP_TU 3, 4, 5)
#define MTGP_TU_DP_ARGS \
  const void* A, const MtgpModel* model, bool jit, bool noise, bool traj, unsigned grid, unsigned block, hipStream_t s
__attribute__((visibility("hidden"))) int mtgp_tu_launch_acrobot_dopri5(MTGP_TU_DP_ARGS);
__attribute__((visibility("hidden"))) int mtgp_tu_launch_harmonic_dopri5(MTGP_TU_DP_ARGS);
__attribute__((visibility("hidden"))) int mtgp_tu_launch_reactor_dopri5(MTGP_TU_DP_ARGS);
template <class Env>
int launch_dp_entry(MTGP_TU_DP_ARGS) {
  if constexpr (Env::kMask) return launch_ctl_dp<Env>(*(const KArgs*)A, model, jit, noise, traj, dim3(grid), dim3(block), s);
  else if constexpr (std::is_same<Env, EnvAcrobot>::value) return mtgp_tu_launch_acrobot_dopri5(A, model, jit, noise, traj, grid, block, s);
  else if constexpr (std::is_same<Env, EnvHarmonic>::value) return mtgp_tu_launch_harmonic_dopri5(A, model, jit, noise, traj, grid, block, s);
  else return mtgp_tu_launch_reactor_dopri5(A, model, jit, noise, traj, grid, block, s);
}

// dynamic / static evaluator on environment Env: shape checks, then the kernel variant
template <class Env>
int launch_ctl(const KArgs& A, const MtgpModel* model, const MtgpRollouts* ro, bool jit, bool noise, bool traj,
               dim3 grid, dim3 block, hipStream_t s) {
  constexpr int NV = Env::NV;
  if (model->n_var != NV || model->n_obs < 1 || model->n_obs > NV || model->n_control != 1 || !ro->params)
    return MTGP_ERR_ARG;
  if (model->n_targets < 0 || (model->n_targets > 0 && !ro->targets)) return MTGP_ERR_ARG;
  if (model->env != MTGP_ENV_ACROBOT && model->n_targets < 1) return MTGP_ERR_ARG;  // x_d needs the target
  if (model->model == MTGP_MODEL_STATIC) {
    if (NV + model->n_targets > kDMax) return MTGP_ERR_ARG;
  } else if (model->state_size > 3) {  // runtime state size: the wide interpreter kernels, every solver
    const int dm = model->state_size > kNaRuntime ? kDWide2 : kDWide;
    // (JIT: LDS-data code, fixed-step solvers; Dopri5: interpreter, one launch -- no parking)
    if (model->state_size > kNaWide || NV + model->state_size + 1 + model->n_targets > dm ||
        (model->solver == MTGP_SOLVER_DOPRI5 && (jit || A.dp_budget > 0)))
      return MTGP_ERR_ARG;
  } else if (NV + model->state_size + 1 + model->n_targets > kDMax) {
    return MTGP_ERR_ARG;
  }
  if (model->solver == MTGP_SOLVER_DOPRI5) {
    int rc = MTGP_OK;
    const int lr = launch_timed([&] {
      if (A.dp_budget <= 0) {
        rc = launch_dp_entry<Env>(&A, model, jit, noise, traj, grid.x, block.x, s);
        return;
      }
      // two launches: every wave for dp_budget attempts, then the parked waves (KArgs.dp_*)
      if (hipMemsetAsync(A.dp_pending, 0, sizeof(int32_t), s) != hipSuccess) { rc = MTGP_ERR_LAUNCH; return; }
      KArgs A1 = A;
      A1.dp_pass = 1;
      rc = launch_dp_entry<Env>(&A1, model, jit, noise, traj, grid.x, block.x, s);
      if (rc != MTGP_OK) return;
      hipLaunchKernelGGL(k_dp_order, dim3(1), dim3(1024), 0, s, A.dp_pending, (const float*)A.dp_state, A.dp_lanes);
      KArgs A2 = A;
      A2.dp_pass = 2;
      rc = launch_dp_entry<Env>(&A2, model, jit, noise, traj, grid.x, block.x, s);
    }, s);
    return rc != MTGP_OK ? rc : lr;
  }
  if (model->model == MTGP_MODEL_STATIC) return launch_timed([&] { MTGP_CTL_VARIANTS(k_ctl_static, Env); }, s);
  switch (model->state_size) {
    case 1: return launch_dyn<Env, 1>(A, jit, noise, traj, grid, block, s);
    case 2: return launch_dyn<Env, 2>(A, jit, noise, traj, grid, block, s);
    case 3: return launch_dyn<Env, 3>(A, jit, noise, traj, grid, block, s);
    default:
      if (model->state_size < 4 || model->state_size > kNaWide) return MTGP_ERR_ARG;
      return model->state_size > kNaRuntime ? launch_dyn<Env, kNaWide>(A, jit, noise, traj, grid, block, s)
                                            : launch_dyn<Env, kNaRuntime>(A, jit, noise, traj, grid, block, s);
  }
}


// entries of the split-off environment TUs (hidden: not part of the C ABI)
#define MTGP_TU_ENTRY_ARGS                                                                              \
  const void* A, const MtgpModel* model, const MtgpRollouts* ro, bool jit, bool noise, bool traj,       \
      unsigned grid, unsigned block, hipStream_t s
__attribute__((visibility("hidden"))) int mtgp_tu_launch_harmonic(MTGP_TU_ENTRY_ARGS);
__attribute__((visibility("hidden"))) int mtgp_tu_launch_reactor(MTGP_TU_ENTRY_ARGS);
__attribute__((visibility("hidden"))) int mtgp_tu_launch_acrobot_mask(MTGP_TU_ENTRY_ARGS);
__attribute__((visibility("hidden"))) int mtgp_tu_launch_acrobot(MTGP_TU_ENTRY_ARGS);
#if MTGP_DEBUG_CHECKS && defined(MTGP_TU)
#define MTGP_DBG_CAT2(a, b) a##b
#define MTGP_DBG_CAT(a, b) MTGP_DBG_CAT2(a, b)
// debug build only: this translation unit's violation counters (read and cleared)
extern "C" int MTGP_DBG_CAT(mtgp_debug_violations_tu, MTGP_TU)(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_viol), 4 * sizeof(unsigned long long)) != hipSuccess) return -1;
  const unsigned long long z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_viol), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#if MTGP_TU == 0
// positive control of the counters: one store at lane offset 5 into a row of 4 (counted, dropped)
__global__ void k_dbg_selftest(float* buf) {
  if (threadIdx.x == 0) store_row(buf, 0, 5, 1.0f, 4);
}
extern "C" int mtgp_debug_selftest(void) {
  float* d = nullptr;
  if (hipMalloc(&d, 4 * sizeof(float)) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_dbg_selftest, dim3(1), dim3(64), 0, 0, d);
  const int rc = hipDeviceSynchronize() == hipSuccess ? 0 : -1;
  (void)hipFree(d);
  return rc;
}
#endif
#endif
#if MTGP_AB_WAVETIME && defined(MTGP_TU) && MTGP_TU == 7
extern "C" int mtgp_ab_wave_times(unsigned long long* t, unsigned int* hw, int n) {  // diagnostic build only
  if (n > kWaveTimeMax) n = kWaveTimeMax;
  if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wave_time), (size_t)n * 2 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_wave_hw), (size_t)n * 2 * sizeof(unsigned int)) != hipSuccess) return -1;
  return n;
}
#endif
#if MTGP_TU_ACRO && MTGP_AB_FBCOUNT
extern "C" int mtgp_ab_fb_count(unsigned long long* host) {  // diagnostic build only; reads and clears
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ab_fb_count), 4 * sizeof(unsigned long long)) != hipSuccess) return -1;
  const unsigned long long z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ab_fb_count), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
#if MTGP_TU_ACRO
int mtgp_tu_launch_acrobot(MTGP_TU_ENTRY_ARGS) {  // fixed-step solvers (Dopri5 goes on to TU 3)
  return launch_ctl<EnvAcrobot>(*(const KArgs*)A, model, ro, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_ACRO_MASK
int mtgp_tu_launch_acrobot_mask(MTGP_TU_ENTRY_ARGS) {  // every solver; the trajectory variants (traj unused)
  (void)traj;
  return launch_ctl<EnvAcrobotMask>(*(const KArgs*)A, model, ro, jit, noise, true, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_ACRO_DOPRI5
int mtgp_tu_launch_acrobot_dopri5(MTGP_TU_DP_ARGS) {
  return launch_ctl_dp<EnvAcrobot>(*(const KArgs*)A, model, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_DP_RT
int mtgp_tu_launch_dp_rt(const void* Ap, int env, bool wide, bool noise, bool traj, unsigned grid, unsigned block,
                         hipStream_t s) {
  const KArgs& A = *(const KArgs*)Ap;
  const dim3 g(grid), b(block);
  switch (env) {
    case 0: return wide ? launch_dp_rt<EnvAcrobot, kNaWide>(A, noise, traj, g, b, s)
                        : launch_dp_rt<EnvAcrobot, kNaRuntime>(A, noise, traj, g, b, s);
    case 1: return wide ? launch_dp_rt<EnvHarmonic, kNaWide>(A, noise, traj, g, b, s)
                        : launch_dp_rt<EnvHarmonic, kNaRuntime>(A, noise, traj, g, b, s);
    default: return wide ? launch_dp_rt<EnvReactor, kNaWide>(A, noise, traj, g, b, s)
                         : launch_dp_rt<EnvReactor, kNaRuntime>(A, noise, traj, g, b, s);
  }
}
#endif
#if MTGP_TU_HARMONIC_DOPRI5
int mtgp_tu_launch_harmonic_dopri5(MTGP_TU_DP_ARGS) {
  return launch_ctl_dp<EnvHarmonic>(*(const KArgs*)A, model, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_REACTOR_DOPRI5
int mtgp_tu_launch_reactor_dopri5(MTGP_TU_DP_ARGS) {
  return launch_ctl_dp<EnvReactor>(*(const KArgs*)A, model, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_HARMONIC
int mtgp_tu_launch_harmonic(MTGP_TU_ENTRY_ARGS) {
  return launch_ctl<EnvHarmonic>(*(const KArgs*)A, model, ro, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif
#if MTGP_TU_REACTOR
int mtgp_tu_launch_reactor(MTGP_TU_ENTRY_ARGS) {
  return launch_ctl<EnvReactor>(*(const KArgs*)A, model, ro, jit, noise, traj, dim3(grid), dim3(block), s);
}
#endif


// the SR kernels (MTGP_TU 8): register-resident n_var <= 4 and the wide-state workgroup kernels
#define MTGP_TU_SR_ARGS \
  const void* A_, const MtgpModel* model, bool jit, bool traj, bool dopri5, unsigned G, unsigned Wset, unsigned grid_, \
      unsigned block_, hipStream_t s
__attribute__((visibility("hidden"))) int mtgp_tu_launch_sr(MTGP_TU_SR_ARGS);
#if MTGP_TU_SR
int mtgp_tu_launch_sr(MTGP_TU_SR_ARGS) {
  const KArgs& A = *(const KArgs*)A_;
  const dim3 grid(grid_), block(block_);
  if (model->n_var > 4) {
    const int nw = (model->n_var + kWideComp - 1) / kWideComp;
    const dim3 wgrid((unsigned)(((long)A.P + G - 1) / G * Wset)), wblock(kWave * nw);
    if (dopri5) {  // + a reduction vector (error norm, MSE)
      const size_t lds_dp = (size_t)(3 * model->n_var + nw * kSMax + nw) * kWave * sizeof(float);
      return launch_timed([&] {
        if (jit) {
          if (traj) hipLaunchKernelGGL((k_sr_wide_dopri5<true, true>), wgrid, wblock, lds_dp, s, A);
          else hipLaunchKernelGGL((k_sr_wide_dopri5<false, true>), wgrid, wblock, lds_dp, s, A);
        } else if (traj) hipLaunchKernelGGL((k_sr_wide_dopri5<true, false>), wgrid, wblock, lds_dp, s, A);
        else hipLaunchKernelGGL((k_sr_wide_dopri5<false, false>), wgrid, wblock, lds_dp, s, A);
      }, s);
    }
    size_t lds = (size_t)(2 * model->n_var + nw * kSMax + nw) * kWave * sizeof(float);
    if (const char* e = getenv("MTGP_WIDE_LDS_MIN")) {  // diagnostic: fewer workgroups per CU (code working set)
      const long v = atol(e);
      if (v > 0 && (size_t)v > lds && v <= 160 * 1024) lds = (size_t)v;
    }
    return launch_timed([&] {
      if (jit) {
        if (traj) hipLaunchKernelGGL((k_sr_wide<true, true>), wgrid, wblock, lds, s, A);
        else hipLaunchKernelGGL((k_sr_wide<false, true>), wgrid, wblock, lds, s, A);
      } else if (traj) hipLaunchKernelGGL((k_sr_wide<true, false>), wgrid, wblock, lds, s, A);
      else hipLaunchKernelGGL((k_sr_wide<false, false>), wgrid, wblock, lds, s, A);
    }, s);
  }
#define MTGP_SR(NV)                                                                                       \
  case NV:                                                                                                \
  return launch_timed([&] {                                                                             \
    if (dopri5) {                                                                                       \
      if (jit) {                                                                                        \
        if (traj) hipLaunchKernelGGL((k_sr_dopri5<NV, true, true>), grid, block, 0, s, A);              \
        else hipLaunchKernelGGL((k_sr_dopri5<NV, false, true>), grid, block, 0, s, A);                  \
      } else if (traj) hipLaunchKernelGGL((k_sr_dopri5<NV, true, false>), grid, block, 0, s, A);        \
      else hipLaunchKernelGGL((k_sr_dopri5<NV, false, false>), grid, block, 0, s, A);                   \
    } else if (jit) {                                                                                   \
      if (traj) hipLaunchKernelGGL((k_sr<NV, true, true>), grid, block, 0, s, A);                       \
      else hipLaunchKernelGGL((k_sr<NV, false, true>), grid, block, 0, s, A);                           \
    } else if (traj) hipLaunchKernelGGL((k_sr<NV, true, false>), grid, block, 0, s, A);                 \
    else hipLaunchKernelGGL((k_sr<NV, false, false>), grid, block, 0, s, A);                            \
  }, s);
  switch (model->n_var) {
    MTGP_SR(1)
    MTGP_SR(2)
    MTGP_SR(3)
    MTGP_SR(4)
    default: return MTGP_ERR_ARG;
  }
#undef MTGP_SR
  return MTGP_ERR_ARG;
}
#endif

#if MTGP_TU_MAIN
// a split-off TU's launch, timed with this TU's events (mtgp_last_kernel_ms)
template <class F>
int launch_tu(F&& entry, hipStream_t s) {
  int rc = MTGP_OK;
  const int lr = launch_timed([&] { rc = entry(); }, s);
  return rc != MTGP_OK ? rc : lr;
}

extern "C" {

int mtgp_abi_version(void) { return MTGP_ABI_VERSION; }


int mtgp_jit_alloc(int32_t device, size_t bytes, void** code) {
  if (!code || bytes == 0) return MTGP_ERR_ARG;
  *code = nullptr;
  static std::once_flag hsa_once;  // thread-safe one-time HSA runtime init (HIP already holds a reference)
  static hsa_status_t hsa_rc = HSA_STATUS_ERROR;
  std::call_once(hsa_once, [] { hsa_rc = hsa_init(); });
  if (hsa_rc != HSA_STATUS_SUCCESS) return MTGP_ERR_LAUNCH;
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
    return MTGP_ERR_ARG;
  JitAgentQuery q{(uint32_t)dom, (uint32_t)(bus << 8 | dev << 3), false, {}, {}, false};
  hsa_iterate_agents(jit_find_agent, &q);
  if (!q.found) return MTGP_ERR_ARG;
  hsa_amd_agent_iterate_memory_pools(q.agent, jit_find_pool, &q);
  if (!q.have_pool) return MTGP_ERR_ARG;
  if (hsa_amd_memory_pool_allocate(q.pool, bytes, HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, code) != HSA_STATUS_SUCCESS) {
    *code = nullptr;
    return MTGP_ERR_LAUNCH;
  }
  return MTGP_OK;
}

int mtgp_jit_free(void* code) {
  if (!code) return MTGP_OK;
  return hsa_amd_memory_pool_free(code) == HSA_STATUS_SUCCESS ? MTGP_OK : MTGP_ERR_ARG;
}

int mtgp_jit_units(int32_t P, int32_t n_prog, int32_t R) {
  JitUnitArgs U;
  static const MtgpInstr dummy = {0u, 0.0f};
  if (!jit_unit_args(&dummy, P, n_prog, 1, R, nullptr, U)) return MTGP_ERR_ARG;
  return U.n_units;
}

int mtgp_jit_plan(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R, const int32_t* order,
                  uint32_t* offsets_out, int32_t* info_out, void* stream) {
  JitUnitArgs U;
  if (!offsets_out || !info_out || !jit_unit_args(prog, P, n_prog, L, R, order, U)) return MTGP_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(info_out, 0, 2 * sizeof(int32_t), s) != hipSuccess) return MTGP_ERR_LAUNCH;
  if (U.n_units == 0) return hipMemsetAsync(offsets_out, 0, sizeof(uint32_t), s) == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  hipLaunchKernelGGL(k_jit_count, dim3((unsigned)((U.n_units + 255) / 256)), dim3(256), 0, s, U, offsets_out,
                     info_out);
  hipLaunchKernelGGL(k_jit_scan, dim3(1), dim3(1024), 0, s, offsets_out, U.n_units, info_out);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_jit_chain(const MtgpModel* model, int32_t n_prog, MtgpJitChain* chain_out) {
  if (!model || !chain_out || n_prog <= 0) return MTGP_ERR_ARG;
  *chain_out = jit_chain_for(*model, n_prog);
  return MTGP_OK;
}

int mtgp_jit_plan_words(const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t R, const int32_t* order,
                        uint32_t* offsets_out, int32_t* info_out, void* stream) {
  return mtgp_jit_plan_words_chain(jit_words, P, n_prog, R, order, nullptr, offsets_out, info_out, stream);
}

int mtgp_jit_plan_words_chain(const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t R, const int32_t* order,
                              const MtgpJitChain* chain, uint32_t* offsets_out, int32_t* info_out, void* stream) {
  JitUnitArgs U;
  static const MtgpInstr dummy = {0u, 0.0f};
  if (!jit_words || !offsets_out || !info_out || !jit_unit_args(&dummy, P, n_prog, 1, R, order, U)) return MTGP_ERR_ARG;
  if (chain) {
    if (!jit_chain_put_ok(*chain)) return MTGP_ERR_ARG;
    U.next = chain->next; U.cond = chain->cond; U.store = chain->store; U.put = chain->put; U.put_slot = chain->put_slot;
  }
  hipStream_t s = (hipStream_t)stream;
  if (U.n_units == 0) {
    if (hipMemsetAsync(info_out, 0, 2 * sizeof(int32_t), s) != hipSuccess) return MTGP_ERR_LAUNCH;
    return hipMemsetAsync(offsets_out, 0, sizeof(uint32_t), s) == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(k_jit_sizes, dim3((unsigned)((U.n_units + 255) / 256)), dim3(256), 0, s, U, jit_words,
                     offsets_out);
  if (U.n_units <= 1024 * 16)
    hipLaunchKernelGGL(k_jit_scan_sizes_reg<16>, dim3(1), dim3(1024), 0, s, offsets_out, U.n_units, info_out);
  else if (U.n_units <= 1024 * 32)
    hipLaunchKernelGGL(k_jit_scan_sizes_reg<32>, dim3(1), dim3(1024), 0, s, offsets_out, U.n_units, info_out);
  else
    hipLaunchKernelGGL(k_jit_scan_sizes, dim3(1), dim3(1024), 0, s, offsets_out, U.n_units, info_out);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_jit_emit_words(const MtgpInstr* prog, const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t L,
                        int32_t R, const int32_t* order, const uint32_t* offsets, void* code, size_t code_bytes,
                        int32_t jit_mode, void* stream) {
  return mtgp_jit_emit_words_chain(prog, jit_words, P, n_prog, L, R, order, nullptr, offsets, code, code_bytes,
                                   jit_mode, stream);
}

int mtgp_jit_emit_words_chain(const MtgpInstr* prog, const int32_t* jit_words, int32_t P, int32_t n_prog, int32_t L,
                              int32_t R, const int32_t* order, const MtgpJitChain* chain, const uint32_t* offsets,
                              void* code, size_t code_bytes, int32_t jit_mode, void* stream) {
  JitUnitArgs U;
  if (!jit_words || !offsets || !code || !jit_unit_args(prog, P, n_prog, L, R, order, U)) return MTGP_ERR_ARG;
  if (jit_mode != mtgp::kJitModeRegs && jit_mode != mtgp::kJitModeLds) return MTGP_ERR_ARG;
  U.mode = jit_mode;
  {  // A/B knob: MTGP_JIT_LDS_PIPE=0 emits LDS-data units without the preload pipelining
    const char* e = getenv("MTGP_JIT_LDS_PIPE");
    U.pipe = !(e && strcmp(e, "0") == 0);
  }
  if (chain) {
    if (jit_mode != mtgp::kJitModeRegs && (chain->next | chain->cond) != 0u) return MTGP_ERR_ARG;  // v26.. are preloads
    if (jit_mode != mtgp::kJitModeLds && chain->store != 0u) return MTGP_ERR_ARG;  // store chains: LDS-data code
    if (!jit_chain_put_ok(*chain) || (jit_mode != mtgp::kJitModeRegs && chain->put != 0u)) return MTGP_ERR_ARG;
    U.next = chain->next;
    U.cond = chain->cond;
    U.store = chain->store;
    U.put = chain->put;
    U.put_slot = chain->put_slot;
  }
  if (U.n_units == 0) return MTGP_OK;
  hipStream_t s = (hipStream_t)stream;
  const long threads = (long)U.n_units * U.G;  // (block 0 also writes the shared sin/cos templates)
  const char* ew = getenv("MTGP_JIT_EMIT");  // A/B knob: MTGP_JIT_EMIT=thread / wave (read per call: tests switch it)
  // register-data units: as many (unit, group) pairs per wave as keep the launch within one round of
  // resident waves (kResidentWaves): one wave per pair up to 8,192 pairs, two up to 16,384, else
  // four (C3: 32,768 pairs; C2's 1,024 run one per wave -- packing only lengthens a wave's chain
  // when the chip has room for all of them).  MTGP_JIT_EMIT=wave64 / halves / quarters force one.
  const bool force64 = ew && strcmp(ew, "wave64") == 0, forceh = ew && strcmp(ew, "halves") == 0,
             forceq = ew && strcmp(ew, "quarters") == 0;
  const bool pack = forceh || forceq || (!force64 && threads > kResidentWaves);
  if (U.mode == mtgp::kJitModeRegs && !(ew && strcmp(ew, "thread") == 0) && pack && U.L <= 5 * kWave) {
    static const JitOpTable optab = jit_op_table();
    const bool quarters = forceq || (!forceh && threads > 2 * kResidentWaves);
    const long hthreads = quarters ? (threads + 3) / 4 * kWave : (threads + 1) / 2 * kWave;
    const dim3 grid((unsigned)((hthreads + 255) / 256));
    if (quarters && U.L <= 3 * kWave)
      hipLaunchKernelGGL((k_jit_emit_halves<12, 16>), grid, dim3(256), 0, s, U, jit_words, offsets, (uint32_t*)code,
                         (uint64_t)code_bytes, optab);
    else if (quarters)
      hipLaunchKernelGGL((k_jit_emit_halves<20, 16>), grid, dim3(256), 0, s, U, jit_words, offsets, (uint32_t*)code,
                         (uint64_t)code_bytes, optab);
    else if (U.L <= 3 * kWave)
      hipLaunchKernelGGL(k_jit_emit_halves<6>, grid, dim3(256), 0, s, U, jit_words, offsets, (uint32_t*)code,
                         (uint64_t)code_bytes, optab);
    else
      hipLaunchKernelGGL(k_jit_emit_halves<10>, grid, dim3(256), 0, s, U, jit_words, offsets, (uint32_t*)code,
                         (uint64_t)code_bytes, optab);
    return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  }
  if (U.mode == mtgp::kJitModeRegs && !(ew && strcmp(ew, "thread") == 0) && U.L <= 5 * kWave) {
    static const JitOpTable optab = jit_op_table();
    const long wthreads = threads * kWave;
    if (U.L <= 3 * kWave)
      hipLaunchKernelGGL(k_jit_emit_waves<3>, dim3((unsigned)((wthreads + 255) / 256)), dim3(256), 0, s, U, jit_words,
                         offsets, (uint32_t*)code, (uint64_t)code_bytes, optab);
    else
      hipLaunchKernelGGL(k_jit_emit_waves<5>, dim3((unsigned)((wthreads + 255) / 256)), dim3(256), 0, s, U, jit_words,
                         offsets, (uint32_t*)code, (uint64_t)code_bytes, optab);
    return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  }
  // LDS-data units: one thread per group (k_jit_emit_groups) by default; MTGP_JIT_EMIT=wave selects the
  // wave-per-group emitter, which measured 3.5x slower at C5 (1.17 vs 0.33 ms, profiles/r04/v11_*:
  // 262k short programs, most lanes of a wave idle, two slot-rank tables per wave)
  if (U.mode == mtgp::kJitModeLds && U.pipe && ew && strcmp(ew, "wave") == 0 && U.L <= 5 * kWave) {
    static const JitOpTable optab = jit_op_table();
    const long blocks = (threads + kEmitLdsWaves - 1) / kEmitLdsWaves;
    if (U.L <= 3 * kWave)
      hipLaunchKernelGGL(k_jit_emit_waves_lds<3>, dim3((unsigned)blocks), dim3(kEmitLdsWaves * kWave), 0, s, U,
                         jit_words, offsets, (uint32_t*)code, (uint64_t)code_bytes, optab);
    else
      hipLaunchKernelGGL(k_jit_emit_waves_lds<5>, dim3((unsigned)blocks), dim3(kEmitLdsWaves * kWave), 0, s, U,
                         jit_words, offsets, (uint32_t*)code, (uint64_t)code_bytes, optab);
    return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(k_jit_emit_groups, dim3((unsigned)((threads + 63) / 64)), dim3(64), 0, s, U, jit_words, offsets,
                     (uint32_t*)code, (uint64_t)code_bytes);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_jit_emit(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R, const int32_t* order,
                  const uint32_t* offsets, void* code, size_t code_bytes, void* stream) {
  JitUnitArgs U;
  if (!offsets || !code || !jit_unit_args(prog, P, n_prog, L, R, order, U)) return MTGP_ERR_ARG;
  if (U.n_units == 0) return MTGP_OK;
  hipLaunchKernelGGL(k_jit_templates, dim3(1), dim3(256), 0, (hipStream_t)stream, (uint32_t*)code,
                     (uint64_t)code_bytes);
  hipLaunchKernelGGL(k_jit_emit, dim3((unsigned)((U.n_units + 255) / 256)), dim3(256), 0, (hipStream_t)stream, U,
                     offsets, (uint32_t*)code, (uint64_t)code_bytes);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_jit_cost(const MtgpInstr* prog, const int32_t* plen, int32_t P, int32_t n_prog, int32_t L, int32_t* cost_out,
                  void* stream) {
  if (!prog || !plen || !cost_out || P < 0 || n_prog <= 0 || L <= 0 || (long)P * n_prog > INT32_MAX) return MTGP_ERR_ARG;
  const long total = (long)P * n_prog;
  if (total == 0) return MTGP_OK;
  hipLaunchKernelGGL(k_jit_cost, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, prog,
                     (int)total, L, plen, cost_out);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

static int jit_unit_host_impl(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                              const int32_t* order, int32_t unit, uint32_t* out, int32_t max_words, int32_t jit_mode,
                              uint32_t next, uint32_t cond, uint32_t store, uint32_t put = 0u, int put_slot = 0) {
  JitUnitArgs U;
  if (!jit_unit_args(prog, P, n_prog, L, R, order, U) || unit < 0 || unit >= U.n_units) return MTGP_ERR_ARG;
  if (jit_mode != mtgp::kJitModeRegs && jit_mode != mtgp::kJitModeLds) return MTGP_ERR_ARG;
  const int wave = unit / n_prog, j = unit - wave * n_prog;
  const int n = mtgp::jit_unit(prog, n_prog, L, P, order, U.G, U.Rp, wave, j, nullptr, mtgp::kJitTemplateBytes, jit_mode,
                               next, cond, store, true, put, put_slot);
  if (n <= 0) return n < 0 ? n - 100 : MTGP_ERR_ARG;
  if (out) {
    if (n > max_words) return MTGP_ERR_ARG;
    mtgp::jit_unit(prog, n_prog, L, P, order, U.G, U.Rp, wave, j, out, mtgp::kJitTemplateBytes, jit_mode, next, cond,
                   store, true, put, put_slot);
  }
  return n;
}

int mtgp_jit_unit_host_ex(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R, const int32_t* order,
                          int32_t unit, uint32_t* out, int32_t max_words, int32_t jit_mode) {
  return jit_unit_host_impl(prog, P, n_prog, L, R, order, unit, out, max_words, jit_mode, 0u, 0u, 0u);
}

int mtgp_jit_unit_host_chain(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R,
                             const int32_t* order, const MtgpJitChain* chain, int32_t unit, uint32_t* out,
                             int32_t max_words, int32_t jit_mode) {
  return jit_unit_host_impl(prog, P, n_prog, L, R, order, unit, out, max_words, jit_mode, chain ? chain->next : 0u,
                            chain ? chain->cond : 0u, chain ? chain->store : 0u, chain ? chain->put : 0u,
                            chain ? chain->put_slot : 0);
}

int mtgp_jit_unit_host(const MtgpInstr* prog, int32_t P, int32_t n_prog, int32_t L, int32_t R, const int32_t* order,
                       int32_t unit, uint32_t* out, int32_t max_words) {
  return mtgp_jit_unit_host_ex(prog, P, n_prog, L, R, order, unit, out, max_words, mtgp::kJitModeRegs);
}

int mtgp_jit_translate_host_ex(const MtgpInstr* prog, int32_t L, uint32_t* out, int32_t max_words, int32_t jit_mode) {
  if (!prog || L <= 0 || (jit_mode != mtgp::kJitModeRegs && jit_mode != mtgp::kJitModeLds)) return MTGP_ERR_ARG;
  const int n = mtgp::jit_translate(prog, L, nullptr, mtgp::kJitTemplateBytes, jit_mode);
  if (n <= 0) return n < 0 ? n - 100 : MTGP_ERR_ARG;  /* translation errors: -101 .. -104 */
  if (out) {
    if (n > max_words) return MTGP_ERR_ARG;
    mtgp::jit_translate(prog, L, out, mtgp::kJitTemplateBytes, jit_mode);
  }
  return n;
}

int mtgp_jit_translate_host(const MtgpInstr* prog, int32_t L, uint32_t* out, int32_t max_words) {
  return mtgp_jit_translate_host_ex(prog, L, out, max_words, mtgp::kJitModeRegs);
}

int mtgp_set_timing(int enabled) {
  g_timing = enabled != 0;
  return MTGP_OK;
}

float mtgp_last_kernel_ms(void) {
  const TimingState& ts = t_timing;  // this thread's last timed launch
  if (ts.count == 0) return -1.0f;
  (void)hipEventSynchronize(ts.ev1[(ts.count - 1) % kTimingRing]);
  return timing_ms(ts, ts.count - 1);
}

int mtgp_kernel_ms_history(float* out, int32_t n) {
  const TimingState& ts = t_timing;
  if (!out || n < 0) return MTGP_ERR_ARG;
  long long avail = ts.count < kTimingRing ? ts.count : kTimingRing;
  if (n > avail) n = (int32_t)avail;
  if (n == 0) return 0;
  for (int32_t i = 0; i < n; ++i) {  // the launches may sit on different streams: wait for each
    (void)hipEventSynchronize(ts.ev1[(ts.count - n + i) % kTimingRing]);
    out[i] = timing_ms(ts, ts.count - n + i);
  }
  return n;
}

int mtgp_flatten_ex(const float* population, int32_t P, int32_t T, int32_t N, const MtgpNodeLibrary* lib,
                    const MtgpProgramSpec* specs, int32_t n_prog, int32_t L, MtgpInstr* prog_out, int32_t* len_out,
                    int32_t* nodes_out, int32_t* status_out, int32_t* jit_words_out, int32_t* jit_cost_out,
                    int32_t jit_mode, void* stream) {
  if (jit_mode != mtgp::kJitModeRegs && jit_mode != mtgp::kJitModeLds) return MTGP_ERR_ARG;
  if (!population || !lib || !specs || !prog_out || !len_out || !nodes_out || !status_out) return MTGP_ERR_ARG;
  if (P < 0 || T <= 0 || N <= 0 || N > MTGP_MAX_NODES || n_prog <= 0 || L <= 0) return MTGP_ERR_ARG;
  if (lib->n_funcs <= 0 || lib->n_funcs > MTGP_MAX_FUNCS) return MTGP_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(population) & 15u) != 0) return MTGP_ERR_ARG;  // 16-byte row loads
  if (P == 0) return MTGP_OK;
  hipStream_t s = (hipStream_t)stream;
  const long total = (long)P * n_prog;
  MtgpNodeLibrary libv = *lib;
  static const int lanes_env = [] {  // A/B knob (scripts/): MTGP_FLAT_LANES=8|16|32 at run time
    const char* e = getenv("MTGP_FLAT_LANES");
    const int v = e ? atoi(e) : MTGP_FLAT_LANES;
    return (v == 8 || v == 16 || v == 32) ? v : MTGP_FLAT_LANES;
  }();
  // one wave per program (k_flatten_wave, default) or one lane per program (k_flatten): A/B knob
  // MTGP_FLAT_MODE=lane at run time
  const char* fm = getenv("MTGP_FLAT_MODE");
  const bool wave_mode = !MTGP_AB_FLAT_LANE || !(fm && strcmp(fm, "lane") == 0);
  static const JitOpTable optab = jit_op_table();  // (host probe of jit_program, once per process)
  // trees of <= 64 rows: two programs per wave, one per 32-lane half (register-mode JIT sizing or
  // none; C3 flatten 75 -> see DESIGN.md "Per-step overhead kernels"); A/B knob MTGP_FLAT_HALVES=0,
  // read per call
  const char* fh = getenv("MTGP_FLAT_HALVES");  // (0 / 1 force; default: more programs than one round)
  const bool halves = (fh ? strcmp(fh, "0") != 0 : total > kResidentWaves) &&
                      (jit_mode == mtgp::kJitModeRegs || (!jit_words_out && !jit_cost_out));
  if (total > (long)UINT32_MAX) return MTGP_ERR_ARG;
  // node counts are summed with atomics into zeros, except by the wave kernel for few trees
  if ((!wave_mode || T > kFlatDirectTrees) && hipMemsetAsync(nodes_out, 0, (size_t)P * sizeof(int32_t), s) != hipSuccess)
    return MTGP_ERR_LAUNCH;
#if MTGP_AB_FLAT_LANE
#define MTGP_FLAT_ONE(NM, TP)                                                                                 \
  hipLaunchKernelGGL((k_flatten<NM, TP>), dim3((unsigned)((total + TP - 1) / TP)), dim3(TP), 0, s, population, P, \
                     T, N, libv, specs, n_prog, L, prog_out, len_out, nodes_out, status_out, jit_words_out,      \
                     jit_cost_out, jit_mode)
#else
#define MTGP_FLAT_ONE(NM, TP) (void)0
#endif
#define MTGP_FLAT_LAUNCH(NM)                                                                                \
  do {                                                                                                      \
    const int tp = NM * lanes_env > 2048 ? 2048 / NM : lanes_env; /* LDS: 16 B x NM x lanes <= 32 KB */   \
    if (wave_mode && NM == 64 && halves)                                                                    \
      hipLaunchKernelGGL((k_flatten_wave<64, kWave / 2>), dim3((unsigned)((total + 1) / 2)), dim3(kWave), 0, s, \
                         population, P, T, N, libv, specs, n_prog, L, prog_out, len_out, nodes_out, status_out, \
                         jit_words_out, jit_cost_out, jit_mode, optab);                                     \
    else if (wave_mode)                                                                                     \
      hipLaunchKernelGGL((k_flatten_wave<NM>), dim3((unsigned)total), dim3(kWave), 0, s, population, P, T, N, \
                         libv, specs, n_prog, L, prog_out, len_out, nodes_out, status_out, jit_words_out,  \
                         jit_cost_out, jit_mode, optab);                                                    \
    else if (tp >= 32) MTGP_FLAT_ONE(NM, 32);                                                               \
    else if (tp >= 16) MTGP_FLAT_ONE(NM, 16);                                                               \
    else MTGP_FLAT_ONE(NM, 8);                                                                              \
    hipLaunchKernelGGL(k_flatten_serial<NM>, dim3((unsigned)(total < 256 * 64 ? (total + 63) / 64 : 256)), \
                       dim3(64), 0, s, population, P, T, N, libv, specs, n_prog, L, prog_out, len_out,     \
                       status_out, jit_words_out, jit_cost_out, jit_mode);                                  \
  } while (0)
  if (N <= 64) MTGP_FLAT_LAUNCH(64);
  else if (N <= 128) MTGP_FLAT_LAUNCH(128);
  else MTGP_FLAT_LAUNCH(256);
#undef MTGP_FLAT_LAUNCH
#undef MTGP_FLAT_ONE
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_flatten(const float* population, int32_t P, int32_t T, int32_t N, const MtgpNodeLibrary* lib,
                 const MtgpProgramSpec* specs, int32_t n_prog, int32_t L, MtgpInstr* prog_out, int32_t* len_out,
                 int32_t* nodes_out, int32_t* status_out, void* stream) {
  return mtgp_flatten_ex(population, P, T, N, lib, specs, n_prog, L, prog_out, len_out, nodes_out, status_out,
                         nullptr, nullptr, mtgp::kJitModeRegs, stream);
}

int mtgp_flatten_tree_host(const float* tree, int32_t N, const MtgpNodeLibrary* lib, int32_t n_data,
                           uint64_t zero_mask, int32_t L, MtgpInstr* out, int32_t* stack_need) {
  if (!tree || !lib || !out || N <= 0 || N > MTGP_MAX_NODES || L <= 0) return MTGP_ERR_ARG;
  mtgp::RowInfo info[MTGP_MAX_NODES];
  int need = 0;
  const int n = mtgp::flatten_tree(tree, N, lib, n_data, zero_mask, out, L, info, &need);
  if (stack_need) *stack_need = need;
  return n;
}

int mtgp_schedule(const int32_t* plen, int32_t P, int32_t n_prog, const int32_t* weights, int32_t R,
                  int32_t* order_out, int32_t* scratch, void* stream) {
  if (!plen || !order_out || !scratch || P < 0 || n_prog <= 0 || n_prog > MTGP_MAX_PROGRAMS) return MTGP_ERR_ARG;
  if (R <= 0 || R > MTGP_MAX_ROLLOUTS) return MTGP_ERR_ARG;  // R: the lane set (or the rollout count)
  if (P == 0) return MTGP_OK;
  SchedW W;
  for (int j = 0; j < MTGP_MAX_PROGRAMS; ++j) W.w[j] = (j < n_prog) ? (weights ? weights[j] : 1) : 0;
  int Rp = 1;
  while (Rp < R) Rp <<= 1;
  const int G = Rp >= kWave ? 1 : kWave / Rp;
  hipStream_t s = (hipStream_t)stream;
  if ((long)P * n_prog <= kSchedFusedMax) {  // small populations: one block does it all
    const int vec4 = n_prog == 4 && (reinterpret_cast<uintptr_t>(plen) & 15u) == 0;  // (C3)
    if (P <= 1024 * kSchedRegP)
      hipLaunchKernelGGL(k_sched_fused<kSchedRegP>, dim3(1), dim3(1024), 0, s, plen, P, n_prog, W, G, order_out, vec4);
    else
      hipLaunchKernelGGL(k_sched_fused<0>, dim3(1), dim3(1024), 0, s, plen, P, n_prog, W, G, order_out, 0);
    return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
  }
  int32_t* hist = scratch;
  int32_t* offs = scratch + MTGP_SCHED_BINS;
  if (hipMemsetAsync(hist, 0, MTGP_SCHED_BINS * sizeof(int32_t), s) != hipSuccess) return MTGP_ERR_LAUNCH;
  const unsigned nb = (unsigned)((P + 255) / 256);
  hipLaunchKernelGGL(k_sched_hist, dim3(nb), dim3(256), 0, s, plen, P, n_prog, W, hist);
  hipLaunchKernelGGL(k_sched_scan, dim3(1), dim3(1024), 0, s, hist, offs);
  hipLaunchKernelGGL(k_sched_scatter, dim3(nb), dim3(256), 0, s, plen, P, n_prog, W, G, offs, order_out);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_eval_programs(const MtgpInstr* prog, const int32_t* plen, int32_t n_prog, int32_t L, int32_t P,
                       const float* data, int32_t M, int32_t n_data, float* out, void* stream) {
  if (!prog || !plen || !data || !out || P < 0 || n_prog <= 0 || L <= 0 || M < 0) return MTGP_ERR_ARG;
  if (n_data <= 0 || n_data > MTGP_MAX_DATA || (L & 3) != 0) return MTGP_ERR_ARG;
  if (P == 0 || M == 0) return MTGP_OK;
  const long items = (long)P * n_prog * ((M + 63) / 64);
  const size_t lds = (size_t)kWavesPerBlock * (n_data + kSMax) * kWave * sizeof(float);
  hipLaunchKernelGGL(k_eval_programs, dim3((unsigned)((items + kWavesPerBlock - 1) / kWavesPerBlock)),
                     dim3(kWave * kWavesPerBlock), lds, (hipStream_t)stream, prog, plen, n_prog, L, P, data, M,
                     n_data, out);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

int mtgp_eval_waves(int32_t P, int32_t R, int32_t lanes) {
  if (P < 0 || R <= 0 || R > MTGP_MAX_ROLLOUTS || lanes < 0) return MTGP_ERR_ARG;
  int Rp = 1;
  while (Rp < R) Rp <<= 1;
  if (lanes > 0) {
    if (lanes < R || (lanes & (lanes - 1)) != 0) return MTGP_ERR_ARG;
    Rp = lanes;
  }
  const long G = Rp >= kWave ? 1 : kWave / Rp, W = Rp > kWave ? Rp / kWave : 1;
  const long waves = (P + G - 1) / G * W;
  return waves > INT32_MAX / kWave ? MTGP_ERR_ARG : (int)waves;
}

int mtgp_eval_rk4(const MtgpModel* model, const MtgpInstr* prog, const int32_t* plen, int32_t n_prog, int32_t L,
                  const int32_t* nodes, int32_t P, const MtgpRollouts* rollouts, const MtgpOutputs* out,
                  void* stream) {
  return mtgp_eval_rk4_jit(model, prog, plen, n_prog, L, nodes, P, rollouts, out, nullptr, stream);
}

int mtgp_eval_rk4_jit(const MtgpModel* model, const MtgpInstr* prog, const int32_t* plen, int32_t n_prog,
                      int32_t L, const int32_t* nodes, int32_t P, const MtgpRollouts* rollouts,
                      const MtgpOutputs* out, const MtgpJitCode* jitc, void* stream) {
  if (!model || !prog || !plen || !nodes || !rollouts || !out || !out->fitness) return MTGP_ERR_ARG;
  if (P < 0 || n_prog <= 0 || L <= 0 || (L & 3) != 0) return MTGP_ERR_ARG;
  if (rollouts->R <= 0 || rollouts->R > MTGP_MAX_ROLLOUTS) return MTGP_ERR_ARG;
  const int set = rollouts->lanes > 0 ? rollouts->lanes : 0;
  if (set && (set < rollouts->R || (set & (set - 1)) != 0 || set > 2 * MTGP_MAX_ROLLOUTS)) return MTGP_ERR_ARG;
  int Rp = 1;
  while (Rp < rollouts->R) Rp <<= 1;
  if (set) Rp = set;
  if (Rp > kWave && !out->rollout_fitness) return MTGP_ERR_ARG;  // the mean is formed from it
  if ((int64_t)P * Rp > INT32_MAX) return MTGP_ERR_ARG;  // lane offsets are 32-bit
  if ((int64_t)P * n_prog * L * (int64_t)sizeof(MtgpInstr) > UINT32_MAX) return MTGP_ERR_ARG;  // 32-bit program offsets
  const bool dopri5 = model->solver == MTGP_SOLVER_DOPRI5;
  if (model->solver != MTGP_SOLVER_RK4 && model->solver != MTGP_SOLVER_EULER && !dopri5) return MTGP_ERR_ARG;
  if (dopri5) {  // adaptive: save points come from ts, steps from the controller
    if (model->model == MTGP_MODEL_SR && (model->n_var < 1 || model->n_var > MTGP_MAX_DATA)) return MTGP_ERR_ARG;
    if (model->n_save < 2 || model->max_steps <= 0 || !(model->h > 0.0f)) return MTGP_ERR_ARG;
    if (!(model->rtol >= 0.0f) || !(model->atol >= 0.0f)) return MTGP_ERR_ARG;
  } else {  // fixed step (ABI v18): diffrax ConstantStepSize from dt0 = h, save points from ts (mtgp_cstep.h)
    if (model->model == MTGP_MODEL_SR && (model->n_var < 1 || model->n_var > MTGP_MAX_DATA)) return MTGP_ERR_ARG;
    if (model->n_save < 2 || model->max_steps < 0 || !(model->h > 0.0f) || !(model->h < 3.0e38f)) return MTGP_ERR_ARG;
  }
  if (!rollouts->x0 || !rollouts->ts) return MTGP_ERR_ARG;
  if (rollouts->fit_kof && (model->model == MTGP_MODEL_SR || model->env != MTGP_ENV_ACROBOT)) return MTGP_ERR_ARG;
  // trajectory layout (ABI v20): lane-major rows only for the adaptive solve (traj_put_dp)
  if (out->traj_layout != MTGP_TRAJ_TIME_MAJOR &&
      (out->traj_layout != MTGP_TRAJ_LANE_MAJOR || model->solver != MTGP_SOLVER_DOPRI5))
    return MTGP_ERR_ARG;
  if (P == 0) return MTGP_OK;
  KArgs A;
  A.m = *model;
  A.prog = prog;
  A.plen = plen;
  A.n_prog = n_prog;
  A.L = L;
  A.nodes = nodes;
  A.P = P;
  A.ro = *rollouts;
  A.out = *out;
  const bool jit = jitc && jitc->code && jitc->offsets;
  A.jit_base = jit ? (uint64_t)(uintptr_t)jitc->code : 0;
  A.jit_off = jit ? jitc->offsets : nullptr;
  A.jit_info = jit ? jitc->info : nullptr;
  A.jit_cap = jit ? jitc->capacity : 0;
  A.chain_state = A.chain_save = A.chain_store = 0;
  A.dp_budget = 0;
  A.dp_pass = 0;
  A.dp_state = nullptr;
  A.dp_pending = nullptr;
  A.dp_lanes = 0;
  if (model->dp_budget > 0 && dopri5 && model->model != MTGP_MODEL_SR) {  // two launches (control models)
    if (!out->dp_state || !out->dp_pending) return MTGP_ERR_ARG;
    A.dp_budget = model->dp_budget;
    A.dp_state = out->dp_state;
    A.dp_pending = out->dp_pending;
  }
  A.chain_merge = 0;
  static std::atomic<uint32_t> launch_epoch{0};
  A.epoch = launch_epoch.fetch_add(1, std::memory_order_relaxed) + 1u;
  if (A.epoch == 0u) A.epoch = 1u;  // (a zero tag would match the table's initial contents)
  {  // MTGP_FAIR: 0 off, k >= 1 on with a lead margin of k - 1 steps (default 3: margin 2)
    const char* f = getenv("MTGP_FAIR");
    A.fair = f ? atoi(f) : 3;
    if (A.fair < 0 || A.fair > 1000) A.fair = 3;
    const char* fm = getenv("MTGP_FAIR_MODE");
    A.fair_mode = fm ? atoi(fm) : 0;
    const char* fd = getenv("MTGP_FAIR_DP");  // (waves resume into freed slots there: off by default)
    A.fair_dp = fd ? atoi(fd) : 0;
    if (A.fair_dp < 0 || A.fair_dp > 1000) A.fair_dp = 0;
  }
  if (jit && (jitc->chain.next | jitc->chain.cond | jitc->chain.store | jitc->chain.put) != 0u) {
    const MtgpJitChain want = jit_chain_for(*model, n_prog);  // must be the chain this model calls
    if (want.next != jitc->chain.next || want.cond != jitc->chain.cond || want.store != jitc->chain.store ||
        want.put != jitc->chain.put || (want.put != 0u && want.put_slot != jitc->chain.put_slot))
      return MTGP_ERR_ARG;
    A.chain_state = (want.next | want.cond) != 0u;
    A.chain_save = want.cond != 0u;
    A.chain_store = want.store != 0u;
    A.chain_merge = want.put != 0u;
  }
  // (the wide-state SR kernel keeps its data vector in LDS: its code is built in kJitModeLds)
  hipStream_t s = (hipStream_t)stream;
  const int G = Rp >= kWave ? 1 : kWave / Rp;  // individuals packed per wave
  const int Wset = Rp > kWave ? Rp / kWave : 1;  // waves per individual
  const long waves = ((long)P + G - 1) / G * Wset;
  if (waves * kWave > (long)UINT32_MAX) return MTGP_ERR_ARG;
  A.dp_lanes = (uint32_t)(waves * kWave);
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)), block(kWave * kWavesPerBlock);
  {  // fair share needs companions: at least two waves per SIMD (C2's 256 waves: 7 % slower with it)
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || waves < 2L * 4L * (long)cus)
      A.fair = 0;
    if (model->model == MTGP_MODEL_SR && model->n_var > 4) A.fair = 0;  // k_sr_wide: barrier-synced workgroups (C5: 1 % slower)
  }
  const bool traj = out->xs || out->ys || out->us || out->acts;
  if (traj && (long)P * rollouts->R * 4 > (long)INT32_MAX) return MTGP_ERR_ARG;  // store_row's 31-bit byte offsets
  const bool noise = rollouts->obs_keys != nullptr;
  if (noise && (!rollouts->obs_w || model->model == MTGP_MODEL_SR)) return MTGP_ERR_ARG;
  if (model->prng_impl != MTGP_PRNG_THREEFRY_ORIGINAL && model->prng_impl != MTGP_PRNG_THREEFRY_PARTITIONABLE)
    return MTGP_ERR_ARG;
  const int rc = [&]() -> int {
  if (model->model == MTGP_MODEL_DYNAMIC || model->model == MTGP_MODEL_STATIC) {
    switch (model->env) {
      case MTGP_ENV_ACROBOT:
        if (rollouts->fit_kof)  // the general cost mask: its own kernels (EnvAcrobotMask, TU 6)
          return launch_tu([&] { return mtgp_tu_launch_acrobot_mask(&A, model, rollouts, jit, noise, traj, grid.x, block.x, s); }, s);
        return launch_tu([&] { return mtgp_tu_launch_acrobot(&A, model, rollouts, jit, noise, traj, grid.x, block.x, s); }, s);
      case MTGP_ENV_HARMONIC_OSCILLATOR:
        return launch_tu([&] { return mtgp_tu_launch_harmonic(&A, model, rollouts, jit, noise, traj, grid.x, block.x, s); }, s);
      case MTGP_ENV_STIRRED_TANK_REACTOR:
        return launch_tu([&] { return mtgp_tu_launch_reactor(&A, model, rollouts, jit, noise, traj, grid.x, block.x, s); }, s);
      default: return MTGP_ERR_ARG;
    }
  } else if (model->model == MTGP_MODEL_SR) {
    if (!rollouts->ys_true) return MTGP_ERR_ARG;
    if (model->n_var > 4 && (model->n_var > MTGP_MAX_DATA || n_prog < model->prog_state + model->n_var))
      return MTGP_ERR_ARG;
    return launch_tu([&] { return mtgp_tu_launch_sr(&A, model, jit, traj, dopri5, (unsigned)G, (unsigned)Wset, grid.x, block.x, s); }, s);
  }
  return MTGP_ERR_ARG;
  }();
  if (rc != MTGP_OK || Wset == 1) return rc;
  hipLaunchKernelGGL(k_rollout_mean, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, out->rollout_fitness, P,
                     rollouts->R, model->max_fitness, model->parsimony, nodes, out->fitness);
  return hipGetLastError() == hipSuccess ? MTGP_OK : MTGP_ERR_LAUNCH;
}

}  // extern "C"
#endif  // MTGP_TU_MAIN
