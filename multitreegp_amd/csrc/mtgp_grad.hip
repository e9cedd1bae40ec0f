// mtgp_grad.hip -- forward-mode sensitivities of the SR fitness for coefficient optimisation.
//
// Reference: GeneticProgramming.optimise / epoch (gp.py:435-473) run
//   loss, grads = vmap(value_and_grad(partial_ff))(candidates[..., 3:], candidates[..., :3], data)
// i.e. reverse-mode through diffeqsolve (SR_evaluator.py:57-83, DirectAdjoint) of the evaluator's
// clipped mean MSE (SR_evaluator.py:30-45).  Here the derivative is taken in forward mode: the
// host (multitreegp_amd/coefficients.py) turns the coefficient rows to differentiate into
// variable rows reading data slots n_var .. n_var + K - 1, flattens that population with the
// ordinary flattener, and every lane of k_sr_grad integrates one (individual, parameter k,
// rollout) triple with dual numbers (value, d/dtheta_k).  The value half performs exactly the
// operations of k_sr (the fixed-step spec include/mtgp_cstep.h, same MSE order), so the loss equals the evaluator's
// fitness bit for bit; the tangent half is the chain rule of those same operations.
// k_grad_reduce then forms the per-individual loss and gradient with the evaluator's NaN/inf ->
// max_fitness replacement, the pairwise rollout sum of finish_group and jnp.clip's derivative.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mtgp.h"
#include "mtgp_f32math.h"
#include "mtgp_prng.h"
#include "mtgp_dual.h"
#include "mtgp_dopri5.h"
#include "mtgp_cstep.h"
#include "mtgp_jit_dual.h"

namespace {

constexpr float kInf = __builtin_huge_valf();

struct Dual {
  float v, d;
};

// d(x op y) with the value computed exactly as the interpreter's handler does
__device__ __forceinline__ Dual d_add(Dual a, Dual b) { return {a.v + b.v, a.d + b.d}; }
__device__ __forceinline__ Dual d_sub(Dual a, Dual b) { return {a.v - b.v, a.d - b.d}; }
__device__ __forceinline__ Dual d_mul(Dual a, Dual b) { return {a.v * b.v, a.d * b.v + a.v * b.d}; }
__device__ __forceinline__ Dual d_div(Dual a, Dual b) {
  const float q = a.v / b.v;
  return {q, (a.d - q * b.d) / b.v};
}
__device__ __forceinline__ Dual d_sin(Dual a) { return {mtgp_sinf(a.v), mtgp_cosf(a.v) * a.d}; }
__device__ __forceinline__ Dual d_cos(Dual a) { return {mtgp_cosf(a.v), -mtgp_sinf(a.v) * a.d}; }

// the round-3 unary operators: include/mtgp_dual.h's rules (shared with the oracle)
__device__ __forceinline__ Dual d_unary(int fn, Dual a) {
  const MtgpDual r = mtgp_dl_unary(fn, mtgp_dl(a.v, a.d));
  return {r.v, r.d};
}

// family member: 0 ADD, 1 SUB (acc - o), 2 RSUB (o - acc), 3 MUL, 4 DIV (acc / o), 5 RDIV (o / acc)
__device__ __forceinline__ Dual d_fam(int f, Dual acc, Dual o) {
  switch (f) {
    case 0: return d_add(acc, o);
    case 1: return d_sub(acc, o);
    case 2: return d_sub(o, acc);
    case 3: return d_mul(acc, o);
    case 4: return d_div(acc, o);
    default: return d_div(o, acc);
  }
}

struct GradArgs {
  MtgpModel m;
  const MtgpInstr* prog;
  int n_prog, L, P, K;
  const float* theta;     // [P, K]
  const int32_t* nparam;  // [P]
  MtgpRollouts ro;
  float* part;            // [P, K, R, 2] per-rollout (F, dF/dtheta_k)
  float* hist;            // [S, P * K * R, 2]: cost prefixes of the general Acrobot mask (fit_kof), else null
  float* loss;            // [P]
  float* grad;            // [P, K]
  // dual-number program code (mtgp_jit_dual.h; mtgp_ctl_grad_jit), or null: interpret
  const uint8_t* jit_code;
  const uint32_t* jit_offs;  // [P * n_prog + 1] byte offsets of the units
  const int32_t* jit_info;   // [2]: [0] < 0 some program untranslatable, [1] bytes the code needs
  uint64_t jit_bytes;
};

// The code of this launch is usable: every program translated and the buffer large enough
// (device-side check, no host round trip; otherwise the interpreter runs)
__device__ __forceinline__ bool dual_jit_ok(const GradArgs& A) {
  if (!A.jit_code) return false;
  const int32_t e = __builtin_amdgcn_readfirstlane(A.jit_info[0]), b = __builtin_amdgcn_readfirstlane(A.jit_info[1]);
  return e == 0 && b > 0 && (uint64_t)(uint32_t)b <= A.jit_bytes;
}
// code address of program j of individual p (wave-uniform)
__device__ __forceinline__ uint64_t dual_unit(const GradArgs& A, int p, int j) {
  const uint32_t off = A.jit_offs[(size_t)p * A.n_prog + j];
  return (uint64_t)(uintptr_t)A.jit_code + (uint32_t)__builtin_amdgcn_readfirstlane((int)off);
}
// Call one dual unit: data values v0-v7, tangents v48-v55, the lane's coefficient index in v25;
// result (value, tangent) in (v8, v56).  Clobbers: mtgp_jit_dual.h's register ABI.
__device__ __forceinline__ Dual dual_call(uint64_t addr_, const float (&dv)[8], const float (&dd)[8], int kk) {
  const uint64_t addr = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)addr_) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(addr_ >> 32)) << 32;
  float v, d;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "={v8}"(v), "={v56}"(d)
               : [tgt] "s"(addr), "{v0}"(dv[0]), "{v1}"(dv[1]), "{v2}"(dv[2]), "{v3}"(dv[3]), "{v4}"(dv[4]),
                 "{v5}"(dv[5]), "{v6}"(dv[6]), "{v7}"(dv[7]), "{v48}"(dd[0]), "{v49}"(dd[1]), "{v50}"(dd[2]),
                 "{v51}"(dd[3]), "{v52}"(dd[4]), "{v53}"(dd[5]), "{v54}"(dd[6]), "{v55}"(dd[7]), "{v25}"(kk)
               : "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v26", "v27", "v28", "v29", "v57", "v58", "v59", "v60", "v61", "v62",
                 "v63", "v64", "s30", "s31", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42",
                 "s43", "s44", "s45", "vcc", "scc", "memory");
  return {v, d};
}

// Lane (individual p, parameter k, rollout r).  Each individual owns K * R lanes rounded up to
// whole waves, so every wave belongs to ONE individual: its programs and coefficients are
// wave-uniform (p is read from the first lane), the dual interpreter fetches instructions with
// scalar loads and branches on them with scalar branches (round 4: with p per lane both were
// vector operations, 22 us per RK4 stage); the padding lanes (k >= K) return at once.
__host__ __device__ __forceinline__ long grad_lanes_per(int K, int R) { return ((long)K * R + 63) / 64 * 64; }
__device__ __forceinline__ bool grad_lane(const GradArgs& A, int& p, int& k, int& r, size_t& slot) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int R = A.ro.R;
  const long LP = grad_lanes_per(A.K, R);
  const long pl = gid / LP;
  if (pl >= A.P) return false;
  const int t = (int)(gid - pl * LP);
  k = t / R;
  r = t - k * R;
  if (k >= A.K) return false;
  p = __builtin_amdgcn_readfirstlane((int)pl);  // (wave-uniform by construction)
  slot = ((size_t)p * A.K + k) * R + r;
  return true;
}

// Data slot s (byte offset s * MTGP_SLOT_BYTES in the program words): the stage state for
// s < nv, parameter theta[s - nv] otherwise (tangent 1 for the lane's own parameter).
template <int NV>
__device__ __forceinline__ Dual slot_val(uint32_t off, const float* sv, const float* sd, int nv, const float* th,
                                         int kk) {
  const int s = (int)(off / MTGP_SLOT_BYTES);
  if (s < nv) {
    if constexpr (NV <= 4) {  // keep the small state in registers: select, not a dynamic index
      float v = 0.0f, d = 0.0f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        v = (i == s) ? sv[i] : v;
        d = (i == s) ? sd[i] : d;
      }
      return {v, d};
    } else {
      return {sv[s], sd[s]};
    }
  }
  return {th[s - nv], (s - nv == kk) ? 1.0f : 0.0f};
}

// One program (mtgp.h format, every opcode incl. the fused forms) in dual numbers; V(off) reads
// data slot off / MTGP_SLOT_BYTES as a Dual.
// The operand stack of a lane: a private array (kernels with registers to spare: the compiler keeps
// it in VGPRs) or, in the register-heavy kernels, a column of the block's LDS (a private array
// would live in scratch memory there: a scratch round trip per push / pop, round 4).
struct PrivStack {
  Dual s[MTGP_STACK_MAX];
  __device__ Dual& at(int i) { return s[i]; }
};
constexpr int kGradBlock = 256;  // threads per block of the gradient kernels
struct LdsStack {
  Dual* col;  // &lds[0][threadIdx.x] of a [MTGP_STACK_MAX][kGradBlock] array
  __device__ Dual& at(int i) { return col[i * kGradBlock]; }
};

template <class Src, class Stk = PrivStack>
__device__ __forceinline__ Dual run_dual_src(const MtgpInstr* code, Src V, Stk stk = Stk()) {
  Dual acc = {0.0f, 0.0f};
  int sp = 0;
  // the next instruction's (scalar) load is issued before this one is dispatched: one load
  // latency per program instead of one per instruction (a read one past the END stays inside the
  // program slot or the flattener's spare block)
  MtgpInstr nxt = code[0];
  for (int pc = 0;; ++pc) {
    const MtgpInstr cur = nxt;
    nxt = code[pc + 1];
    const uint32_t w = cur.op, op = w >> MTGP_OP_SHIFT, ax = w & 0xffffffu;
    const float imm = cur.imm;
    const uint32_t ib = __float_as_uint(imm);
    const Dual C = {imm, 0.0f};
    auto push = [&]() { stk.at(sp < MTGP_STACK_MAX ? sp : MTGP_STACK_MAX - 1) = acc; ++sp; };
    auto pop = [&]() { --sp; return stk.at(sp < 0 ? 0 : (sp < MTGP_STACK_MAX ? sp : MTGP_STACK_MAX - 1)); };
    switch (op) {
      case MTGP_OP_END: return acc;
      case MTGP_OP_LDC: acc = C; break;
      case MTGP_OP_LDCP: push(); acc = C; break;
      case MTGP_OP_LDV: acc = V(ib); break;
      case MTGP_OP_LDVP: push(); acc = V(ib); break;
      case MTGP_OP_ADDC: acc = d_fam(0, acc, C); break;
      case MTGP_OP_SUBC: acc = d_fam(1, acc, C); break;
      case MTGP_OP_RSUBC: acc = d_fam(2, acc, C); break;
      case MTGP_OP_MULC: acc = d_fam(3, acc, C); break;
      case MTGP_OP_DIVC: acc = d_fam(4, acc, C); break;
      case MTGP_OP_RDIVC: acc = d_fam(5, acc, C); break;
      case MTGP_OP_ADDV: acc = d_fam(0, acc, V(ib)); break;
      case MTGP_OP_SUBV: acc = d_fam(1, acc, V(ib)); break;
      case MTGP_OP_RSUBV: acc = d_fam(2, acc, V(ib)); break;
      case MTGP_OP_MULV: acc = d_fam(3, acc, V(ib)); break;
      case MTGP_OP_DIVV: acc = d_fam(4, acc, V(ib)); break;
      case MTGP_OP_RDIVV: acc = d_fam(5, acc, V(ib)); break;
      case MTGP_OP_ADDS: { const Dual s = pop(); acc = d_add(acc, s); break; }
      case MTGP_OP_SUBS: { const Dual s = pop(); acc = d_sub(acc, s); break; }
      case MTGP_OP_RSUBS: { const Dual s = pop(); acc = d_sub(s, acc); break; }
      case MTGP_OP_MULS: { const Dual s = pop(); acc = d_mul(acc, s); break; }
      case MTGP_OP_DIVS: { const Dual s = pop(); acc = d_div(acc, s); break; }
      case MTGP_OP_RDIVS: { const Dual s = pop(); acc = d_div(s, acc); break; }
      case MTGP_OP_SIN: acc = d_sin(acc); break;
      case MTGP_OP_COS: acc = d_cos(acc); break;
      case MTGP_OP_SINV: acc = d_sin(V(ib)); break;
      case MTGP_OP_COSV: acc = d_cos(V(ib)); break;
      case MTGP_OP_SINVP: push(); acc = d_sin(V(ib)); break;
      case MTGP_OP_COSVP: push(); acc = d_cos(V(ib)); break;
      case MTGP_OP_EXP: acc = d_unary(MTGP_FN_EXP, acc); break;
      case MTGP_OP_LOG: acc = d_unary(MTGP_FN_LOG, acc); break;
      case MTGP_OP_SQRT: acc = d_unary(MTGP_FN_SQRT, acc); break;
      case MTGP_OP_TANH: acc = d_unary(MTGP_FN_TANH, acc); break;
      case MTGP_OP_ABS: acc = d_unary(MTGP_FN_ABS, acc); break;
      // VC_f: acc = f(v[aux], imm); VCP: push first
      case MTGP_OP_VC_ADD: acc = d_fam(0, V(ax), C); break;
      case MTGP_OP_VC_SUB: acc = d_fam(1, V(ax), C); break;
      case MTGP_OP_VC_RSUB: acc = d_fam(2, V(ax), C); break;
      case MTGP_OP_VC_MUL: acc = d_fam(3, V(ax), C); break;
      case MTGP_OP_VC_DIV: acc = d_fam(4, V(ax), C); break;
      case MTGP_OP_VC_RDIV: acc = d_fam(5, V(ax), C); break;
      case MTGP_OP_VCP_ADD: push(); acc = d_fam(0, V(ax), C); break;
      case MTGP_OP_VCP_SUB: push(); acc = d_fam(1, V(ax), C); break;
      case MTGP_OP_VCP_RSUB: push(); acc = d_fam(2, V(ax), C); break;
      case MTGP_OP_VCP_MUL: push(); acc = d_fam(3, V(ax), C); break;
      case MTGP_OP_VCP_DIV: push(); acc = d_fam(4, V(ax), C); break;
      case MTGP_OP_VCP_RDIV: push(); acc = d_fam(5, V(ax), C); break;
      // VV_f: acc = f(v[imm], v[aux]); VVP: push first
      case MTGP_OP_VV_ADD: acc = d_add(V(ib), V(ax)); break;
      case MTGP_OP_VV_SUB: acc = d_sub(V(ib), V(ax)); break;
      case MTGP_OP_VV_MUL: acc = d_mul(V(ib), V(ax)); break;
      case MTGP_OP_VV_DIV: acc = d_div(V(ib), V(ax)); break;
      case MTGP_OP_VVP_ADD: push(); acc = d_add(V(ib), V(ax)); break;
      case MTGP_OP_VVP_SUB: push(); acc = d_sub(V(ib), V(ax)); break;
      case MTGP_OP_VVP_MUL: push(); acc = d_mul(V(ib), V(ax)); break;
      case MTGP_OP_VVP_DIV: push(); acc = d_div(V(ib), V(ax)); break;
      default: return acc;  // unknown word: the flattener never emits one
    }
  }
}

template <int NV, class Stk = PrivStack>
__device__ Dual run_dual(const MtgpInstr* code, const float* sv, const float* sd, int nv, const float* th, int kk,
                         Stk stk = Stk()) {
  return run_dual_src(code, [&](uint32_t off) { return slot_val<NV>(off, sv, sd, nv, th, kk); }, stk);
}

// One (individual p, parameter k, rollout r) per lane; k_sr's integration in dual numbers.
template <int NV>
__global__ void __launch_bounds__(256) k_sr_grad(GradArgs A) {
  const int R = A.ro.R;
  int p, k, r;
  size_t slot;
  if (!grad_lane(A, p, k, r, slot)) return;
  float* out = A.part + slot * 2;
  const int np = A.nparam[p];
  if (k > 0 && k >= np) {  // unused parameter slot of this individual
    out[0] = 0.0f;
    out[1] = 0.0f;
    return;
  }
  const int kk = k < np ? k : -1;
  const bool use_jit = NV <= 4 && dual_jit_ok(A);  // the programs as dual-number code (mtgp_jit_dual.h)
  if (use_jit) asm volatile("s_icache_inv");  // the code was written by this call's emit kernel
  const int nv = A.m.n_var;
  const float* th = A.theta + (size_t)p * A.K;
  const MtgpInstr* progs = A.prog + ((size_t)p * A.n_prog + A.m.prog_state) * A.L;
  const int S = A.m.n_save;
  const float* ts = A.ro.ts;
  const bool euler = A.m.solver == MTGP_SOLVER_EULER;
  const int n_stages = euler ? 1 : 4;
  float x[NV], dx[NV], kx[NV], dkx[NV], fx0[NV], dfx0[NV], ax[NV], dax[NV], sv[NV], sd[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    x[i] = i < nv ? A.ro.x0[(size_t)r * nv + i] : 0.0f;
    dx[i] = kx[i] = dkx[i] = fx0[i] = dfx0[i] = ax[i] = dax[i] = 0.0f;
  }
  auto bad = [&](const float* v) {
    bool b = false;
#pragma unroll
    for (int i = 0; i < NV; ++i) b = b || (i < nv && !mtgp_isfinite(v[i]));
    return b;
  };
  bool prev_ok = !bad(x);
  float tot = 0.0f, dtot = 0.0f;
  // the fixed-step grid of include/mtgp_cstep.h (uniform: ts is shared), saves by the dense output
  const float t_end = ts[S - 1], dt0 = A.m.h;
  float t = ts[0], tn = mtgp_cs_first_end(t, dt0, t_end);
  int steps = 0, ks = 0;
  while (t < t_end && mtgp_cs_advancing(steps, t, tn) && (A.m.max_steps <= 0 || steps < A.m.max_steps)) {
    const float dt = tn - t;
    float zv[NV], zd[NV];  // the zero tableau entries' terms, value and tangent (mtgp_cstep.h)
#pragma unroll 1
    for (int stage = 0; stage < n_stages; ++stage) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        sv[i] = stage == 0 ? x[i] : mtgp_rk4_in(stage, x[i], kx[i], zv[i], dt);
        sd[i] = stage == 0 ? dx[i] : mtgp_rk4_in(stage, dx[i], dkx[i], zd[i], dt);
        if (stage == 1 || stage == 2) {
          zv[i] = mtgp_rk4_zero(stage, zv[i], kx[i]);
          zd[i] = mtgp_rk4_zero(stage, zd[i], dkx[i]);
        }
      }
      if constexpr (NV <= 4) {  // one program site: the dual-number code (mtgp_jit_dual.h) or the interpreter
#pragma unroll 1
        for (int i = 0; i < nv; ++i) {
          Dual o;
          if (use_jit) {
            float dv8[8], dd8[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              dv8[c] = c < NV ? sv[c < NV ? c : 0] : 0.0f;
              dd8[c] = c < NV ? sd[c < NV ? c : 0] : 0.0f;
            }
            o = dual_call(dual_unit(A, p, A.m.prog_state + i), dv8, dd8, kk);
          } else {
            o = run_dual<NV>(progs + (size_t)i * A.L, sv, sd, nv, th, kk);
          }
#pragma unroll
          for (int c = 0; c < NV; ++c)
            if (c == i) {
              kx[c] = o.v;
              dkx[c] = o.d;
            }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          if (i >= nv) continue;
          const Dual o = run_dual<NV>(progs + (size_t)i * A.L, sv, sd, nv, th, kk);
          kx[i] = o.v;
          dkx[i] = o.d;
        }
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (stage == 0) {
          fx0[i] = kx[i];
          dfx0[i] = dkx[i];
        }
        ax[i] = mtgp_rk4_acc(stage, ax[i], kx[i]);
        dax[i] = mtgp_rk4_acc(stage, dax[i], dkx[i]);
      }
    }
    float x1[NV], dx1[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      x1[i] = euler ? x[i] + fx0[i] * dt : mtgp_rk4_out(x[i], ax[i], dt);
      dx1[i] = euler ? dx[i] + dfx0[i] * dt : mtgp_rk4_out(dx[i], dax[i], dt);
    }
    while (ks < S && ts[ks] <= tn) {  // MSE term of each save point (SR_evaluator.py:24) by the dense output
      const float tq = mtgp_cs_rescale(t, ts[ks], tn);
      float sq = 0.0f, dsq = 0.0f;
#pragma unroll
      for (int d = 0; d < NV; ++d) {
        if (d >= nv) continue;
        const float xv = euler ? mtgp_cs_linear(x[d], x1[d], tq) : mtgp_cs_hermite(x[d], x1[d], fx0[d] * dt, kx[d] * dt, tq);
        const float xd = euler ? mtgp_cs_linear(dx[d], dx1[d], tq)
                               : mtgp_cs_hermite(dx[d], dx1[d], dfx0[d] * dt, dkx[d] * dt, tq);
        const float e = xv - A.ro.ys_true[((size_t)ks * nv + d) * R + r];
        const float de = xd * (2.0f * e);  // jnp.square's JVP: g * (2 x)
        sq = (d == 0) ? e * e : sq + e * e;
        dsq = (d == 0) ? de : dsq + de;
      }
      tot = tot + sq;
      dtot = dtot + dsq;
      ++ks;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      x[i] = x1[i];
      dx[i] = dx1[i];
    }
    ++steps;
    t = tn;
    tn = mtgp_cs_next_end(t, dt0, t_end);
    const bool ok = !bad(x);
    if (prev_ok && !ok) break;  // the NaN event (sr.py:93-94)
    prev_ok = ok;
  }
  if (ks < S) tot = mtgp_isfinite(tot) ? kInf : tot;  // later save points are +inf
  out[0] = tot / (float)S;
  out[1] = dtot / (float)S;
}

// Dopri5 tableau rows read with a run-time stage index (wave-uniform: scalar loads)
__constant__ float kDpA[7][6] = MTGP_DP_TABLE_A;
__constant__ float kDpE[7] = MTGP_DP_TABLE_E;
__constant__ float kDpCM[7] = MTGP_DP_TABLE_CMID;

// k_sr_grad for the adaptive solve (SR_evaluator.py:76-79 with Dopri5 + PIDController): k_sr_dopri5's
// integration (include/mtgp_dopri5.h) in dual numbers, the step sizes, accept / reject decisions and
// the event held at their primal values (oracle sr_rollout_dual_dp: the derivative of the discrete
// solution along the step sequence the solve took).  The value half is the evaluator's MSE of the
// saved points bit for bit.  Lanes run independently (no wave-uniform program calls: the grad
// launch is small, one lane per (individual, parameter, rollout)).
template <int NV>
__global__ void __launch_bounds__(kGradBlock) k_sr_grad_dp(GradArgs A) {
  __shared__ Dual s_stk[MTGP_STACK_MAX][kGradBlock];
  const LdsStack stk{&s_stk[0][threadIdx.x]};
  const int R = A.ro.R;
  int p, k, r;
  size_t slot;
  if (!grad_lane(A, p, k, r, slot)) return;
  float* out = A.part + slot * 2;
  const int np = A.nparam[p];
  if (k > 0 && k >= np) {  // unused parameter slot of this individual
    out[0] = 0.0f;
    out[1] = 0.0f;
    return;
  }
  const int kk = k < np ? k : -1;
  const bool use_jit = NV <= 4 && dual_jit_ok(A);  // the programs as dual-number code (mtgp_jit_dual.h)
  if (use_jit) asm volatile("s_icache_inv");  // the code was written by this call's emit kernel
  const int nv = A.m.n_var;
  const float* th = A.theta + (size_t)p * A.K;
  const MtgpInstr* progs = A.prog + ((size_t)p * A.n_prog + A.m.prog_state) * A.L;
  const int S = A.m.n_save, max_steps = A.m.max_steps;
  const float rtol = A.m.rtol, atol = A.m.atol, dtmin = A.m.dtmin, dtmax = A.m.dtmax;
  const float* __restrict__ ts = A.ro.ts;
  const float t_end = ts[S - 1];
  float tot = 0.0f, dtot = 0.0f;
  int ks = 1;
  const MtgpDpPid pid = A.m.pid_custom ? MtgpDpPid{A.m.pid_c1, A.m.pid_c2, A.m.pid_c3, A.m.pid_safety,
                                                   A.m.pid_factormin, A.m.pid_factormax}
                                       : MtgpDpPid MTGP_DP_PID_DEFAULT;
  MtgpDpCtl ctl{1.0f, 1.0f, 0};
  const int force_dtmin = !A.m.no_force_dtmin;
  if constexpr (NV <= 4) {
    // small states: k_ctl_grad's register form -- compile-time component indices, the tableau sums
    // accumulated as the stages arrive (each sum's ascending-j order of mtgp_dp_term), one rhs site
    float yv[NV], yd[NV], sv[NV], sd[NV], f0v[NV], f0d[NV], fcv[NV], fcd[NV];
    float acv[6][NV], acd[6][NV], aev[NV], amv[NV], amd[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      yv[i] = i < nv ? A.ro.x0[(size_t)r * nv + i] : 0.0f;
      yd[i] = 0.0f;
    }
    auto bad = [&]() {
      bool b = false;
#pragma unroll
      for (int i = 0; i < NV; ++i) b = b || (i < nv && !mtgp_isfinite(yv[i]));
      return b;
    };
    auto rhs = [&](const float (&xv)[NV], const float (&xd)[NV]) {
#pragma unroll 1
      for (int i = 0; i < nv; ++i) {
        Dual o;
        if (use_jit) {
          float dv8[8], dd8[8];
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            dv8[c] = c < NV ? xv[c < NV ? c : 0] : 0.0f;
            dd8[c] = c < NV ? xd[c < NV ? c : 0] : 0.0f;
          }
          o = dual_call(dual_unit(A, p, A.m.prog_state + i), dv8, dd8, kk);
        } else {
          o = run_dual<NV>(progs + (size_t)i * A.L, xv, xd, nv, th, kk, stk);
        }
#pragma unroll
        for (int c = 0; c < NV; ++c)
          if (c == i) {
            fcv[c] = o.v;
            fcd[c] = o.d;
          }
      }
    };
    auto mse = [&](int q, const float (&xv)[NV], const float (&xd)[NV]) {  // SR_evaluator.py:24
      float sq = 0.0f, dsq = 0.0f;
#pragma unroll
      for (int d = 0; d < NV; ++d) {
        if (d >= nv) continue;
        const float e = xv[d] - A.ro.ys_true[((size_t)q * nv + d) * R + r];
        const float de = xd[d] * (2.0f * e);
        sq = (d == 0) ? e * e : sq + e * e;
        dsq = (d == 0) ? de : dsq + de;
      }
      tot = tot + sq;
      dtot = dtot + dsq;
    };
    auto contrib = [&](int j) __attribute__((always_inline)) {  // stage j's f = (fcv, fcd)
      const bool first = j == 0;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        if (q + 1 <= j) continue;
        const float w = kDpA[q + 1][j];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          acv[q][i] = mtgp_dp_term(acv[q][i], w, fcv[i], first);
          acd[q][i] = mtgp_dp_term(acd[q][i], w, fcd[i], first);
        }
      }
      const float we = kDpE[j], wm = kDpCM[j];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        aev[i] = mtgp_dp_term(aev[i], we, fcv[i], first);
        amv[i] = mtgp_dp_term(amv[i], wm, fcv[i], first);
        amd[i] = mtgp_dp_term(amd[i], wm, fcd[i], first);
      }
    };
    mse(0, yv, yd);
    int steps = 0;
    float t = ts[0];
    float tnext = t + A.m.h;
    tnext = tnext > t_end ? t_end : tnext;
    bool prev_ok = !bad(), have_f0 = false;
    while (t < t_end && steps < max_steps) {
      const float h = tnext - t;
      if (have_f0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          fcv[i] = f0v[i];
          fcd[i] = f0d[i];
        }
        contrib(0);
      }
#pragma unroll 1
      for (int st = have_f0 ? 1 : 0; st <= 6; ++st) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          float av = acv[0][i], ad = acd[0][i];
#pragma unroll
          for (int q = 1; q < 6; ++q) {
            av = (st == q + 1) ? acv[q][i] : av;
            ad = (st == q + 1) ? acd[q][i] : ad;
          }
          sv[i] = st == 0 ? yv[i] : MTGP_FMAF(h, av, yv[i]);
          sd[i] = st == 0 ? yd[i] : MTGP_FMAF(h, ad, yd[i]);
        }
        rhs(sv, sd);
        if (st == 0) {
#pragma unroll
          for (int i = 0; i < NV; ++i) {
            f0v[i] = fcv[i];
            f0d[i] = fcd[i];
          }
          have_f0 = true;
        }
        contrib(st);
      }
      // sv, sd = y1 (stage 6's input); fcv, fcd = f_6
      float msum = 0.0f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (i >= nv) continue;
        const float sc = mtgp_dp_scaled(h * aev[i], yv[i], sv[i], rtol, atol);
        msum = (i == 0) ? sc * sc : msum + sc * sc;
      }
      const float ms = msum / (float)nv;
      int keep, fail;
      const float dt = mtgp_dp_control(ms, h, dtmin, dtmax, force_dtmin, &pid, &ctl, &keep, &fail);
      ++steps;
      bool done = fail != 0;
      if (keep) {
        const float t1 = tnext;
        while (ks < S && ts[ks] <= t1) {  // SaveAt(ts) by the dense output at the primal theta
          const float thk = (ts[ks] - t) / h;
          float qv[NV], qd[NV];
#pragma unroll
          for (int i = 0; i < NV; ++i) {
            const float ymid = MTGP_FMAF(h, amv[i], yv[i]), dymid = MTGP_FMAF(h, amd[i], yd[i]);
            qv[i] = mtgp_dp_interp(yv[i], sv[i], ymid, h * f0v[i], h * fcv[i], thk);
            qd[i] = mtgp_dp_interp(yd[i], sd[i], dymid, h * f0d[i], h * fcd[i], thk);
          }
          mse(ks, qv, qd);
          ++ks;
        }
        t = t1;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          yv[i] = sv[i];
          yd[i] = sd[i];
          f0v[i] = fcv[i];  // FSAL
          f0d[i] = fcd[i];
        }
        const bool ok = !bad();
        if (prev_ok && !ok) done = true;  // the NaN event (sr.py:93-94)
        prev_ok = ok;
      }
      if (done) break;
      tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
  } else {
    constexpr float TA[7][6] = MTGP_DP_TABLE_A;
    constexpr float E[7] = MTGP_DP_TABLE_E;
    constexpr float CM[7] = MTGP_DP_TABLE_CMID;
    float yv[NV], yd[NV], y1v[NV], y1d[NV], fv[7][NV], fd[7][NV], sv[NV], sd[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      yv[i] = i < nv ? A.ro.x0[(size_t)r * nv + i] : 0.0f;
      yd[i] = 0.0f;
    }
    auto bad = [&]() {
      bool b = false;
#pragma unroll
      for (int i = 0; i < NV; ++i) b = b || (i < nv && !mtgp_isfinite(yv[i]));
      return b;
    };
    auto rhs = [&](const float* xv, const float* xd, float* ov, float* od) {
      for (int i = 0; i < nv; ++i) {
        const Dual o = run_dual<NV>(progs + (size_t)i * A.L, xv, xd, nv, th, kk, stk);
        ov[i] = o.v;
        od[i] = o.d;
      }
    };
    auto mse = [&](int ks, const float* xv, const float* xd) {  // SR_evaluator.py:24, save point ks
      float sq = 0.0f, dsq = 0.0f;
      for (int d = 0; d < nv; ++d) {
        const float e = xv[d] - A.ro.ys_true[((size_t)ks * nv + d) * R + r];
        const float de = xd[d] * (2.0f * e);
        sq = (d == 0) ? e * e : sq + e * e;
        dsq = (d == 0) ? de : dsq + de;
      }
      tot = tot + sq;
      dtot = dtot + dsq;
    };
    mse(0, yv, yd);
    int steps = 0;
    float t = ts[0];
    float tnext = t + A.m.h;
    tnext = tnext > t_end ? t_end : tnext;
    bool prev_ok = !bad();
    rhs(yv, yd, fv[0], fd[0]);
    while (t < t_end && steps < max_steps) {
      const float h = tnext - t;
      for (int st = 1; st <= 6; ++st) {
        for (int i = 0; i < nv; ++i) {
          float acc = 0.0f, dacc = 0.0f;
          for (int j = 0; j < st; ++j) {
            acc = mtgp_dp_term(acc, TA[st][j], fv[j][i], j == 0);
            dacc = mtgp_dp_term(dacc, TA[st][j], fd[j][i], j == 0);
          }
          sv[i] = MTGP_FMAF(h, acc, yv[i]);
          sd[i] = MTGP_FMAF(h, dacc, yd[i]);
          if (st == 6) { y1v[i] = sv[i]; y1d[i] = sd[i]; }
        }
        rhs(sv, sd, fv[st], fd[st]);
      }
      float msum = 0.0f;
      for (int i = 0; i < nv; ++i) {
        float acc = 0.0f;
        for (int j = 0; j < 7; ++j) acc = mtgp_dp_term(acc, E[j], fv[j][i], j == 0);
        const float sc = mtgp_dp_scaled(h * acc, yv[i], y1v[i], rtol, atol);
        msum = (i == 0) ? sc * sc : msum + sc * sc;
      }
      const float ms = msum / (float)nv;
      int keep, fail;
      const float dt = mtgp_dp_control(ms, h, dtmin, dtmax, force_dtmin, &pid, &ctl, &keep, &fail);
      ++steps;
      bool done = fail != 0;
      if (keep) {
        const float t1 = tnext;
        while (ks < S && ts[ks] <= t1) {  // SaveAt(ts) by the dense output at the primal theta
          const float thk = (ts[ks] - t) / h;
          for (int i = 0; i < nv; ++i) {
            float acc = 0.0f, dacc = 0.0f;
            for (int j = 0; j < 7; ++j) {
              acc = mtgp_dp_term(acc, CM[j], fv[j][i], j == 0);
              dacc = mtgp_dp_term(dacc, CM[j], fd[j][i], j == 0);
            }
            const float ymid = MTGP_FMAF(h, acc, yv[i]), dymid = MTGP_FMAF(h, dacc, yd[i]);
            sv[i] = mtgp_dp_interp(yv[i], y1v[i], ymid, h * fv[0][i], h * fv[6][i], thk);
            sd[i] = mtgp_dp_interp(yd[i], y1d[i], dymid, h * fd[0][i], h * fd[6][i], thk);
          }
          mse(ks, sv, sd);
          ++ks;
        }
        t = t1;
        for (int i = 0; i < nv; ++i) {
          yv[i] = y1v[i];
          yd[i] = y1d[i];
          fv[0][i] = fv[6][i];  // FSAL
          fd[0][i] = fd[6][i];
        }
        const bool ok = !bad();
        if (prev_ok && !ok) done = true;  // the NaN event (sr.py:93-94)
        prev_ok = ok;
      }
      if (done) break;
      tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
  }
  // unsaved points are +inf: the squared error is +inf (NaN stays NaN)
  if (ks < S && mtgp_isfinite(tot)) tot = kInf;
  out[0] = tot / (float)S;
  out[1] = dtot / (float)S;
}

// One (individual, parameter) per thread: NaN/inf -> max_fitness (derivative 0), pairwise sum
// over rollouts in finish_group's order, mean, jnp.clip(., 0, max_fitness) with JAX's derivative
// of max/min (1 inside, 1/2 on a tie, 0 outside).
__global__ void __launch_bounds__(256) k_grad_reduce(GradArgs A) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)A.P * A.K) return;
  const int p = (int)(gid / A.K), k = (int)(gid % A.K);
  const int R = A.ro.R;
  int Rp = 1;
  while (Rp < R) Rp <<= 1;
  const float mx = A.m.max_fitness;
  float v[64], dv[64];
  for (int r = 0; r < Rp; ++r) {
    float f = 0.0f, df = 0.0f;
    if (r < R) {
      const float* q = A.part + (((size_t)p * A.K + k) * R + r) * 2;
      f = q[0];
      df = q[1];
      if (!mtgp_isfinite(f)) { f = mx; df = 0.0f; }
    }
    v[r] = f;
    dv[r] = df;
  }
  for (int n = Rp; n > 1; n >>= 1)
    for (int i = 0; i < n / 2; ++i) {
      v[i] = v[2 * i] + v[2 * i + 1];
      dv[i] = dv[2 * i] + dv[2 * i + 1];
    }
  const float mean = v[0] / (float)R;
  float dmean = dv[0] / (float)R;
  float c = mean;
  if (mean < 0.0f) { c = 0.0f; dmean = 0.0f; }
  else if (mean == 0.0f) dmean = 0.5f * dmean;
  if (c > mx) { c = mx; dmean = 0.0f; }
  else if (c == mx) dmean = 0.5f * dmean;
  if (k == 0) A.loss[p] = c;
  A.grad[gid] = k < A.nparam[p] ? dmean : 0.0f;
}

// ------------------------------------------------------------------------------------------
// Control evaluators (dynamic_evaluate.py:37-118, feedforward_evaluate.py:36-110) with a
// fixed-step solve: one (individual p, parameter k, rollout r) per lane, the evaluator's solve in
// dual numbers -- f_obs (C @ x + noise, Acrobot wrap), the readout / policy and state programs
// (parameterised: data slots D .. D + K - 1 are the coefficients), the environment drift in the
// spec of include/mtgp_dual.h, RK4 / Euler, the Event, the save-point readout and an online
// fitness whose every addition is the oracle's (oracle_ctl_grad; value = the evaluator's rollout
// fitness bit for bit).  The data vector is the reference's [y(n_obs), a, u, tg] (no slot gap).
__device__ __forceinline__ MtgpDual tod(Dual a) { return mtgp_dl(a.v, a.d); }
__device__ __forceinline__ Dual frd(MtgpDual a) { return {a.v, a.d}; }

template <int ENV>
struct CtlEnv;
template <>
struct CtlEnv<0> {  // Acrobot
  static constexpr int NV = 4, NP = 4;
};
template <>
struct CtlEnv<1> {  // HarmonicOscillator
  static constexpr int NV = 2, NP = 2;
};
template <>
struct CtlEnv<2> {  // StirredTankReactor
  static constexpr int NV = 3, NP = 8;
};

constexpr int kCtlData = 8;  // data slots of the control models (mtgp_kernels.hip kDMax)

// DP: the Dopri5 + PID solve, else the fixed-step one -- separate kernels, so neither pays for
// the other's arrays.  Every per-component array is indexed at compile time (unrolled loops, a
// run-time index only selects among registers), so the dual state lives in VGPRs, not scratch
// (round 4: 450-576 bytes of scratch per lane, a scratch round trip per access on a latency-bound
// launch).
template <int ENV, int NA, bool DP>
__global__ void __launch_bounds__(kGradBlock) k_ctl_grad(GradArgs A) {
  __shared__ Dual s_stk[MTGP_STACK_MAX][kGradBlock];
  const LdsStack stk{&s_stk[0][threadIdx.x]};
  constexpr int NV = CtlEnv<ENV>::NV, NP = CtlEnv<ENV>::NP, ND = NV + NA;
  constexpr bool DYN = NA > 0;
  const int R = A.ro.R;
  int p, k, r;
  size_t slot;
  if (!grad_lane(A, p, k, r, slot)) return;
  float* out = A.part + slot * 2;
  const int np = A.nparam[p];
  if (k > 0 && k >= np) {
    out[0] = 0.0f;
    out[1] = 0.0f;
    return;
  }
  const int kk = k < np ? k : -1;
  const float* th = A.theta + (size_t)p * A.K;
  const int no = A.m.n_obs, nt = A.m.n_targets;
  const int D = DYN ? no + NA + 1 + nt : no + nt;
  const MtgpInstr* pr = A.prog + (size_t)p * A.n_prog * A.L;
  const MtgpInstr* p_read = pr + (size_t)A.m.prog_readout * A.L;
  const MtgpInstr* p_save = pr + (size_t)A.m.prog_readout_save * A.L;
  const MtgpInstr* p_state = pr + (size_t)(A.m.prog_state < 0 ? 0 : A.m.prog_state) * A.L;
  float prm[NP], tg[kCtlData];
#pragma unroll
  for (int i = 0; i < NP; ++i) prm[i] = A.ro.params[(size_t)r * NP + i];
#pragma unroll
  for (int i = 0; i < kCtlData; ++i) {
    tg[i] = 0.0f;
    if (i < nt) tg[i] = A.ro.targets[(size_t)r * nt + i];
  }
  const uint32_t* key = A.ro.obs_keys ? A.ro.obs_keys + 2 * (size_t)r : nullptr;
  // the data vector of a program call, and its reader
  float dvv[kCtlData], dvd[kCtlData];
  const bool use_jit = dual_jit_ok(A);  // the programs as dual-number code (mtgp_jit_dual.h)
  // the code was written by this call's emit kernel, possibly over code an earlier launch ran from
  // (the same buffer, or a freed buffer's address reused): drop the CU's stale instruction lines
  if (use_jit) asm volatile("s_icache_inv");
  auto V = [&](uint32_t off) -> Dual {
    const int sl = (int)(off / MTGP_SLOT_BYTES);
    if (sl < D) {
      float v = 0.0f, d = 0.0f;
#pragma unroll
      for (int i = 0; i < kCtlData; ++i) {
        v = (i == sl) ? dvv[i] : v;
        d = (i == sl) ? dvd[i] : d;
      }
      return {v, d};
    }
    return {th[sl - D], (sl - D == kk) ? 1.0f : 0.0f};
  };
  auto put = [&](int i, Dual x) {
#pragma unroll
    for (int j = 0; j < kCtlData; ++j) {
      dvv[j] = (j == i) ? x.v : dvv[j];
      dvd[j] = (j == i) ? x.d : dvd[j];
    }
  };
  // f_obs (cbase.py:43-48, acrobot.py:29-32) in duals: the oracle's ctl_f_obs_dual
  auto f_obs = [&](float t, const Dual* x, Dual* y) {
    float nz[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) nz[j] = 0.0f;
    if (key) {  // mtgp_obs_normals word by word (compile-time indices)
      uint32_t n0, n1;
      mtgp_fold_in(key[0], key[1], mtgp_f2u(t), &n0, &n1);
      float n[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i)
        n[i] = i < no ? mtgp_normal_from_bits(mtgp_random_bits_word(n0, n1, i, no, A.m.prng_impl)) : 0.0f;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        if (j >= no) continue;
        float sacc = n[0] * A.ro.obs_w[0 * no + j];
#pragma unroll
        for (int i = 1; i < NV; ++i)
          if (i < no) sacc = sacc + n[i] * A.ro.obs_w[i * no + j];
        nz[j] = sacc;
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (i >= no) { y[i] = {0.0f, 0.0f}; continue; }
      MtgpDual sacc = mtgp_dl_cmul(i == 0 ? 1.0f : 0.0f, tod(x[0]));
#pragma unroll
      for (int j = 1; j < NV; ++j) sacc = mtgp_dl_add(sacc, mtgp_dl_cmul(i == j ? 1.0f : 0.0f, tod(x[j])));
      y[i] = frd(mtgp_dl_addc(sacc, nz[i]));
    }
    if (ENV == 0) {
      y[0] = frd(mtgp_dl_wrap_angle(tod(y[0])));
      if (no > 1) y[1] = frd(mtgp_dl_wrap_angle(tod(y[1])));
    }
  };
  auto drift = [&](const Dual* x, Dual u, Dual* dx) {
    MtgpDual xx[NV], d[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) xx[i] = tod(x[i]);
    if constexpr (ENV == 0) mtgp_dl_acro_drift(prm, xx, tod(u), d);
    else if constexpr (ENV == 1) mtgp_dl_ho_drift(prm, xx, tod(u), d);
    else mtgp_dl_reactor_drift(prm, xx, tod(u), d);
#pragma unroll
    for (int i = 0; i < NV; ++i) dx[i] = frd(d[i]);
  };
  // _drift (dyn.py:107-118 / ff.py:104-110) in duals.  The readout and the state programs run
  // from ONE interpreter site (program q = 0 the readout, q >= 1 state program q - 1), and the
  // drift after them (it reads only the state and u; no program reads its result): the inlined
  // interpreter is then one copy per rhs, its data vector registers (a called interpreter would
  // read the data vector through memory -- scratch, round 4).
  auto rhs = [&](float t, const Dual* st, Dual* ds) {
    Dual y[NV];
    f_obs(t, st, y);
#pragma unroll
    for (int j = 0; j < kCtlData; ++j) { dvv[j] = 0.0f; dvd[j] = 0.0f; }
    if (DYN) {
#pragma unroll
      for (int j = 0; j < (DYN ? NA : 1); ++j) put(no + j, st[NV + j]);
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (i < no) put(i, y[i]);
    }
#pragma unroll
    for (int j = 0; j < kCtlData; ++j)
      if (j < nt) put(DYN ? no + NA + 1 + j : no + j, {tg[j], 0.0f});
    Dual u = {0.0f, 0.0f};
#pragma unroll 1
    for (int q = 0; q <= NA; ++q) {
      if (DYN && q == 1) {  // the state programs read [y, a, u, tg]; the readout read [0, a, 0, tg]
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (i < no) put(i, y[i]);
        put(no + NA, u);
      }
      const Dual o = use_jit ? dual_call(dual_unit(A, p, q == 0 ? A.m.prog_readout : A.m.prog_state + q - 1), dvv, dvd, kk)
                             : run_dual_src(q == 0 ? p_read : p_state + (size_t)(q - 1) * A.L, V, stk);
      if (q == 0) u = o;
#pragma unroll
      for (int j = 0; j < (DYN ? NA : 1); ++j)
        if (DYN && q == j + 1) ds[NV + j] = o;
    }
    drift(st, u, ds);
  };
  // online fitness over the save points (oracle_ctl_grad's full-array loop, addition for addition)
  const int S = A.m.n_save;
  const float* ts = A.ro.ts;
  const float dts = ts[1] - ts[0];
  bool settled = false;
  int fs = 0;
  MtgpDual cs = mtgp_dl(0.0f, 0.0f), c0 = mtgp_dl(0.0f, 0.0f);
  // the general Acrobot mask (MtgpRollouts.fit_kof: ts / dts off the one-pass grid): the kept costs
  // are the first K = kof[fs] saves, so the oracle's sum is A_K = ((0 + c_0) + ...) + c_{K-1}, then
  // + 0 for the masked rest.  pre = the running prefix (its values kept in hist: K may lie behind
  // the first success), Kt = K once known, AK = A_K once complete.
  const int32_t* kof = ENV == 0 ? A.ro.fit_kof : nullptr;
  const size_t nsl = (size_t)A.P * A.K * R;
  MtgpDual pre = mtgp_dl(0.0f, 0.0f), AK = mtgp_dl(0.0f, 0.0f);
  int Kt = -1, q_pre = -1;  // q_pre: the last save folded into pre
  bool a_set = false;
  auto hist_put = [&](int q, MtgpDual v) {
    float* h = A.hist + ((size_t)q * nsl + slot) * 2;
    h[0] = v.v;
    h[1] = v.d;
  };
  auto hist_get = [&](int q) {
    const float* h = A.hist + ((size_t)q * nsl + slot) * 2;
    return mtgp_dl(h[0], h[1]);
  };
  auto prefix_done = [&]() {  // settled with Kt known: A_K from pre / hist when complete
    if (Kt == 0) { AK = mtgp_dl(0.0f, 0.0f); a_set = true; }
    else if (Kt - 1 <= q_pre) { AK = Kt - 1 == q_pre ? pre : hist_get(Kt - 1); a_set = true; }
  };
  auto save_point = [&](int q, const Dual* xq) {
    Dual y[NV];
    f_obs(ts[q], xq, y);
#pragma unroll
    for (int j = 0; j < kCtlData; ++j) { dvv[j] = 0.0f; dvd[j] = 0.0f; }
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (i < no) put(i, y[i]);
    Dual u;
    if (DYN) {
#pragma unroll
      for (int j = 0; j < (DYN ? NA : 1); ++j) put(no + j, xq[NV + j]);
#pragma unroll
      for (int j = 0; j < kCtlData; ++j)
        if (j < nt) put(no + NA + 1 + j, {tg[j], 0.0f});
      u = use_jit ? dual_call(dual_unit(A, p, A.m.prog_readout_save), dvv, dvd, kk)
                  : run_dual_src(p_save, V, stk);  // dyn.py:101 [y, a, 0, tg]
    } else {
#pragma unroll
      for (int j = 0; j < kCtlData; ++j)
        if (j < nt) put(no + j, {tg[j], 0.0f});
      u = use_jit ? dual_call(dual_unit(A, p, A.m.prog_readout), dvv, dvd, kk)
                  : run_dual_src(p_read, V, stk);  // ff.py:97
    }
    if constexpr (ENV == 0) {
      const MtgpDual ud = tod(u);
      const MtgpDual cost = mtgp_dl_mul(mtgp_dl_mulc(ud, 0.01f), ud);
      const bool reached = ((-mtgp_cosf(xq[0].v)) - mtgp_cosf(xq[0].v + xq[1].v)) > 1.5f;
      if (kof) {
        if (!settled || !a_set) {  // fold c_q into the prefix while it may still be needed
          pre = mtgp_dl_add(q == 0 ? mtgp_dl(0.0f, 0.0f) : pre, cost);
          q_pre = q;
          if (!settled) hist_put(q, pre);
        }
        if (!settled && reached) {
          settled = true;
          fs = q;
          Kt = kof[fs];
        }
        if (settled && !a_set) prefix_done();
        return;
      }
      if (q == 0) {
        const bool incl0 = !((ts[0] / dts) > 0.0f);
        c0 = mtgp_dl_add(mtgp_dl(0.0f, 0.0f), incl0 ? cost : mtgp_dl(0.0f, 0.0f));
        cs = mtgp_dl_add(mtgp_dl(0.0f, 0.0f), cost);
        if (reached) { settled = true; fs = 0; cs = c0; }
      } else if (settled) {
        cs = mtgp_dl_add(cs, mtgp_dl(0.0f, 0.0f));
      } else if (reached) {
        fs = q;
        cs = mtgp_dl_add(cs, ((ts[q] / dts) > (float)q) ? mtgp_dl(0.0f, 0.0f) : cost);
        settled = true;
      } else {
        cs = mtgp_dl_add(cs, cost);
      }
    } else if constexpr (ENV == 1) {
      const float Q[4] = {0.5f, 0.0f, 0.0f, 0.0f};
      const float ud0 = (-0.0f * 0.0f + -1.0f * (-prm[0])) * tg[0] + ((-0.0f) * 1.0f + (-1.0f) * (-prm[1])) * 0.0f;
      const MtgpDual e[2] = {mtgp_dl_subc(tod(xq[0]), tg[0]), mtgp_dl_subc(tod(xq[1]), 0.0f)};
      const MtgpDual du = mtgp_dl_subc(tod(u), ud0);
      cs = mtgp_dl_add(cs, mtgp_dl_add(mtgp_dl_quad_form(e, Q, 2), mtgp_dl_mul(mtgp_dl_mulc(du, 0.5f), du)));
    } else {
      const float Q[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.01f, 0.0f, 0.0f, 0.0f, 0.0f};
      const MtgpDual e[3] = {mtgp_dl_subc(tod(xq[0]), 0.0f), mtgp_dl_subc(tod(xq[1]), tg[0]),
                             mtgp_dl_subc(tod(xq[2]), 0.0f)};
      cs = mtgp_dl_add(cs, mtgp_dl_add(mtgp_dl_quad_form(e, Q, 3), mtgp_dl_mul(mtgp_dl_mulc(tod(u), 0.0001f), tod(u))));
    }
  };
  auto bad = [&](const Dual* st) {  // cond_fn (acrobot.py:86-87; the others: any non-finite)
    bool b = false;
#pragma unroll
    for (int i = 0; i < ND; ++i) b = b || !mtgp_isfinite(st[i].v);
    if (ENV == 0) {
      b = b || (!mtgp_isnan(st[2].v) && __builtin_fabsf(st[2].v) > MTGP_8PI_F);
      b = b || (!mtgp_isnan(st[3].v) && __builtin_fabsf(st[3].v) > MTGP_18PI_F);
    }
    return b;
  };
  Dual s[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) s[i] = {i < NV ? A.ro.x0[(size_t)r * NV + i] : 0.0f, 0.0f};
  bool prev_ok = !bad(s);
  const float h = A.m.h;
  int q_saved = 0;
  if constexpr (DP) {
    save_point(0, s);
    // k_ctl_dopri5's solve in duals (oracle ctl_dopri5_dual): the step sizes, accept / reject
    // decisions and the event held at their primal values; save points by the dense output.
    // The tableau sums are accumulated as the stages arrive -- stage j's f adds its a_ij f_j to
    // the sum of every later stage i, the error sum and the midpoint sum -- which is each sum's
    // ascending-j order of mtgp_dp_term exactly, with no per-stage f kept (f_0 and f_6 aside).
    const float t_end = ts[S - 1];
    Dual f0[ND], fc[ND], yi[ND], sk[ND];
    Dual ac[6][ND], am[ND];  // ac[i - 1]: stage i's sum; am: the midpoint sum
    float ae[ND];            // the error sum (values only)
    auto contrib = [&](int j, const Dual* f) __attribute__((always_inline)) {
      const bool first = j == 0;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        if (q + 1 <= j) continue;  // stages up to j are done
        const float w = kDpA[q + 1][j];
#pragma unroll
        for (int i = 0; i < ND; ++i)
          ac[q][i] = {mtgp_dp_term(ac[q][i].v, w, f[i].v, first), mtgp_dp_term(ac[q][i].d, w, f[i].d, first)};
      }
      const float we = kDpE[j], wm = kDpCM[j];
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        ae[i] = mtgp_dp_term(ae[i], we, f[i].v, first);
        am[i] = {mtgp_dp_term(am[i].v, wm, f[i].v, first), mtgp_dp_term(am[i].d, wm, f[i].d, first)};
      }
    };
    int ks = 1, steps = 0;
    float t = ts[0];
    float tnext = t + h;
    tnext = tnext > t_end ? t_end : tnext;
    bool have_f0 = false;  // f_0 of the first attempt comes from the stage loop (one rhs site)
    const MtgpDpPid pid = A.m.pid_custom ? MtgpDpPid{A.m.pid_c1, A.m.pid_c2, A.m.pid_c3, A.m.pid_safety,
                                                     A.m.pid_factormin, A.m.pid_factormax}
                                         : MtgpDpPid MTGP_DP_PID_DEFAULT;
    MtgpDpCtl ctl{1.0f, 1.0f, 0};
    const int force_dtmin = !A.m.no_force_dtmin;
    while (t < t_end && steps < A.m.max_steps) {
      const float hs = tnext - t;
      if (have_f0) contrib(0, f0);
#pragma unroll 1
      for (int st = have_f0 ? 1 : 0; st <= 6; ++st) {
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          Dual a = ac[0][i];
#pragma unroll
          for (int q = 1; q < 6; ++q) a = (st == q + 1) ? ac[q][i] : a;
          yi[i] = st == 0 ? s[i] : Dual{MTGP_FMAF(hs, a.v, s[i].v), MTGP_FMAF(hs, a.d, s[i].d)};
        }
        rhs(st == 0 ? t : t + mtgp_dp_c(st) * hs, yi, fc);
        if (st == 0) {
#pragma unroll
          for (int i = 0; i < ND; ++i) f0[i] = fc[i];
          have_f0 = true;
        }
        contrib(st, fc);
      }
      // yi = y1 (stage 6's input), fc = f_6
      float msum = 0.0f;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const float sc = mtgp_dp_scaled(hs * ae[i], s[i].v, yi[i].v, A.m.rtol, A.m.atol);
        msum = (i == 0) ? sc * sc : msum + sc * sc;
      }
      const float ms = msum / (float)ND;
      int keep, fail;
      const float dt = mtgp_dp_control(ms, hs, A.m.dtmin, A.m.dtmax, force_dtmin, &pid, &ctl, &keep, &fail);
      ++steps;
      bool stop = fail != 0;
      if (keep) {
        const float t1 = tnext;
        while (ks < S && ts[ks] <= t1) {
          const float th = (ts[ks] - t) / hs;
#pragma unroll
          for (int i = 0; i < ND; ++i) {
            const float ymid = MTGP_FMAF(hs, am[i].v, s[i].v), dymid = MTGP_FMAF(hs, am[i].d, s[i].d);
            sk[i] = {mtgp_dp_interp(s[i].v, yi[i].v, ymid, hs * f0[i].v, hs * fc[i].v, th),
                     mtgp_dp_interp(s[i].d, yi[i].d, dymid, hs * f0[i].d, hs * fc[i].d, th)};
          }
          save_point(ks, sk);
          ++ks;
        }
        t = t1;
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          s[i] = yi[i];
          f0[i] = fc[i];  // FSAL
        }
        const bool ok = !bad(s);
        if (prev_ok && !ok) stop = true;  // Event(cond_fn_nan), dyn.py:94
        prev_ok = ok;
      }
      if (stop) break;
      tnext = mtgp_dp_clip_end(t, dt, t_end, keep);
    }
    q_saved = ks - 1;
  } else {
    // the fixed-step solve (include/mtgp_cstep.h, k_ctl_dynamic / k_ctl_static) in duals: the time
    // grid and the event primal, the stage sums, step update and dense output applied to both halves
    const bool euler = A.m.solver == MTGP_SOLVER_EULER;
    const float t_end = ts[S - 1];
    float t = ts[0], tn = mtgp_cs_first_end(t, h, t_end);
    int steps = 0, ks = 0;
    Dual f0[ND], y1[ND], sk[ND], kx[ND], acc[ND], tmp[ND];
    while (t < t_end && mtgp_cs_advancing(steps, t, tn) && (A.m.max_steps <= 0 || steps < A.m.max_steps)) {
      const float dt = tn - t;
      Dual z[ND];  // the zero tableau entries' terms (mtgp_cstep.h), value and tangent
      // the stages from one rhs site (stage 0 included; Euler: stage 0 only)
#pragma unroll 1
      for (int st = 0; st <= (euler ? 0 : 3); ++st) {
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          tmp[i] = st == 0 ? s[i]
                           : Dual{mtgp_rk4_in(st, s[i].v, kx[i].v, z[i].v, dt), mtgp_rk4_in(st, s[i].d, kx[i].d, z[i].d, dt)};
          if (st == 1 || st == 2) z[i] = Dual{mtgp_rk4_zero(st, z[i].v, kx[i].v), mtgp_rk4_zero(st, z[i].d, kx[i].d)};
        }
        rhs(st == 0 ? t : mtgp_rk4_time(st, t, dt), tmp, kx);
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          if (st == 0) f0[i] = kx[i];
          acc[i] = {mtgp_rk4_acc(st, acc[i].v, kx[i].v), mtgp_rk4_acc(st, acc[i].d, kx[i].d)};
        }
      }
#pragma unroll
      for (int i = 0; i < ND; ++i)
        y1[i] = euler ? Dual{s[i].v + f0[i].v * dt, s[i].d + f0[i].d * dt}
                      : Dual{mtgp_rk4_out(s[i].v, acc[i].v, dt), mtgp_rk4_out(s[i].d, acc[i].d, dt)};
      while (ks < S && ts[ks] <= tn) {  // SaveAt(ts) by the dense output
        const float th = mtgp_cs_rescale(t, ts[ks], tn);
#pragma unroll
        for (int i = 0; i < ND; ++i)
          sk[i] = euler ? Dual{mtgp_cs_linear(s[i].v, y1[i].v, th), mtgp_cs_linear(s[i].d, y1[i].d, th)}
                        : Dual{mtgp_cs_hermite(s[i].v, y1[i].v, f0[i].v * dt, kx[i].v * dt, th),
                               mtgp_cs_hermite(s[i].d, y1[i].d, f0[i].d * dt, kx[i].d * dt, th)};
        save_point(ks, sk);
        ++ks;
      }
#pragma unroll
      for (int i = 0; i < ND; ++i) s[i] = y1[i];
      ++steps;
      t = tn;
      tn = mtgp_cs_next_end(t, h, t_end);
      const bool ok = !bad(s);
      if (prev_ok && !ok) break;  // Event(cond_fn_nan), dyn.py:94
      prev_ok = ok;
    }
    q_saved = ks - 1;
  }
  // the +inf fill after the event (constants): Acrobot masks it (zero additions), the quadratic
  // costs become non-finite
  float F, dF;
  if constexpr (ENV == 0) {
    if (kof) {
      // the fill saves (+inf states: never a success) still count while the kept prefix runs into
      // them: their readout costs are folded in as the oracle's full arrays hold them
      Dual fillx[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) fillx[i] = {kInf, 0.0f};
      for (int q = q_saved + 1; q < S; ++q) {
        const int need = settled ? (a_set ? -1 : Kt - 1) : kof[0] - 1;
        if (q > need) break;
        save_point(q, fillx);
      }
      if (!settled) {  // no success: first_success = argmax of all-false = 0
        fs = 0;
        Kt = kof[0];
        settled = true;
        prefix_done();
      }
      cs = Kt < S ? mtgp_dl_add(AK, mtgp_dl(0.0f, 0.0f)) : AK;
      const MtgpDual Fd = mtgp_dl_cadd((float)(fs + (fs == 0) * S), cs);
      out[0] = Fd.v;
      out[1] = Fd.d;
      return;
    }
    if (q_saved + 1 < S && settled) cs = mtgp_dl_add(cs, mtgp_dl(0.0f, 0.0f));
    if (!settled) {
      fs = 0;
      cs = S > 1 ? mtgp_dl_add(c0, mtgp_dl(0.0f, 0.0f)) : c0;
    }
    const MtgpDual Fd = mtgp_dl_cadd((float)(fs + (fs == 0) * S), cs);
    F = Fd.v;
    dF = Fd.d;
  } else {
    F = q_saved + 1 < S ? mtgp_qnan() : cs.v;
    dF = cs.d;
  }
  out[0] = F;
  out[1] = dF;
}

// ---- dual-number program code (mtgp_jit_dual.h): count, scan, subroutines, emit --------------
// Units: one per (individual p, program j), each starting on a 64-byte line; the shared
// subroutines (sin, cos, exp, log, tanh, sqrt) at the start of the buffer.  All on the stream, no
// host round trip: the gradient kernel checks info and interprets when the code is unusable.
struct DualJitArgs {
  const MtgpInstr* prog;
  int n_prog, L, P, K, D;
  const float* theta;  // [P, K]
};
constexpr uint32_t kDualAlign = 64u;

__global__ void __launch_bounds__(256) k_dual_count(DualJitArgs J, uint32_t* __restrict__ offs,
                                                    int32_t* __restrict__ info) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= J.P * J.n_prog) return;
  const int p = u / J.n_prog;
  const int n = mtgp::jit_dual_words(J.prog + (size_t)u * J.L, J.L, J.D, J.theta + (size_t)p * J.K, J.K);
  offs[u] = n > 0 ? ((uint32_t)n * 4u + kDualAlign - 1u) & ~(kDualAlign - 1u) : 0u;
  if (n < 0) atomicMin(&info[0], n);
}

// exclusive scan of the unit spans in place (after the subroutine area); offs[total], info[1] = bytes
__global__ void __launch_bounds__(1024) k_dual_scan(uint32_t* __restrict__ offs, int total, int32_t* __restrict__ info) {
  __shared__ uint64_t part[1024];
  const int t = threadIdx.x;
  const int per = (total + 1023) / 1024;
  const int b = t * per, e = b + per < total ? b + per : total;
  uint64_t sum = 0;
  for (int i = b; i < e; ++i) sum += offs[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const uint64_t sub = (mtgp::kJitTemplateBytes + kDualAlign - 1u) & ~(uint64_t)(kDualAlign - 1u);
  uint64_t run = part[t] - sum + sub;
  for (int i = b; i < e; ++i) {
    const uint64_t w = offs[i];
    offs[i] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
    run += w;
  }
  if (t == 1023) {
    const uint64_t tot = part[1023] + sub;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

__global__ void __launch_bounds__(256) k_dual_templates(uint32_t* __restrict__ code, uint64_t code_bytes) {
  if (code_bytes < mtgp::kJitTemplateBytes) return;
  for (int i = threadIdx.x; i < MTGP_JIT_SUB_WORDS; i += blockDim.x) code[i] = mtgp_jit_sub_blob[i];
}

__global__ void __launch_bounds__(256) k_dual_emit(DualJitArgs J, const uint32_t* __restrict__ offs,
                                                   uint32_t* __restrict__ code, uint64_t code_bytes) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= J.P * J.n_prog) return;
  const uint32_t b = offs[u], e = offs[u + 1];
  if (e <= b || (uint64_t)e > code_bytes) return;  // untranslatable or short buffer (checked on use)
  const int p = u / J.n_prog;
  mtgp::JitOut o{code + b / 4, 0};
  o.base = b;
  mtgp::jit_dual_program(o, J.prog + (size_t)u * J.L, J.L, J.D, J.theta + (size_t)p * J.K, J.K);
}

}  // namespace

// Emit the dual code of a launch (or do nothing without a buffer); fills A's jit fields.
static int dual_jit_prepare(GradArgs& A, const MtgpGradJit* jit, int D, hipStream_t s) {
  A.jit_code = nullptr;
  A.jit_offs = nullptr;
  A.jit_info = nullptr;
  A.jit_bytes = 0;
  if (!jit || !jit->code) return MTGP_OK;
  if (!jit->offsets || !jit->info || jit->code_bytes < mtgp::kJitTemplateBytes) return MTGP_ERR_ARG;
  const int units = A.P * A.n_prog;
  DualJitArgs J{A.prog, A.n_prog, A.L, A.P, A.K, D, A.theta};
  if (hipMemsetAsync(jit->info, 0, 2 * sizeof(int32_t), s) != hipSuccess) return MTGP_ERR_LAUNCH;
  const dim3 g((unsigned)((units + 255) / 256)), b(256);
  hipLaunchKernelGGL(k_dual_count, g, b, 0, s, J, jit->offsets, jit->info);
  hipLaunchKernelGGL(k_dual_scan, dim3(1), dim3(1024), 0, s, jit->offsets, units, jit->info);
  hipLaunchKernelGGL(k_dual_templates, dim3(1), dim3(256), 0, s, (uint32_t*)jit->code, (uint64_t)jit->code_bytes);
  hipLaunchKernelGGL(k_dual_emit, g, b, 0, s, J, jit->offsets, (uint32_t*)jit->code, (uint64_t)jit->code_bytes);
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  A.jit_code = (const uint8_t*)jit->code;
  A.jit_offs = jit->offsets;
  A.jit_info = jit->info;
  A.jit_bytes = jit->code_bytes;
  return MTGP_OK;
}

// host translation of one program in dual numbers (tests: the emulator runs it)
extern "C" int mtgp_jit_dual_translate_host(const MtgpInstr* prog, int32_t L, int32_t D, const float* theta, int32_t K,
                                            uint32_t base, uint32_t* out, int32_t max_words) {
  if (!prog || L <= 0 || (K > 0 && !theta)) return MTGP_ERR_ARG;
  const int n = mtgp::jit_dual_words(prog, L, D, theta, K);
  if (n < 0) return n;
  if (!out) return n;
  if (n > max_words) return MTGP_ERR_ARG;
  mtgp::JitOut o{out, 0};
  o.base = base;
  mtgp::jit_dual_program(o, prog, L, D, theta, K);
  return o.n;
}

static bool grad_args(GradArgs& A, const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                      const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* ro, float* scratch,
                      float* loss_out, float* grad_out) {
  A.m = *model;
  A.prog = prog;
  A.n_prog = n_prog;
  A.L = L;
  A.P = P;
  A.K = K;
  A.theta = theta;
  A.nparam = nparam;
  A.ro = *ro;
  A.part = scratch;
  A.hist = nullptr;
  A.loss = loss_out;
  A.grad = grad_out;
  A.jit_code = nullptr;
  A.jit_offs = nullptr;
  A.jit_info = nullptr;
  A.jit_bytes = 0;
  return true;
}

extern "C" int mtgp_ctl_grad_jit(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L,
                                 int32_t P, const float* theta, const int32_t* nparam, int32_t K,
                                 const MtgpRollouts* ro, float* scratch, float* loss_out, float* grad_out,
                                 const MtgpGradJit* jit, void* stream) {
  if (!model || !prog || !ro || !nparam || !scratch || !loss_out || !grad_out || P < 0 || K < 1 || L <= 0 ||
      n_prog <= 0 || !theta)
    return MTGP_ERR_ARG;
  const bool dyn = model->model == MTGP_MODEL_DYNAMIC;
  if (!dyn && model->model != MTGP_MODEL_STATIC) return MTGP_ERR_ARG;
  const bool dopri5 = model->solver == MTGP_SOLVER_DOPRI5;
  if (model->solver != MTGP_SOLVER_RK4 && model->solver != MTGP_SOLVER_EULER && !dopri5) return MTGP_ERR_ARG;
  if (dopri5 && (model->max_steps <= 0 || !(model->h > 0.0f))) return MTGP_ERR_ARG;
  const int nv = model->env == MTGP_ENV_ACROBOT ? 4 : (model->env == MTGP_ENV_HARMONIC_OSCILLATOR ? 2 : 3);
  if (model->env < 0 || model->env > 2 || model->n_var != nv || model->n_obs < 1 || model->n_obs > nv ||
      model->n_control != 1 || model->n_targets < 0 || model->n_targets > 8 || !ro->params || !ro->x0 || !ro->ts ||
      (model->n_targets > 0 && !ro->targets) || (ro->obs_keys && !ro->obs_w) || ro->R < 1 || ro->R > 64 ||
      model->n_save < 2 || !(model->h > 0.0f) || model->prog_readout < 0 ||
      model->prog_readout >= n_prog || (ro->fit_kof && model->env != MTGP_ENV_ACROBOT))
    return MTGP_ERR_ARG;
  const int na = dyn ? model->state_size : 0;
  const int D = model->n_obs + (dyn ? na + 1 : 0) + model->n_targets;
  if (na < 0 || na > 3 || D > kCtlData || D + K > MTGP_MAX_DATA) return MTGP_ERR_ARG;
  if (dyn && (model->prog_state < 0 || model->prog_state + na > n_prog || model->prog_readout_save < 0 ||
              model->prog_readout_save >= n_prog))
    return MTGP_ERR_ARG;
  if (P == 0) return MTGP_OK;
  GradArgs A;
  grad_args(A, model, prog, n_prog, L, P, theta, nparam, K, ro, scratch, loss_out, grad_out);
  // the general Acrobot mask keeps its cost prefixes behind the partials (mtgp.h: scratch size)
  if (ro->fit_kof) A.hist = scratch + (size_t)P * K * ro->R * 2;
  hipStream_t s = (hipStream_t)stream;
  const int jrc = dual_jit_prepare(A, jit, D, s);
  if (jrc != MTGP_OK) return jrc;
  const long lanes = (long)P * grad_lanes_per(K, ro->R);  // whole waves per individual (grad_lane)
  const dim3 grid((unsigned)((lanes + 255) / 256)), block(256);
#define MTGP_CG2(E, DPV)                                                                  \
  switch (na) {                                                                           \
    case 0: hipLaunchKernelGGL((k_ctl_grad<E, 0, DPV>), grid, block, 0, s, A); break;     \
    case 1: hipLaunchKernelGGL((k_ctl_grad<E, 1, DPV>), grid, block, 0, s, A); break;     \
    case 2: hipLaunchKernelGGL((k_ctl_grad<E, 2, DPV>), grid, block, 0, s, A); break;     \
    default: hipLaunchKernelGGL((k_ctl_grad<E, 3, DPV>), grid, block, 0, s, A); break;    \
  }
#define MTGP_CG(E)              \
  if (dopri5) MTGP_CG2(E, true) \
  else MTGP_CG2(E, false)
  if (model->env == MTGP_ENV_ACROBOT) { MTGP_CG(0) }
  else if (model->env == MTGP_ENV_HARMONIC_OSCILLATOR) { MTGP_CG(1) }
  else { MTGP_CG(2) }
#undef MTGP_CG
#undef MTGP_CG2
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  hipLaunchKernelGGL(k_grad_reduce, dim3((unsigned)(((long)P * K + 255) / 256)), dim3(256), 0, s, A);
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  return MTGP_OK;
}

extern "C" int mtgp_ctl_grad(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                             const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* ro,
                             float* scratch, float* loss_out, float* grad_out, void* stream) {
  return mtgp_ctl_grad_jit(model, prog, n_prog, L, P, theta, nparam, K, ro, scratch, loss_out, grad_out, nullptr,
                           stream);
}

extern "C" int mtgp_sr_grad_jit(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L,
                                int32_t P, const float* theta, const int32_t* nparam, int32_t K,
                                const MtgpRollouts* ro, float* scratch, float* loss_out, float* grad_out,
                                const MtgpGradJit* jit, void* stream) {
  if (!model || !prog || !ro || !nparam || !scratch || !loss_out || !grad_out || P < 0 || K < 1 || L <= 0 ||
      n_prog <= 0 || (K > 0 && !theta))
    return MTGP_ERR_ARG;
  if (model->model != MTGP_MODEL_SR || model->n_var < 1 || model->n_var > MTGP_MAX_DATA ||
      model->n_var + K > MTGP_MAX_DATA || ro->R < 1 || ro->R > 64 || !ro->x0 || !ro->ys_true ||
      model->n_save < 2 || !(model->h > 0.0f) || !ro->ts || model->prog_state < 0 ||
      model->prog_state + model->n_var > n_prog)
    return MTGP_ERR_ARG;
  const bool dopri5 = model->solver == MTGP_SOLVER_DOPRI5;
  if (model->solver != MTGP_SOLVER_RK4 && model->solver != MTGP_SOLVER_EULER && !dopri5) return MTGP_ERR_ARG;
  if (dopri5 && (model->n_save < 2 || model->max_steps <= 0 || !(model->h > 0.0f) || !ro->ts)) return MTGP_ERR_ARG;
  if (P == 0) return MTGP_OK;
  GradArgs A;
  A.m = *model;
  A.prog = prog;
  A.n_prog = n_prog;
  A.L = L;
  A.P = P;
  A.K = K;
  A.theta = theta;
  A.nparam = nparam;
  A.ro = *ro;
  A.part = scratch;
  A.hist = nullptr;
  A.loss = loss_out;
  A.grad = grad_out;
  hipStream_t s = (hipStream_t)stream;
  // dual-number code for the register-state kernels (n_var <= 4: data slots = the state)
  const int jrc = dual_jit_prepare(A, model->n_var <= 4 ? jit : nullptr, model->n_var, s);
  if (jrc != MTGP_OK) return jrc;
  const long lanes = (long)P * grad_lanes_per(K, ro->R);  // whole waves per individual (grad_lane)
  const dim3 grid((unsigned)((lanes + 255) / 256)), block(256);
  const int nv = model->n_var;
  if (dopri5) {
    if (nv <= 2) hipLaunchKernelGGL(k_sr_grad_dp<2>, grid, block, 0, s, A);
    else if (nv <= 4) hipLaunchKernelGGL(k_sr_grad_dp<4>, grid, block, 0, s, A);
    else if (nv <= 16) hipLaunchKernelGGL(k_sr_grad_dp<16>, grid, block, 0, s, A);
    else hipLaunchKernelGGL(k_sr_grad_dp<64>, grid, block, 0, s, A);
  } else if (nv <= 2) hipLaunchKernelGGL(k_sr_grad<2>, grid, block, 0, s, A);
  else if (nv <= 4) hipLaunchKernelGGL(k_sr_grad<4>, grid, block, 0, s, A);
  else if (nv <= 16) hipLaunchKernelGGL(k_sr_grad<16>, grid, block, 0, s, A);
  else hipLaunchKernelGGL(k_sr_grad<64>, grid, block, 0, s, A);
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  hipLaunchKernelGGL(k_grad_reduce, dim3((unsigned)(((long)P * K + 255) / 256)), dim3(256), 0, s, A);
  if (hipGetLastError() != hipSuccess) return MTGP_ERR_LAUNCH;
  return MTGP_OK;
}

extern "C" int mtgp_sr_grad(const MtgpModel* model, const MtgpInstr* prog, int32_t n_prog, int32_t L, int32_t P,
                            const float* theta, const int32_t* nparam, int32_t K, const MtgpRollouts* ro,
                            float* scratch, float* loss_out, float* grad_out, void* stream) {
  return mtgp_sr_grad_jit(model, prog, n_prog, L, P, theta, nparam, K, ro, scratch, loss_out, grad_out, nullptr,
                          stream);
}
