// mtgp_jit_dual.h -- program JIT in dual numbers: a flattened MtgpInstr program -> straight-line
// gfx950 code that computes (value, d value / d theta_k) per lane, operation for operation the
// dual interpreter of csrc/mtgp_grad.hip (run_dual_src: d_add / d_sub / d_mul / d_div, the
// include/mtgp_dual.h rules of the unary operators, constants with tangent 0).
//
// Why: coefficient optimisation (gp.py:435-473) runs one lane per (candidate, coefficient,
// rollout), one wave per candidate -- ~200 waves for 50 candidates, one wave per SIMD at most, so
// the launch is latency-bound on the interpreter's per-instruction dispatch (a scalar fetch, a
// compare tree, an exec-masked loop latch: ~200 SIMD cycles per program instruction, 11 us per
// RK4 stage of the Acrobot gradient).  Translated, an instruction is 2-6 VALU words.
//
// The coefficients theta are baked into the code as literals (the code is re-emitted per epoch:
// a count + scan + emit pass of a few microseconds); a parameter slot's tangent is 1 in the lanes
// whose coefficient index (v25) is that parameter, 0 elsewhere.
//
// Register ABI of a dual unit (the gradient kernel's call site pins these):
//   v0-v7    data values (slots 0 .. D-1, D <= 8)     v48-v55  data tangents
//   v8       result value (= template output)       v56      result tangent
//   v9-v16   operand stack values                   v57-v64  operand stack tangents
//   v17-v24  template temporaries (v17 / v18 inputs of the subroutines and the division)
//   v25      this lane's coefficient index k (int; -1: none)   v26-v29  dual-op temporaries
//   s[30:31] return address; s[34:45] template temporaries; vcc
// The shared subroutines (sin, cos, exp, log, tanh, sqrt) and the division are the templates of
// mtgp_jit_blobs.h, exactly as the evaluators' JIT uses them.
#ifndef MTGP_JIT_DUAL_H
#define MTGP_JIT_DUAL_H

#include "mtgp_jit.h"

namespace mtgp {

constexpr int kDvData = 0, kDdData = 48, kDvAcc = 8, kDdAcc = 56, kDvStack = 9, kDdStack = 57;
constexpr int kDKk = 25, kDT0 = 26, kDT1 = 27, kDP0 = 28, kDP1 = 29;
constexpr int kDualMaxData = 8;

// gfx9 encodings (checked against llvm-mc in tests/test_jit_dual.py)
constexpr uint32_t kVop2Xor = 21u, kVop2And = 19u;
constexpr uint32_t kVopcEqU32 = 0xCAu, kVopcGtF32 = 0x44u, kVopcLtF32 = 0x41u;
constexpr uint32_t kInlZero = 128u, kInlHalf = 240u, kInlOne = 242u, kInlMinusOne = 243u;

// A dual operand: value and tangent, each a VGPR or a literal (bits).
struct DualSrc {
  bool vlit;
  int vreg;
  uint32_t vbits;
  bool dlit;
  int dreg;
  uint32_t dbits;
};

MTGP_JIT_HD inline DualSrc dual_regs(int v, int d) { return DualSrc{false, v, 0u, false, d, 0u}; }

// source operand field of a literal: an inline constant when the bits are one, else 255 (+ word)
MTGP_JIT_HD inline uint32_t dual_inline(uint32_t bits) {
  switch (bits) {
    case 0x00000000u: return kInlZero;
    case 0x3f000000u: return kInlHalf;
    case 0x3f800000u: return kInlOne;
    case 0xbf800000u: return kInlMinusOne;
    default: return kJitSrcLiteral;
  }
}

struct DualOut {
  JitOut& o;
  // v_mov_b32 vdst, (reg | literal)
  MTGP_JIT_HD void mov(int vdst, bool lit, int reg, uint32_t bits) {
    if (!lit) {
      if (reg != vdst) o.movv(vdst, reg);
      return;
    }
    const uint32_t s = dual_inline(bits);
    o.mov(vdst, s, bits);
  }
  // VOP2 vdst = a OP b; a may be a literal, b must be a VGPR: callers arrange that
  MTGP_JIT_HD void op2(uint32_t op, int vdst, bool alit, int areg, uint32_t abits, int breg) {
    if (alit) {
      const uint32_t s = dual_inline(abits);
      o.vop2(op, vdst, s, breg, abits);
    } else {
      o.vop2(op, vdst, 256u + (uint32_t)areg, breg);
    }
  }
  // vdst = a OP b for a commutative OP (add, mul) with either operand a literal; tmp takes a
  // literal when both are
  MTGP_JIT_HD void comm(uint32_t op, int vdst, bool alit, int areg, uint32_t abits, bool blit, int breg,
                        uint32_t bbits, int tmp) {
    if (alit && blit) {
      mov(tmp, true, 0, bbits);
      op2(op, vdst, true, 0, abits, tmp);
    } else if (blit) {
      op2(op, vdst, true, 0, bbits, areg);
    } else {
      op2(op, vdst, alit, areg, abits, breg);
    }
  }
  // vdst = a - b
  MTGP_JIT_HD void sub(int vdst, bool alit, int areg, uint32_t abits, bool blit, int breg, uint32_t bbits, int tmp) {
    if (alit && blit) {
      mov(tmp, true, 0, bbits);
      op2(kVop2Sub, vdst, true, 0, abits, tmp);
    } else if (blit) {
      op2(kVop2Subrev, vdst, true, 0, bbits, areg);  // subrev(b, a) = a - b
    } else {
      op2(kVop2Sub, vdst, alit, areg, abits, breg);
    }
  }
};

// v8 = SUB(v17) (a shared subroutine, PC-relative call)
MTGP_JIT_HD inline void dual_sub_call(JitOut& o, uint32_t target, int exec_words) {
  o.sub += exec_words;
  const uint32_t pc_next = o.base + (uint32_t)(o.n + 1) * 4u;
  const int64_t rel = (int64_t)target - (int64_t)pc_next;
  o.w(kGetpcS44);
  o.w(kAddS44);
  o.w((uint32_t)(int32_t)rel);
  o.w(rel < 0 ? kAddcS45M1 : kAddcS45Z);
  o.w(kSwappcS40);
}

// tangent of parameter j into vdst: (v25 == j) ? 1.0 : 0.0
MTGP_JIT_HD inline void dual_param_tangent(JitOut& o, int vdst, int j) {
  const uint32_t src0 = j == 0 ? kInlZero : (j <= 64 ? 128u + (uint32_t)j : kJitSrcLiteral);
  o.w(0x7C000000u | kVopcEqU32 << 17 | (uint32_t)kDKk << 9 | src0);  // v_cmp_eq_u32 vcc, j, v25
  if (src0 == kJitSrcLiteral) o.w((uint32_t)j);
  o.w(0xD1000000u | (uint32_t)vdst);                                   // v_cndmask_b32_e64 vdst, 0, 1.0, vcc
  o.w(kInlZero | kInlOne << 9 | 106u << 18);
}

// vdst = cond ? (lit src1) : vsrc0 with cond = vcc (v_cndmask_b32_e64 vdst, vsrc0, src1, vcc)
MTGP_JIT_HD inline void dual_cndmask_lit(JitOut& o, int vdst, int vsrc0, uint32_t inl1) {
  o.w(0xD1000000u | (uint32_t)vdst);
  o.w((256u + (uint32_t)vsrc0) | inl1 << 9 | 106u << 18);
}

enum { kDualErrParam = -5 };

// Translate one END-terminated program (at most L instructions) in dual numbers; D data slots
// (< 8), K coefficients theta[0..K) (slots D .. D+K-1).  With `ret` the END becomes s_setpc.
MTGP_JIT_HD inline int jit_dual_program(JitOut& o, const MtgpInstr* prog, int L, int D, const float* theta, int K,
                                        bool ret = true) {
  if (D > kDualMaxData || D < 0 || K < 0) return kJitErrSlot;
  DualOut e{o};
  int sp = 0;
  int nparam = 0;  // parameter tangents materialized for the current instruction (kDP0, kDP1)
  auto V = [&](int s, bool& ok) -> DualSrc {
    if (s < D) return dual_regs(kDvData + s, kDdData + s);
    const int j = s - D;
    if (j >= K || nparam >= 2) {
      ok = false;
      return dual_regs(0, 0);
    }
    union { float f; uint32_t u; } cv;
    cv.f = theta[j];
    const int reg = nparam++ == 0 ? kDP0 : kDP1;
    dual_param_tangent(o, reg, j);
    return DualSrc{true, 0, cv.u, false, reg, 0u};
  };
  const DualSrc acc = dual_regs(kDvAcc, kDdAcc);
  auto push = [&]() -> bool {
    if (sp >= MTGP_STACK_MAX) return false;
    o.movv(kDvStack + sp, kDvAcc);
    o.movv(kDdStack + sp, kDdAcc);
    ++sp;
    return true;
  };
  // acc = x (a move of both halves)
  auto load = [&](const DualSrc& x) {
    e.mov(kDvAcc, x.vlit, x.vreg, x.vbits);
    e.mov(kDdAcc, x.dlit, x.dreg, x.dbits);
  };
  // acc = unary f(x) for the six subroutine operators and abs (x = acc for abs)
  auto unary = [&](int fn, const DualSrc& x) {
    switch (fn) {
      case MTGP_FN_SIN:
      case MTGP_FN_COS: {  // sin: (sin x, cos x * dx); cos: (cos x, -sin x * dx)
        const bool s = fn == MTGP_FN_SIN;
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        o.movv(kDT0, kJitT0);
        dual_sub_call(o, s ? kJitSinOffset : kJitCosOffset, s ? kJitSinExec : kJitCosExec);
        o.movv(kDT1, kDvAcc);  // the value
        o.movv(kJitT0, kDT0);
        dual_sub_call(o, s ? kJitCosOffset : kJitSinOffset, s ? kJitCosExec : kJitSinExec);
        int f = kDvAcc;
        if (!s) {  // -sin x (a sign flip: (-s) * dx rounds as -(s * dx))
          o.vop2(kVop2Xor, kDT0, kJitSrcLiteral, kDvAcc, 0x80000000u);
          f = kDT0;
        }
        e.comm(kVop2Mul, kDdAcc, false, f, 0u, x.dlit, x.dreg, x.dbits, kJitT1);
        o.movv(kDvAcc, kDT1);
        break;
      }
      case MTGP_FN_EXP:  // (e, e * dx)
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        dual_sub_call(o, MTGP_JIT_EXP_OFFSET, kJitExpExec);
        e.comm(kVop2Mul, kDdAcc, false, kDvAcc, 0u, x.dlit, x.dreg, x.dbits, kJitT1);
        break;
      case MTGP_FN_LOG:  // (log x, dx / x)
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        o.movv(kDT0, kJitT0);
        dual_sub_call(o, MTGP_JIT_LOG_OFFSET, kJitLogExec);
        o.movv(kDT1, kDvAcc);
        e.mov(kJitT0, x.dlit, x.dreg, x.dbits);
        o.movv(kJitT1, kDT0);
        o.blob(mtgp_jit_div_blob, MTGP_JIT_DIV_WORDS);
        o.movv(kDdAcc, kDvAcc);
        o.movv(kDvAcc, kDT1);
        break;
      case MTGP_FN_SQRT:  // (s, dx * (0.5 / s))
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        dual_sub_call(o, MTGP_JIT_SQRT_OFFSET, kJitSqrtExec);
        o.movv(kDT1, kDvAcc);
        o.mov(kJitT0, kInlHalf);
        o.movv(kJitT1, kDvAcc);
        o.blob(mtgp_jit_div_blob, MTGP_JIT_DIV_WORDS);
        e.comm(kVop2Mul, kDdAcc, x.dlit, x.dreg, x.dbits, false, kDvAcc, 0u, kDT0);
        o.movv(kDvAcc, kDT1);
        break;
      case MTGP_FN_TANH:  // (t, (dx + dx * t) * (1 - t))
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        dual_sub_call(o, MTGP_JIT_TANH_OFFSET, kJitTanhExec);
        e.comm(kVop2Mul, kDT0, x.dlit, x.dreg, x.dbits, false, kDvAcc, 0u, kJitT1);
        e.comm(kVop2Add, kDT0, x.dlit, x.dreg, x.dbits, false, kDT0, 0u, kJitT1);
        e.op2(kVop2Sub, kDT1, true, 0, 0x3f800000u, kDvAcc);
        o.vop2(kVop2Mul, kDdAcc, 256u + (uint32_t)kDT0, kDT1);
        break;
      default: {  // abs of acc: (|x|, sign(x) * dx), jnp.sign keeping +-0 and NaN
        o.w(0x7C000000u | kVopcGtF32 << 17 | (uint32_t)kDvAcc << 9 | kInlZero);  // v_cmp_gt_f32 vcc, 0, v8 (x < 0)
        dual_cndmask_lit(o, kDT0, kDvAcc, kInlMinusOne);
        o.w(0x7C000000u | kVopcLtF32 << 17 | (uint32_t)kDvAcc << 9 | kInlZero);  // v_cmp_lt_f32 vcc, 0, v8 (x > 0)
        dual_cndmask_lit(o, kDT0, kDT0, kInlOne);
        o.vop2(kVop2Mul, kDdAcc, 256u + (uint32_t)kDT0, kDdAcc);
        o.blob(mtgp_jit_abs_blob, MTGP_JIT_ABS_WORDS);
        break;
      }
    }
  };
  // acc = x OP y, OP one of add / sub / mul / div (d_add, d_sub, d_mul, d_div)
  auto binop = [&](int fn, const DualSrc& x, const DualSrc& y) {
    switch (fn) {
      case MTGP_FN_ADD:
        e.comm(kVop2Add, kDdAcc, x.dlit, x.dreg, x.dbits, y.dlit, y.dreg, y.dbits, kJitT1);
        e.comm(kVop2Add, kDvAcc, x.vlit, x.vreg, x.vbits, y.vlit, y.vreg, y.vbits, kJitT0);
        break;
      case MTGP_FN_SUB:
        e.sub(kDdAcc, x.dlit, x.dreg, x.dbits, y.dlit, y.dreg, y.dbits, kJitT1);
        e.sub(kDvAcc, x.vlit, x.vreg, x.vbits, y.vlit, y.vreg, y.vbits, kJitT0);
        break;
      case MTGP_FN_MUL:  // d = dx * y + x * dy, then v = x * y
        e.comm(kVop2Mul, kDT0, x.dlit, x.dreg, x.dbits, y.vlit, y.vreg, y.vbits, kJitT0);
        e.comm(kVop2Mul, kDT1, x.vlit, x.vreg, x.vbits, y.dlit, y.dreg, y.dbits, kJitT0);
        o.vop2(kVop2Add, kDdAcc, 256u + (uint32_t)kDT0, kDT1);
        e.comm(kVop2Mul, kDvAcc, x.vlit, x.vreg, x.vbits, y.vlit, y.vreg, y.vbits, kJitT0);
        break;
      default: {  // q = x / y; d = (dx - q * dy) / y
        e.mov(kJitT0, x.vlit, x.vreg, x.vbits);
        e.mov(kJitT1, y.vlit, y.vreg, y.vbits);
        o.blob(mtgp_jit_div_blob, MTGP_JIT_DIV_WORDS);  // v8 = v17 / v18 (v17, v18 kept)
        o.movv(kDT1, kDvAcc);
        e.comm(kVop2Mul, kDT0, false, kDvAcc, 0u, y.dlit, y.dreg, y.dbits, kJitT0);
        e.sub(kJitT0, x.dlit, x.dreg, x.dbits, false, kDT0, 0u, kJitT0);
        o.blob(mtgp_jit_div_blob, MTGP_JIT_DIV_WORDS);  // (dx - q dy) / y (v18 = y still)
        o.movv(kDdAcc, kDvAcc);
        o.movv(kDvAcc, kDT1);
        break;
      }
    }
  };
  for (int i = 0; i < L; ++i) {
    const uint32_t w = prog[i].op;
    const uint32_t code = w >> MTGP_OP_SHIFT, ax = w & 0xffffffu;
    union { float f; uint32_t u; } cv;
    cv.f = prog[i].imm;
    const uint32_t ib = cv.u;
    const int sib = (int)(ib / MTGP_SLOT_BYTES), sax = (int)(ax / MTGP_SLOT_BYTES);
    const DualSrc c = DualSrc{true, 0, ib, true, 0, 0u};
    bool ok = true;
    nparam = 0;
    int fam = -1, kind = -1;
    switch (code) {
      case MTGP_OP_END:
        if (ret) o.w(kSetpcS30);
        return kJitOk;
      case MTGP_OP_LDC: load(c); continue;
      case MTGP_OP_LDCP: if (!push()) return kJitErrStack; load(c); continue;
      case MTGP_OP_LDV: { const DualSrc x = V(sib, ok); if (!ok) return kDualErrParam; load(x); continue; }
      case MTGP_OP_LDVP: {
        if (!push()) return kJitErrStack;
        const DualSrc x = V(sib, ok);
        if (!ok) return kDualErrParam;
        load(x);
        continue;
      }
      case MTGP_OP_SIN: unary(MTGP_FN_SIN, acc); continue;
      case MTGP_OP_COS: unary(MTGP_FN_COS, acc); continue;
      case MTGP_OP_EXP: unary(MTGP_FN_EXP, acc); continue;
      case MTGP_OP_LOG: unary(MTGP_FN_LOG, acc); continue;
      case MTGP_OP_SQRT: unary(MTGP_FN_SQRT, acc); continue;
      case MTGP_OP_TANH: unary(MTGP_FN_TANH, acc); continue;
      case MTGP_OP_ABS: unary(MTGP_FN_ABS, acc); continue;
      case MTGP_OP_SINV: case MTGP_OP_COSV: case MTGP_OP_SINVP: case MTGP_OP_COSVP: {
        if ((code == MTGP_OP_SINVP || code == MTGP_OP_COSVP) && !push()) return kJitErrStack;
        const DualSrc x = V(sib, ok);
        if (!ok) return kDualErrParam;
        unary(code == MTGP_OP_SINV || code == MTGP_OP_SINVP ? MTGP_FN_SIN : MTGP_FN_COS, x);
        continue;
      }
#define MTGP_DJ_FAM(F, I)                                 \
      case MTGP_OP_##F##C: fam = I; kind = 0; break;      \
      case MTGP_OP_##F##V: fam = I; kind = 1; break;      \
      case MTGP_OP_##F##S: fam = I; kind = 2; break;
      MTGP_DJ_FAM(ADD, 0)
      MTGP_DJ_FAM(SUB, 1)
      MTGP_DJ_FAM(RSUB, 2)
      MTGP_DJ_FAM(MUL, 3)
      MTGP_DJ_FAM(DIV, 4)
      MTGP_DJ_FAM(RDIV, 5)
#undef MTGP_DJ_FAM
#define MTGP_DJ_VC(F, I)                                  \
      case MTGP_OP_VC_##F: fam = I; kind = 3; break;      \
      case MTGP_OP_VCP_##F: fam = I; kind = 4; break;
      MTGP_DJ_VC(ADD, 0)
      MTGP_DJ_VC(SUB, 1)
      MTGP_DJ_VC(RSUB, 2)
      MTGP_DJ_VC(MUL, 3)
      MTGP_DJ_VC(DIV, 4)
      MTGP_DJ_VC(RDIV, 5)
#undef MTGP_DJ_VC
#define MTGP_DJ_VV(F, I)                                  \
      case MTGP_OP_VV_##F: fam = I; kind = 5; break;      \
      case MTGP_OP_VVP_##F: fam = I; kind = 6; break;
      MTGP_DJ_VV(ADD, 0)
      MTGP_DJ_VV(SUB, 1)
      MTGP_DJ_VV(MUL, 3)
      MTGP_DJ_VV(DIV, 4)
#undef MTGP_DJ_VV
      default:
        return kJitErrOpcode;
    }
    // family f in (ADD, SUB, RSUB, MUL, DIV, RDIV): d_fam(f, x, y), the R* forms swap the operands
    const int base_fn = fam == 0 ? MTGP_FN_ADD : fam <= 2 ? MTGP_FN_SUB : fam == 3 ? MTGP_FN_MUL : MTGP_FN_DIV;
    const bool rev = fam == 2 || fam == 5;
    DualSrc x, y;
    if (kind <= 2) {  // acc OP {c, V(ib), pop}
      x = acc;
      if (kind == 0) y = c;
      else if (kind == 1) y = V(sib, ok);
      else {
        if (sp <= 0) return kJitErrStack;
        --sp;
        y = dual_regs(kDvStack + sp, kDdStack + sp);
      }
    } else if (kind <= 4) {  // V(ax) OP c, optional push first
      if (kind == 4 && !push()) return kJitErrStack;
      x = V(sax, ok);
      y = c;
    } else {  // V(ib) OP V(ax)
      if (kind == 6 && !push()) return kJitErrStack;
      x = V(sib, ok);
      y = V(sax, ok);
    }
    if (!ok) return kDualErrParam;
    if (rev) { const DualSrc t = x; x = y; y = t; }
    binop(base_fn, x, y);
  }
  return kJitErrNoEnd;
}

// words of one dual unit (< 0: untranslatable)
MTGP_JIT_HD inline int jit_dual_words(const MtgpInstr* prog, int L, int D, const float* theta, int K) {
  JitOut o{nullptr, 0};
  const int rc = jit_dual_program(o, prog, L, D, theta, K);
  return rc < 0 ? rc : o.n;
}

}  // namespace mtgp

#endif  // MTGP_JIT_DUAL_H
