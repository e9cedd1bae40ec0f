// mtgp_jit.h -- program JIT: flattened MtgpInstr programs -> straight-line gfx950 machine code.
//
// The interpreter (mtgp_kernels.hip run_prog) pays a scalar fetch + dispatch-tree walk per
// program instruction (~50 SIMD cycles); the programs are fixed for a whole
// population evaluation (800 RK4 stages at C3), so they are translated once per flattened
// population into machine code the evaluator calls with s_swappc_b64.  Each program
// instruction becomes 1-3 VOP1/VOP2 words (operands straight from registers: the data
// vector and the operand stack live in VGPRs, the stack depth is resolved at translation
// time), sin/cos/division copy the templates of mtgp_jit_blobs.h.  Results are
// bit-identical to the interpreter: every IEEE operation has the same operands in the same
// order; the templates (sin, cos, exp, log, tanh, sqrt as shared subroutines, abs and the
// division inline) follow include/mtgp_f32math.h op for op, special cases included, so every
// opcode of the node library translates.  s[32:33] (fallback lanes for the evaluator's
// interpreter re-run) stays part of the ABI but no template sets it.
//
// Register ABI of a generated program (the evaluator's call site pins these):
//   v0-v7    data slots 0-7 (read only)          v8      accumulator = result
//   v9-v16   operand stack (depth <= 8)          v17-v25 template / unit temporaries
//   s[30:31] return address (s_swappc_b64)       s[32:33] fallback lanes (OR-accumulated)
//   s[34:45] template temporaries, the sin/cos subroutine return address s[40:41] and
//            target s[44:45], the unit's lane mask s[42:43]; vcc
//   exec     restored (the sin/cos subroutines mask their slow-reduction blocks)
// The host ABI (mtgp.h mtgp_jit_*) places the code in executable device memory.
#ifndef MTGP_JIT_H
#define MTGP_JIT_H

#include <stdint.h>
#include "mtgp.h"
#include "mtgp_jit_blobs.h"

#if defined(__HIPCC__)
#define MTGP_JIT_HD __host__ __device__
#else
#define MTGP_JIT_HD
#endif

namespace mtgp {

constexpr int kJitData = 0, kJitAcc = 8, kJitStack = 9, kJitT0 = 17, kJitT1 = 18;
constexpr int kJitMaxData = 8;
// LDS-data mode (the wide-state SR kernel, data vector = the LDS stage vector): v0 holds this
// lane's LDS byte address of slot 0 (slot s at +s * MTGP_SLOT_BYTES); a program first loads the
// first kJitPreSlots distinct slots it reads into v26.. (all loads in flight, one wait), slots
// beyond that are loaded at their use into v42 / v43.
enum { kJitModeRegs = 0, kJitModeLds = 1 };
constexpr int kJitLdsAddr = 0, kJitPre = 26, kJitPreSlots = 16, kJitLoadTmp = 42;
constexpr uint32_t kDsReadB32 = 0xd86c0000u;   // ds_read_b32 (word 0; | offset)
// ds_read2st64_b32 (word 0; | offset1 << 8 | offset0, in units of 64 dwords = one data slot):
// two preloads into an even-aligned register pair with one instruction (round 4: the preloads were
// a quarter of the wide-state SR code, whose working set outgrew the L2)
constexpr uint32_t kDsRead2St64B32 = 0xd8700000u;
// preload instructions (= words / 2) of n preloaded slots: pairs, the odd one alone
MTGP_JIT_HD inline int jit_preload_instrs(int n) { return (n + 1) / 2; }
constexpr uint32_t kWaitLgkm0 = 0xbf8cc07fu;   // s_waitcnt lgkmcnt(0)
constexpr uint32_t kJitSrcLiteral = 255u;
// VOP2 opcodes (gfx9 encoding)
constexpr uint32_t kVop2Add = 1u, kVop2Sub = 2u, kVop2Subrev = 3u, kVop2Mul = 5u;
constexpr uint32_t kSetpcS30 = 0xbe801d1eu;  // s_setpc_b64 s[30:31]
// largest translation of one program instruction (an upper bound: push + two moves + the sin template)
constexpr int kJitMaxWordsPerInstr = 1 + 4 + (MTGP_JIT_COS_WORDS > MTGP_JIT_SIN_WORDS ? MTGP_JIT_COS_WORDS : MTGP_JIT_SIN_WORDS);

// The sin / cos / exp / log / tanh / sqrt templates are shared subroutines at the start of the
// code buffer (mtgp_jit_sub_blob: one copy each, hot in the instruction cache); generated code
// calls them with a PC-relative address.
constexpr uint32_t kJitSinOffset = MTGP_JIT_SIN_OFFSET, kJitCosOffset = MTGP_JIT_COS_OFFSET;
constexpr uint32_t kJitTemplateBytes = MTGP_JIT_SUB_WORDS * 4u;
// executed words of one call of each subroutine (the schedule's cost model: the hot path up to
// the return).  Only sin / cos have out-of-line words after the return (the |x| >= 2^17 Payne-
// Hanek reduction, run only when some lane needs it); exp / log / tanh / sqrt are branch-free,
// their special ranges (exp |x| > 88.72 or NaN, log of anything but a positive normal, tanh
// |x| >= 0.625, sqrt x < 2^-96 / 0 / inf / NaN) handled by selects inside the counted words, so
// their SKIPPABLE counts are 0 (tests/test_jit.py checks these counts against the blobs)
constexpr int kJitSinExec = MTGP_JIT_SIN_WORDS - MTGP_JIT_SIN_SKIPPABLE_WORDS;
constexpr int kJitCosExec = MTGP_JIT_COS_WORDS - MTGP_JIT_COS_SKIPPABLE_WORDS;
constexpr int kJitExpExec = MTGP_JIT_EXP_WORDS - MTGP_JIT_EXP_SKIPPABLE_WORDS;
constexpr int kJitLogExec = MTGP_JIT_LOG_WORDS - MTGP_JIT_LOG_SKIPPABLE_WORDS;
constexpr int kJitTanhExec = MTGP_JIT_TANH_WORDS - MTGP_JIT_TANH_SKIPPABLE_WORDS;
constexpr int kJitSqrtExec = MTGP_JIT_SQRT_WORDS - MTGP_JIT_SQRT_SKIPPABLE_WORDS;
constexpr uint32_t kGetpcS44 = 0xbeac1c00u;     // s_getpc_b64 s[44:45]
constexpr uint32_t kAddS44 = 0x802cff2cu;       // s_add_u32 s44, s44, literal
constexpr uint32_t kAddcS45M1 = 0x822dc12du;    // s_addc_u32 s45, s45, -1
constexpr uint32_t kAddcS45Z = 0x822d802du;     // s_addc_u32 s45, s45, 0
constexpr uint32_t kSwappcS40 = 0xbea81e2cu;    // s_swappc_b64 s[40:41], s[44:45]

struct JitOut {
  uint32_t* out;  // nullptr: count only
  int n;
  int sub = 0;        // executed words of the subroutine calls emitted (cost model)
  uint32_t base = 0;  // byte offset of out[0] in the code buffer (for PC-relative calls)
  MTGP_JIT_HD void w(uint32_t v) {
    if (out) out[n] = v;
    ++n;
  }
  MTGP_JIT_HD void blob(const uint32_t* b, int len) {
    for (int i = 0; i < len; ++i) w(b[i]);
  }
  // v_mov_b32 vdst, src (src: 256 + vgpr or literal)
  MTGP_JIT_HD void mov(int vdst, uint32_t src, uint32_t lit = 0) {
    w(0x7e000000u | (uint32_t)vdst << 17 | 1u << 9 | src);
    if (src == kJitSrcLiteral) w(lit);
  }
  MTGP_JIT_HD void movv(int vdst, int vsrc) { mov(vdst, 256u + (uint32_t)vsrc); }
  MTGP_JIT_HD void movc(int vdst, uint32_t bits) { mov(vdst, kJitSrcLiteral, bits); }
  // VOP2: vdst = src0 OP vsrc1 (src0: 256 + vgpr or literal)
  MTGP_JIT_HD void vop2(uint32_t op, int vdst, uint32_t src0, int vsrc1, uint32_t lit = 0) {
    w(op << 25 | (uint32_t)vdst << 17 | (uint32_t)vsrc1 << 9 | src0);
    if (src0 == kJitSrcLiteral) w(lit);
  }
};

// Source descriptor of an operand: a VGPR or a literal constant.
struct JitSrc {
  bool lit;
  int reg;
  uint32_t bits;
};

MTGP_JIT_HD inline JitSrc jit_reg(int r) { return JitSrc{false, r, 0u}; }
MTGP_JIT_HD inline JitSrc jit_lit(uint32_t b) { return JitSrc{true, 0, b}; }

// acc = x OP y for the four IEEE operations, operand order preserved.
MTGP_JIT_HD inline void jit_binop(JitOut& o, int fn, JitSrc x, JitSrc y) {
  if (fn == MTGP_FN_DIV) {  // the template divides v17 by v18
    if (x.lit) o.movc(kJitT0, x.bits); else o.movv(kJitT0, x.reg);
    if (y.lit) o.movc(kJitT1, y.bits); else o.movv(kJitT1, y.reg);
    o.blob(mtgp_jit_div_blob, MTGP_JIT_DIV_WORDS);
    return;
  }
  // VOP2 takes a literal only as src0 and needs src1 in a VGPR
  if (y.lit && x.lit) {
    o.movc(kJitT0, y.bits);
    y = jit_reg(kJitT0);
  }
  const bool comm = fn == MTGP_FN_ADD || fn == MTGP_FN_MUL;
  const uint32_t opc = fn == MTGP_FN_ADD ? kVop2Add : fn == MTGP_FN_MUL ? kVop2Mul : kVop2Sub;
  if (y.lit) {  // x is a register: put the literal in src0
    if (comm) o.vop2(opc, kJitAcc, kJitSrcLiteral, x.reg, y.bits);  // c OP x == x OP c (commutative)
    else o.vop2(kVop2Subrev, kJitAcc, kJitSrcLiteral, x.reg, y.bits);  // x - c = subrev(c, x)
    return;
  }
  if (x.lit) o.vop2(opc, kJitAcc, kJitSrcLiteral, y.reg, x.bits);
  else o.vop2(opc, kJitAcc, 256u + (uint32_t)x.reg, y.reg);
}

// v8 = SUB(x): x into v17, then a PC-relative s_swappc_b64 into the subroutine at byte `target`
MTGP_JIT_HD inline void jit_call(JitOut& o, uint32_t target, int exec_words, JitSrc x) {
  o.sub += exec_words;
  if (x.lit) o.movc(kJitT0, x.bits); else o.movv(kJitT0, x.reg);
  // s_getpc_b64 yields the address of the next instruction: target = that + rel
  const uint32_t pc_next = o.base + (uint32_t)(o.n + 1) * 4u;
  const int64_t rel = (int64_t)target - (int64_t)pc_next;
  o.w(kGetpcS44);
  o.w(kAddS44);
  o.w((uint32_t)(int32_t)rel);
  o.w(rel < 0 ? kAddcS45M1 : kAddcS45Z);
  o.w(kSwappcS40);
}
MTGP_JIT_HD inline void jit_trig(JitOut& o, bool is_sin, JitSrc x) {
  jit_call(o, is_sin ? kJitSinOffset : kJitCosOffset, is_sin ? kJitSinExec : kJitCosExec, x);
}

enum { kJitOk = 0, kJitErrOpcode = -1, kJitErrSlot = -2, kJitErrStack = -3, kJitErrNoEnd = -4 };

// Translate one END-terminated program (at most L instructions) into o; with `ret` the END
// becomes s_setpc_b64 s[30:31], otherwise nothing (the code falls through).  Returns kJitOk
// or a negative kJitErr* code.
// LDS-data mode in parts (the pipelined units, jit_unit_lds): part 1 emits only the program's
// preloads (into v[pre_base..]; *npre_out = their number), part 2 only the rest -- the wait for
// them (s_waitcnt lgkmcnt(wait_n): later loads may stay in flight) and the body; part 0 is both.
constexpr int kJitPreB = 44;  // the second preload register set (v44..v59) of a pipelined unit
MTGP_JIT_HD inline uint32_t jit_wait_lgkm(int n) { return kWaitLgkm0 | (uint32_t)(n > 15 ? 15 : n) << 8; }

// sp_init: operand-stack depth before prog[0] (the per-instruction sizing of k_flatten_wave
// translates a pop on its own with one element on the stack).
// Part 3 (the wave-parallel emitter, k_jit_emit_waves_lds): the body of a piece of a program only
// -- no preloads, no wait -- with the whole program's preload table given (pre_ext[0..npre_ext)).
MTGP_JIT_HD inline int jit_program(JitOut& o, const MtgpInstr* prog, int L, bool ret, int mode = kJitModeRegs,
                                   int part = 0, int pre_base = kJitPre, int wait_n = 0, int* npre_out = nullptr,
                                   int sp_init = 0, const int* pre_ext = nullptr, int npre_ext = 0,
                                   int remap_slot = -1, int remap_reg = 0) {
  int sp = sp_init;
  int pre[kJitPreSlots];
  int npre = 0;
  if (mode == kJitModeLds && pre_ext) {
    npre = npre_ext < kJitPreSlots ? npre_ext : kJitPreSlots;
    for (int q = 0; q < npre; ++q) pre[q] = pre_ext[q];
  } else if (mode == kJitModeLds) {  // preload the first kJitPreSlots distinct data slots the program reads
    for (int i = 0; i < L; ++i) {
      const uint32_t w = prog[i].op, code = w >> MTGP_OP_SHIFT;
      if (code == MTGP_OP_END) break;
      union { float f; uint32_t u; } cv;
      cv.f = prog[i].imm;
      int cand[2], nc = 0;
      switch (code) {
        case MTGP_OP_LDV: case MTGP_OP_LDVP: case MTGP_OP_SINV: case MTGP_OP_COSV: case MTGP_OP_SINVP:
        case MTGP_OP_COSVP: case MTGP_OP_ADDV: case MTGP_OP_SUBV: case MTGP_OP_RSUBV: case MTGP_OP_MULV:
        case MTGP_OP_DIVV: case MTGP_OP_RDIVV:
          cand[nc++] = (int)(cv.u / MTGP_SLOT_BYTES); break;
        case MTGP_OP_VV_ADD: case MTGP_OP_VV_SUB: case MTGP_OP_VV_MUL: case MTGP_OP_VV_DIV: case MTGP_OP_VVP_ADD:
        case MTGP_OP_VVP_SUB: case MTGP_OP_VVP_MUL: case MTGP_OP_VVP_DIV:
          cand[nc++] = (int)(cv.u / MTGP_SLOT_BYTES);
          cand[nc++] = (int)((w & 0xffffffu) / MTGP_SLOT_BYTES); break;
        case MTGP_OP_VC_ADD: case MTGP_OP_VC_SUB: case MTGP_OP_VC_RSUB: case MTGP_OP_VC_MUL: case MTGP_OP_VC_DIV:
        case MTGP_OP_VC_RDIV: case MTGP_OP_VCP_ADD: case MTGP_OP_VCP_SUB: case MTGP_OP_VCP_RSUB: case MTGP_OP_VCP_MUL:
        case MTGP_OP_VCP_DIV: case MTGP_OP_VCP_RDIV:
          cand[nc++] = (int)((w & 0xffffffu) / MTGP_SLOT_BYTES); break;
        default: break;
      }
      for (int k = 0; k < nc; ++k) {
        if (cand[k] >= MTGP_MAX_DATA) return kJitErrSlot;
        bool have = false;
        for (int q = 0; q < npre; ++q) have = have || pre[q] == cand[k];
        if (!have && npre < kJitPreSlots) pre[npre++] = cand[k];
      }
    }
  }
  if (mode == kJitModeLds) {
    if (npre_out) *npre_out = npre;
    if (part != 2 && part != 3) {
      for (int q = 0; q < npre; q += 2) {  // rank pairs (q, q + 1) into v[pre_base + q : + 1]
        if (q + 1 < npre) o.w(kDsRead2St64B32 | (uint32_t)pre[q + 1] << 8 | (uint32_t)pre[q]);
        else o.w(kDsReadB32 | (uint32_t)(pre[q] * (int)MTGP_SLOT_BYTES));
        o.w((uint32_t)(pre_base + q) << 24 | (uint32_t)kJitLdsAddr);
      }
    }
    if (part == 1) return kJitOk;
    // part 2: wait_n = the slots the NEXT program preloads after these (its instructions may stay in flight)
    if (npre > 0 && part != 3) o.w(part == 2 ? jit_wait_lgkm(jit_preload_instrs(wait_n)) : kWaitLgkm0);
  }
  // register holding data slot s: v0-v7 (register mode) or its preload / a load at the use
  auto vslot = [&](int s_, int tmp) -> int {
    if (mode != kJitModeLds) return s_ == remap_slot ? remap_reg : kJitData + s_;  // (remap: jit_put_remap)
    for (int q = 0; q < npre; ++q)
      if (pre[q] == s_) return pre_base + q;
    o.w(kDsReadB32 | (uint32_t)(s_ * (int)MTGP_SLOT_BYTES));
    o.w((uint32_t)tmp << 24 | (uint32_t)kJitLdsAddr);
    o.w(kWaitLgkm0);
    return tmp;
  };
  const int max_slot = mode == kJitModeLds ? MTGP_MAX_DATA : kJitMaxData;
  for (int i = 0; i < L; ++i) {
    const uint32_t w = prog[i].op;
    const uint32_t code = w >> MTGP_OP_SHIFT, ax = w & 0xffffffu;
    union { float f; uint32_t u; } cv;
    cv.f = prog[i].imm;
    const uint32_t ib = cv.u;
    const int sib = (int)(ib / MTGP_SLOT_BYTES), sax = (int)(ax / MTGP_SLOT_BYTES);
    auto push = [&]() -> bool {
      if (sp >= MTGP_STACK_MAX) return false;
      o.movv(kJitStack + sp, kJitAcc);
      ++sp;
      return true;
    };
    const JitSrc acc = jit_reg(kJitAcc), c = jit_lit(ib);
    // which operand kinds this opcode reads (checked below)
    bool uses_ib_slot = false, uses_ax_slot = false, ok = true;
    int fam = -1, kind = -1;  // family ADD SUB RSUB MUL DIV RDIV; kind 0 C, 1 V, 2 S
    switch (code) {
      case MTGP_OP_END:
        if (ret) o.w(kSetpcS30);
        return kJitOk;
      case MTGP_OP_LDC: o.movc(kJitAcc, ib); continue;
      case MTGP_OP_LDCP: ok = push(); o.movc(kJitAcc, ib); break;
      case MTGP_OP_LDV: uses_ib_slot = true; if (sib >= max_slot) return kJitErrSlot; o.movv(kJitAcc, vslot(sib, kJitLoadTmp)); continue;
      case MTGP_OP_LDVP: if (sib >= max_slot) return kJitErrSlot; ok = push(); o.movv(kJitAcc, vslot(sib, kJitLoadTmp)); break;
      case MTGP_OP_SIN: jit_trig(o, true, acc); continue;
      case MTGP_OP_COS: jit_trig(o, false, acc); continue;
      case MTGP_OP_EXP: jit_call(o, MTGP_JIT_EXP_OFFSET, kJitExpExec, acc); continue;
      case MTGP_OP_LOG: jit_call(o, MTGP_JIT_LOG_OFFSET, kJitLogExec, acc); continue;
      case MTGP_OP_TANH: jit_call(o, MTGP_JIT_TANH_OFFSET, kJitTanhExec, acc); continue;
      case MTGP_OP_SQRT: jit_call(o, MTGP_JIT_SQRT_OFFSET, kJitSqrtExec, acc); continue;
      case MTGP_OP_ABS: o.blob(mtgp_jit_abs_blob, MTGP_JIT_ABS_WORDS); continue;
      case MTGP_OP_SINV: case MTGP_OP_COSV: case MTGP_OP_SINVP: case MTGP_OP_COSVP:
        if (sib >= max_slot) return kJitErrSlot;
        if (code == MTGP_OP_SINVP || code == MTGP_OP_COSVP) ok = push();
        jit_trig(o, code == MTGP_OP_SINV || code == MTGP_OP_SINVP, jit_reg(vslot(sib, kJitLoadTmp)));
        break;
#define MTGP_JIT_FAM(F, I)                                                  \
      case MTGP_OP_##F##C: fam = I; kind = 0; break;                        \
      case MTGP_OP_##F##V: fam = I; kind = 1; uses_ib_slot = true; break;   \
      case MTGP_OP_##F##S: fam = I; kind = 2; break;
      MTGP_JIT_FAM(ADD, 0)
      MTGP_JIT_FAM(SUB, 1)
      MTGP_JIT_FAM(RSUB, 2)
      MTGP_JIT_FAM(MUL, 3)
      MTGP_JIT_FAM(DIV, 4)
      MTGP_JIT_FAM(RDIV, 5)
#undef MTGP_JIT_FAM
#define MTGP_JIT_VC(F, I) \
      case MTGP_OP_VC_##F: fam = I; kind = 3; uses_ax_slot = true; break; \
      case MTGP_OP_VCP_##F: fam = I; kind = 4; uses_ax_slot = true; break;
      MTGP_JIT_VC(ADD, 0)
      MTGP_JIT_VC(SUB, 1)
      MTGP_JIT_VC(RSUB, 2)
      MTGP_JIT_VC(MUL, 3)
      MTGP_JIT_VC(DIV, 4)
      MTGP_JIT_VC(RDIV, 5)
#undef MTGP_JIT_VC
#define MTGP_JIT_VV(F, I) \
      case MTGP_OP_VV_##F: fam = I; kind = 5; uses_ib_slot = uses_ax_slot = true; break; \
      case MTGP_OP_VVP_##F: fam = I; kind = 6; uses_ib_slot = uses_ax_slot = true; break;
      MTGP_JIT_VV(ADD, 0)
      MTGP_JIT_VV(SUB, 1)
      MTGP_JIT_VV(MUL, 3)
      MTGP_JIT_VV(DIV, 4)
#undef MTGP_JIT_VV
      default:
        return kJitErrOpcode;
    }
    if (!ok) return kJitErrStack;
    if (fam < 0) continue;  // handled above
    if ((uses_ib_slot && sib >= max_slot) || (uses_ax_slot && sax >= max_slot)) return kJitErrSlot;
    // family f in (ADD, SUB, RSUB, MUL, DIV, RDIV): R* forms swap the operands
    const int base_fn = fam == 0 ? MTGP_FN_ADD : fam <= 2 ? MTGP_FN_SUB : fam == 3 ? MTGP_FN_MUL : MTGP_FN_DIV;
    const bool rev = fam == 2 || fam == 5;
    JitSrc x, y;
    if (kind <= 2) {  // acc OP {c, V(ib), pop}
      x = acc;
      if (kind == 0) y = c;
      else if (kind == 1) y = jit_reg(vslot(sib, kJitLoadTmp));
      else {
        if (sp <= 0) return kJitErrStack;
        --sp;
        y = jit_reg(kJitStack + sp);
      }
    } else if (kind <= 4) {  // V(ax) OP c, optional push first
      if (kind == 4 && !push()) return kJitErrStack;
      x = jit_reg(vslot(sax, kJitLoadTmp));
      y = c;
    } else {  // V(ib) OP V(ax)
      if (kind == 6 && !push()) return kJitErrStack;
      x = jit_reg(vslot(sib, kJitLoadTmp));
      y = jit_reg(vslot(sax, kJitLoadTmp + 1));
    }
    if (rev) { const JitSrc t = x; x = y; y = t; }
    jit_binop(o, base_fn, x, y);
  }
  return kJitErrNoEnd;
}

// Operand-stack effect of one instruction in jit_program: +1 where it calls push() (LDCP, LDVP,
// SINVP, COSVP, VCP_*, VVP_*), -1 for the stack-operand forms (kind 2: ADDS .. RDIVS), else 0.
MTGP_JIT_HD inline int jit_stack_delta(uint32_t code) {
  switch (code) {
    case MTGP_OP_LDCP: case MTGP_OP_LDVP: case MTGP_OP_SINVP: case MTGP_OP_COSVP:
    case MTGP_OP_VCP_ADD: case MTGP_OP_VCP_SUB: case MTGP_OP_VCP_RSUB: case MTGP_OP_VCP_MUL: case MTGP_OP_VCP_DIV:
    case MTGP_OP_VCP_RDIV: case MTGP_OP_VVP_ADD: case MTGP_OP_VVP_SUB: case MTGP_OP_VVP_MUL: case MTGP_OP_VVP_DIV:
      return 1;
    case MTGP_OP_ADDS: case MTGP_OP_SUBS: case MTGP_OP_RSUBS: case MTGP_OP_MULS: case MTGP_OP_DIVS: case MTGP_OP_RDIVS:
      return -1;
    default:
      return 0;
  }
}

// One callable program: number of 32-bit code words (out == nullptr: count only) or < 0.
MTGP_JIT_HD inline int jit_translate(const MtgpInstr* prog, int L, uint32_t* out, uint32_t base = kJitTemplateBytes,
                                     int mode = kJitModeRegs) {
  JitOut o{out, 0};
  o.base = base;
  const int rc = jit_program(o, prog, L, true, mode);
  return rc < 0 ? rc : o.n;
}

// Estimated issue cost of one program (schedule weight): code words actually executed, i.e.
// the program's own words plus the subroutines' executed words (JitOut::sub).
MTGP_JIT_HD inline int jit_cost(const MtgpInstr* prog, int L) {
  JitOut o{nullptr, 0};
  const int rc = jit_program(o, prog, L, true);
  if (rc < 0) return rc;
  const int w = o.n + o.sub;
  return w > 1 ? w : 1;
}

// ---- per-wave units ------------------------------------------------------------------
// The evaluator calls program j for all G individuals of its wave at once: one unit of code per
// (wave, program) runs the G individuals' programs back to back with full exec; after group
// g > 0 a v_cndmask keeps group g's lanes (g*Rp .. g*Rp+Rp-1) from the new value and the
// other lanes from the running result (v25), so v8 ends with every lane's own individual's
// value -- one call instead of G, no selects at the call site.  (Variants that switched exec
// per group, or returned several programs' results in v25-v28, measured slower: DESIGN.md.)
constexpr int kJitKeep = 25;
constexpr uint32_t kMovS42 = 0xbeaa00ffu;   // s_mov_b32 s42, literal
constexpr uint32_t kMovS43 = 0xbeab00ffu;   // s_mov_b32 s43, literal
constexpr uint32_t kSelLo = 0xd1000008u;    // v_cndmask_b32_e64 v8, v25, v8, s[42:43]
constexpr uint32_t kSelHi = 0x00aa1119u;
constexpr uint32_t kLshlS42 = 0x8eaa002au;  // s_lshl_b64 s[42:43], s[42:43], inline constant (| (128 + n) << 8)
constexpr uint32_t kBfmS42 = 0x91aa0000u;   // s_bfm_b64 s[42:43], width, offset (inline constants)

// The merge of the G groups' results of a unit (round 3; was 7 words per group g > 0): the
// running result lives in v25 -- `v_mov v25, v8` after group 0 (emitted before group 1's program),
// `v_cndmask v25, v25, v8, s[42:43]` after every later group, except that the LAST group selects
// into v8 (`v_cndmask v8, v25, v8, s[42:43]`), where the unit's result is expected.  The lane
// mask of group g's Rp lanes: group 1 forms it with one s_bfm_b64 (Rp ones at bit Rp), group
// g >= 2 shifts the previous one by Rp (s[42:43] survives the programs: the sin/cos/div templates
// never write it).  Words per group: 4 for g = 1, 3 for g >= 2 -- at C5 (8 groups per unit) the
// literal-move merges were a quarter of the code and most of the SALU instructions.
constexpr uint32_t kSelLoRun = 0xd1000019u;  // v_cndmask_b32_e64 v25, v25, v8, s[42:43] (+ kSelHi)
MTGP_JIT_HD inline int jit_merge_words(int g) { return g <= 0 ? 0 : (g == 1 ? 4 : 3); }
MTGP_JIT_HD inline bool jit_merge_keep(int g) { return g == 1; }  // `v_mov v25, v8` before group g's program
MTGP_JIT_HD inline void jit_merge_tail(JitOut& o, int g, int Rp, bool last) {
  const uint32_t r = (uint32_t)(128 + Rp);  // inline integer constant Rp (1 .. 32: g > 0 implies Rp < 64)
  o.w(g == 1 ? (kBfmS42 | r << 8 | r) : (kLshlS42 | r << 8));
  o.w(last ? kSelLo : kSelLoRun);
  o.w(kSelHi);
}

// ---- role chains (ABI v13, MtgpJitChain) ---------------------------------------------------
// A role that runs several programs back to back (the state equations of a dynamic policy, the
// n_var trees of SR) is ONE call: unit j with bit j of chain.next set ends by copying its result
// to v(26 + k) (k = its position in the chain) and falls through into unit j + 1, which is laid
// out right behind it (no alignment padding); the last unit of the chain copies its result too
// and returns.  With bit j of chain.cond also set, unit j continues only when the call site set
// s46 != 0 and returns otherwise; the unit after it (the save-point readout) then leaves its
// result in v8 as a plain unit does.  Per chained call one fetch redirect replaces a return + a
// call (two), and the call-site bookkeeping of the extra calls disappears.
//
// LDS store chains (ABI v14, chain.store = S > 0; the wide-state SR kernel in LDS-data mode):
// every unit j ends with `ds_write_b32 v1, v8 offset:j*256` -- its result into the caller's LDS
// output vector, v1 = that vector's slot-0 address -- and falls through into unit j + 1 unless
// j + 1 is a multiple of S (or the last program): the S components a wave owns are one call.
constexpr int kJitChainOut = 26, kJitChainMax = 4;
constexpr uint32_t kDsWriteV1V8 = 0xd81a0000u;  // ds_write_b32 v1, v8 (word 0; | offset)
constexpr uint32_t kDsWriteV1V8Hi = 0x00000801u;
constexpr uint32_t kCmpS46Zero = 0xbf06802eu;  // s_cmp_eq_u32 s46, 0
constexpr uint32_t kBranchScc0Skip1 = 0xbf840001u;  // s_cbranch_scc0 +1 (over the s_setpc)

// position of unit j in its chain (0 for the first)
MTGP_JIT_HD inline int jit_chain_pos(uint32_t next, int j) {
  int k = 0;
  if (j >= 32) return 0;
  while (j - k - 1 >= 0 && ((next >> (j - k - 1)) & 1u)) ++k;
  return k;
}

// unit j of an LDS store chain falls through into unit j + 1
MTGP_JIT_HD inline bool jit_store_cont(uint32_t store, int n_prog, int j) {
  return store > 0u && ((uint32_t)(j + 1) % store) != 0u && j + 1 < n_prog;
}

// the end of unit j: s_setpc (plain unit), or the chain epilogue
MTGP_JIT_HD inline void jit_unit_end(JitOut& o, uint32_t next, uint32_t cond, int j, uint32_t store = 0u,
                                     int n_prog = 0) {
  if (store > 0u) {  // LDS store chain
    o.w(kDsWriteV1V8 | ((uint32_t)j * (uint32_t)MTGP_SLOT_BYTES & 0xffffu));
    o.w(kDsWriteV1V8Hi);
    if (!jit_store_cont(store, n_prog, j)) {
      o.w(kWaitLgkm0);
      o.w(kSetpcS30);
    }
    return;
  }
  if (j >= 32) { o.w(kSetpcS30); return; }  // chains cover the first 32 programs
  const bool cont = (next >> j) & 1u;
  const bool after = j > 0 && ((next >> (j - 1)) & 1u);
  const bool tail_of_cond = after && ((cond >> (j - 1)) & 1u);  // the optional continuation: result stays in v8
  if ((cont || after) && !tail_of_cond) o.movv(kJitChainOut + jit_chain_pos(next, j), kJitAcc);
  if (!cont) {
    o.w(kSetpcS30);
    return;
  }
  if ((cond >> j) & 1u) {  // continue only when s46 != 0
    o.w(kCmpS46Zero);
    o.w(kBranchScc0Skip1);
    o.w(kSetpcS30);
  }
}

// words of the end of unit j (jit_unit_end)
MTGP_JIT_HD inline int jit_unit_end_words(uint32_t next, uint32_t cond, int j, uint32_t store = 0u, int n_prog = 0) {
  JitOut o{nullptr, 0};
  jit_unit_end(o, next, cond, j, store, n_prog);
  return o.n;
}

// unit j falls through into unit j + 1, which is laid out right behind it (no alignment padding)
MTGP_JIT_HD inline bool jit_unit_packed(uint32_t next, int j, uint32_t store = 0u, int n_prog = 0) {
  if (store > 0u) return jit_store_cont(store, n_prog, j);
  return j < 32 && ((next >> j) & 1u) != 0u;
}

// Put chains (ABI v18, MtgpJitChain.put): a unit p with bit p of `put` passes its result on AS a
// data slot -- the units it falls through into (within its chain) read data slot put_slot from
// v(26 + position of p), where the chain epilogue of p leaves it, instead of from v[put_slot].
// (The fixed-step dynamic policy: readout -> the state programs read u = the readout's result.)
// -> the register, or -1 when unit j reads its data slots plainly.
MTGP_JIT_HD inline int jit_put_remap(uint32_t next, uint32_t put, int j) {
  if (put == 0u || j <= 0 || j >= 32) return -1;
  for (int p = j - 1; p >= 0 && ((next >> p) & 1u); --p)
    if ((put >> p) & 1u) return kJitChainOut + jit_chain_pos(next, p);
  return -1;
}

// LDS-data units are software-pipelined: the preloads of group g + 1's program are issued before
// group g's body runs (alternating register sets v26.. / v44..), so the LDS latency of one
// program hides behind the previous one's arithmetic.  Layout: [P_0] then per group g
// [P_(g+1)] [v_mov v25, v8 (g > 0)] [wait for P_g + body_g] [select (g > 0)]; per group the same
// words as the plain layout (preload, wait, body), only reordered, so group g (> 0) starts
// jit_preload_words(prog_g) words after its plain position.  Register set of group g's preloads:
MTGP_JIT_HD inline int jit_pre_set(int g) { return (g & 1) ? kJitPreB : kJitPre; }

// words of the preloads of one LDS-mode program (< 0: untranslatable)
MTGP_JIT_HD inline int jit_preload_words(const MtgpInstr* prog, int L) {
  JitOut o{nullptr, 0};
  const int rc = jit_program(o, prog, L, false, kJitModeLds, 1);
  return rc < 0 ? rc : o.n;
}

// Region of group g of an LDS-mode unit (see above); `next` = the program of group g + 1 or null.
MTGP_JIT_HD inline int jit_lds_region(JitOut& o, const MtgpInstr* cur, const MtgpInstr* next, int L, int g) {
  if (g == 0) {
    const int rc = jit_program(o, cur, L, false, kJitModeLds, 1, jit_pre_set(0));
    if (rc < 0) return rc;
  }
  int np1 = 0;
  if (next) {
    const int rc = jit_program(o, next, L, false, kJitModeLds, 1, jit_pre_set(g + 1), 0, &np1);
    if (rc < 0) return rc;
  }
  if (jit_merge_keep(g)) o.movv(kJitKeep, kJitAcc);
  return jit_program(o, cur, L, false, kJitModeLds, 2, jit_pre_set(g), np1);
}

// Code of unit (wave, program j): individuals order[wave*G + g] (identity without a schedule).
MTGP_JIT_HD inline int jit_unit(const MtgpInstr* prog, int n_prog, int L, int P, const int32_t* order, int G, int Rp,
                                int wave, int j, uint32_t* out, uint32_t base, int mode = kJitModeRegs,
                                uint32_t next = 0u, uint32_t cond = 0u, uint32_t store = 0u, bool pipe = true,
                                uint32_t put = 0u, int put_slot = 0) {
  JitOut o{out, 0};
  o.base = base;
  for (int g = 0; g < G; ++g) {
    const int q = wave * G + g;
    if (q >= P) break;
    const int ind = order ? order[q] : q;
    const MtgpInstr* cur = prog + ((size_t)ind * n_prog + j) * L;
    int rc;
    if (mode == kJitModeLds && pipe) {
      const MtgpInstr* nxt = nullptr;
      if (g + 1 < G && q + 1 < P) nxt = prog + ((size_t)(order ? order[q + 1] : q + 1) * n_prog + j) * L;
      rc = jit_lds_region(o, cur, nxt, L, g);
    } else {
      if (jit_merge_keep(g)) o.movv(kJitKeep, kJitAcc);
      const int rr = jit_put_remap(next, put, j);
      rc = jit_program(o, cur, L, false, mode, 0, kJitPre, 0, nullptr, 0, nullptr, 0, rr < 0 ? -1 : put_slot, rr);
    }
    if (rc < 0) return rc;
    if (g > 0) jit_merge_tail(o, g, Rp, g == G - 1 || q + 1 >= P);
  }
  jit_unit_end(o, next, cond, j, store, n_prog);
  return o.n;
}

// Group g of the unit whose first schedule slot is q0 (program j): the code jit_unit emits for
// that group, written at `out` (= byte offset `base` in the buffer), plus the unit's final
// s_setpc when `last`.  jit_unit == the concatenation of its groups.
MTGP_JIT_HD inline int jit_unit_group(const MtgpInstr* prog, int n_prog, int L, const int32_t* order, int Rp, int q0,
                                      int g, int j, bool last, uint32_t* out, uint32_t base, int mode = kJitModeRegs,
                                      uint32_t next = 0u, uint32_t cond = 0u, uint32_t store = 0u,
                                      bool pipe = true, uint32_t put = 0u, int put_slot = 0) {
  JitOut o{out, 0};
  o.base = base;
  const int q = q0 + g;
  const int ind = order ? order[q] : q;
  const MtgpInstr* cur = prog + ((size_t)ind * n_prog + j) * L;
  int rc;
  if (mode == kJitModeLds && pipe) {  // (the caller placed this region jit_preload_words(g) words after the plain start)
    const MtgpInstr* nxt = nullptr;
    if (!last) nxt = prog + ((size_t)(order ? order[q + 1] : q + 1) * n_prog + j) * L;
    rc = jit_lds_region(o, cur, nxt, L, g);
  } else {
    if (jit_merge_keep(g)) o.movv(kJitKeep, kJitAcc);
    const int rr = jit_put_remap(next, put, j);
    rc = jit_program(o, cur, L, false, mode, 0, kJitPre, 0, nullptr, 0, nullptr, 0, rr < 0 ? -1 : put_slot, rr);
  }
  if (rc < 0) return rc;
  if (g > 0) jit_merge_tail(o, g, Rp, last);
  if (last) jit_unit_end(o, next, cond, j, store, n_prog);
  return o.n;
}

}  // namespace mtgp

#endif  // MTGP_JIT_H
