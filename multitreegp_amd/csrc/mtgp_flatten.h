// mtgp_flatten.h -- population tree -> straight-line accumulator program.
//
// Semantics restated from the reference interpreter (gp.py:356-388):
//   for i in 0..N-1 (ascending):  f, a, b, c = tree[i]
//       x = tree[int(a), 3]; y = tree[int(b), 3]          (value column, as updated so far)
//       tree[i, 3] = (f == 1) ? c : switch(int(f), fns, x, y, data)
//   result = tree[N-1, 3]
// * int(): f32 -> int32 truncation (saturating, NaN -> 0); negative index i -> i + N,
//   then clamped to [0, N-1] (jnp dynamic indexing); lax.switch clamps the branch index.
// * A reference to row j < i reads row j's evaluated value; a reference to j >= i reads
//   the ORIGINAL value column (row not evaluated yet in this pass).
// * Only rows reachable from the root affect the result, so a postorder walk from row N-1
//   yields bit-identical values.  Leaves (coefficients, variables, folded constants) are
//   folded into their parent instruction; constant subtrees are evaluated here with the
//   same fp32 primitives as the kernel (mtgp_f32math.h), so folding is bit-exact.
// * Binary operands are ordered by Sethi-Ullman need so the operand stack stays shallow.
//
// This header is compiled for the host (tests, CPU tooling) and for gfx950 (flatten kernel).
#pragma once
#include <stdint.h>
#include "mtgp.h"
#include "mtgp_f32math.h"

namespace mtgp {

enum : uint8_t { K_CONST = 0, K_VAR = 1, K_UNARY = 2, K_BINARY = 3 };

// operand reference: row >= 0 -> evaluated row, row == -1 -> constant `val`
struct Ref {
  int16_t row;
  float val;
};

struct RowInfo {
  uint8_t kind;
  uint8_t fn;
  uint8_t slot;      // K_VAR data slot
  uint8_t isconst;   // value known at flatten time
  uint8_t afirst;    // binary, both subtrees: evaluate a first
  uint8_t need;      // Sethi-Ullman stack need
  int16_t len;       // instructions to compute this row into acc
  float cval;        // constant value when isconst
  Ref a, b;
};

MTGP_INLINE MTGP_HD int32_t f2i_sat(float v) {
  if (mtgp_isnan(v)) return 0;
  if (v >= 2147483648.0f) return 2147483647;
  if (v <= -2147483648.0f) return (-2147483647 - 1);
  return (int32_t)v;
}

MTGP_INLINE MTGP_HD int norm_index(float v, int N) {
  int32_t i = f2i_sat(v);
  int64_t j = i;
  if (j < 0) j += N;
  if (j < 0) j = 0;
  if (j > N - 1) j = N - 1;
  return (int)j;
}

MTGP_INLINE MTGP_HD float apply_fn(int fn, float x, float y) {
  switch (fn) {
    case MTGP_FN_ADD: return x + y;
    case MTGP_FN_SUB: return x - y;
    case MTGP_FN_MUL: return x * y;
    case MTGP_FN_DIV: return x / y;
    case MTGP_FN_SIN: return mtgp_sinf(x);
    case MTGP_FN_COS: return mtgp_cosf(x);
    case MTGP_FN_EXP: return mtgp_expf(x);
    case MTGP_FN_LOG: return mtgp_logf(x);
    case MTGP_FN_SQRT: return mtgp_sqrtf(x);
    case MTGP_FN_TANH: return mtgp_tanhf(x);
    case MTGP_FN_ABS: return mtgp_absf(x);
    default: return 0.0f;
  }
}

MTGP_INLINE MTGP_HD int fn_arity(int fn) {
  return (fn >= MTGP_FN_ADD && fn <= MTGP_FN_DIV) ? 2 : (MTGP_FN_IS_UNARY(fn) ? 1 : 0);
}

// a unary function whose leaf operand fuses into one instruction (SINV / COSV and their push
// forms); the other unary functions are a load followed by the operation
MTGP_INLINE MTGP_HD bool unary_fuses(int fn) { return fn == MTGP_FN_SIN || fn == MTGP_FN_COS; }

// program opcode of a unary function (acc = f(acc))
MTGP_INLINE MTGP_HD uint32_t unary_op(int fn) {
  switch (fn) {
    case MTGP_FN_SIN: return MTGP_OP_SIN;
    case MTGP_FN_COS: return MTGP_OP_COS;
    case MTGP_FN_EXP: return MTGP_OP_EXP;
    case MTGP_FN_LOG: return MTGP_OP_LOG;
    case MTGP_FN_SQRT: return MTGP_OP_SQRT;
    case MTGP_FN_TANH: return MTGP_OP_TANH;
    default: return MTGP_OP_ABS;
  }
}

// Rows whose value is the constant 0.0 without any lookup: f != 1.0 and int(f) (clamped) an
// empty / zero opcode (gp.py:135).  Such rows below the root get no RowInfo: a reference to one
// (j < i, already "evaluated") is the constant 0.0, exactly what its RowInfo would fold to.
// zrows: bitmask over rows (N <= MTGP_MAX_NODES = 256).
MTGP_INLINE MTGP_HD bool zero_row(const float* tree, int i, const MtgpNodeLibrary* lib) {
  const float fv = tree[4 * i + 0];
  if (fv == 1.0f) return false;
  int32_t f = f2i_sat(fv);
  if (f < 0) f = 0;
  if (f > lib->n_funcs - 1) f = lib->n_funcs - 1;
  return lib->fn[f] == MTGP_FN_ZERO;
}

// Resolve row i of `tree` ([N,4] f32) into info[i]; rows < i must be resolved already (or be
// zero rows marked in zrows).
MTGP_INLINE MTGP_HD void resolve_row(const float* tree, int N, int i, const MtgpNodeLibrary* lib,
                                     int n_data, uint64_t zero_mask, RowInfo* info, const uint64_t* zrows,
                                     int gap_at = 0, int gap = 0) {
  RowInfo& r = info[i];
  const float fv = tree[4 * i + 0];
  r.afirst = 1;
  r.need = 0;
  r.len = 1;
  r.a.row = -1; r.a.val = 0.0f;
  r.b.row = -1; r.b.val = 0.0f;
  r.slot = 0;
  if (fv == 1.0f) {  // coefficient (gp.py:372 select)
    r.kind = K_CONST; r.fn = MTGP_FN_ZERO; r.isconst = 1; r.cval = tree[4 * i + 3];
    return;
  }
  int32_t f = f2i_sat(fv);
  if (f < 0) f = 0;
  if (f > lib->n_funcs - 1) f = lib->n_funcs - 1;
  const int fn = lib->fn[f];
  r.fn = (uint8_t)fn;
  if (fn == MTGP_FN_VAR) {
    int slot = f - lib->var_start;
    if (slot > n_data - 1) slot = n_data - 1;  // (caller guarantees n_data >= V)
    r.slot = (uint8_t)(slot >= gap_at ? slot + gap : slot);  // the evaluator's layout (MtgpProgramSpec.gap)
    if ((zero_mask >> slot) & 1ull) { r.kind = K_CONST; r.isconst = 1; r.cval = 0.0f; }
    else { r.kind = K_VAR; r.isconst = 0; r.cval = 0.0f; }
    return;
  }
  const int ar = fn_arity(fn);
  if (ar == 0) {  // empty node or coefficient-through-switch: 0.0 (gp.py:135)
    r.kind = K_CONST; r.isconst = 1; r.cval = 0.0f;
    return;
  }
  // operands: x from a_idx, y from b_idx
  for (int k = 0; k < ar; ++k) {
    const int j = norm_index(tree[4 * i + 1 + k], N);
    Ref ref;
    if (j < i && ((zrows[j >> 6] >> (j & 63)) & 1ull)) { ref.row = -1; ref.val = 0.0f; }  // evaluated zero row
    else if (j < i) { ref.row = (int16_t)j; ref.val = 0.0f; }
    else { ref.row = -1; ref.val = tree[4 * j + 3]; }  // not evaluated yet: original column
    if (k == 0) r.a = ref; else r.b = ref;
  }
  r.kind = (ar == 1) ? K_UNARY : K_BINARY;
  // constant folding
  const bool ac = (r.a.row < 0) || info[r.a.row].isconst;
  const bool bc = (ar == 1) || (r.b.row < 0) || info[r.b.row].isconst;
  if (ac && bc) {
    const float xa = (r.a.row < 0) ? r.a.val : info[r.a.row].cval;
    const float yb = (ar == 1) ? 0.0f : ((r.b.row < 0) ? r.b.val : info[r.b.row].cval);
    r.isconst = 1;
    r.cval = apply_fn(fn, xa, yb);
    return;
  }
  r.isconst = 0;
  r.cval = 0.0f;
}

// leaf operand: constant or (non-zeroed) variable row
MTGP_INLINE MTGP_HD bool ref_is_leaf(const Ref& x, const RowInfo* info) {
  return x.row < 0 || info[x.row].isconst || info[x.row].kind == K_VAR;
}

MTGP_INLINE MTGP_HD void size_row(int i, RowInfo* info) {
  RowInfo& r = info[i];
  if (r.isconst || r.kind == K_VAR) { r.len = 1; r.need = 0; return; }
  const bool al = ref_is_leaf(r.a, info);
  if (r.kind == K_UNARY) {
    if (al) { r.len = 2; r.need = 0; }
    else { r.len = info[r.a.row].len + 1; r.need = info[r.a.row].need; }
    return;
  }
  const bool bl = ref_is_leaf(r.b, info);
  if (al && bl) { r.len = 2; r.need = 0; return; }
  if (bl) { r.len = info[r.a.row].len + 1; r.need = info[r.a.row].need; return; }
  if (al) { r.len = info[r.b.row].len + 1; r.need = info[r.b.row].need; return; }
  const int p = info[r.a.row].need, q = info[r.b.row].need;
  const int len = info[r.a.row].len + info[r.b.row].len + 1;
  r.len = (int16_t)(len > 32767 ? 32767 : len);
  if (p >= q) { r.afirst = 1; r.need = (uint8_t)((p > q + 1) ? p : q + 1); }
  else { r.afirst = 0; r.need = (uint8_t)((q > p + 1) ? q : p + 1); }
}

// Opcode of family member idx (ADD, SUB, RSUB, MUL, DIV, RDIV) for operand kind C / V / S and
// of the fused forms (opcode values are generated, not contiguous).
enum { FK_C = 0, FK_V = 1, FK_S = 2, FK_VC = 3, FK_VCP = 4 };
MTGP_INLINE MTGP_HD uint32_t fam_op(int kind, int idx) {
  switch (kind) {
    case FK_C: { const uint32_t t[6] = {MTGP_OP_ADDC, MTGP_OP_SUBC, MTGP_OP_RSUBC, MTGP_OP_MULC, MTGP_OP_DIVC, MTGP_OP_RDIVC}; return t[idx]; }
    case FK_V: { const uint32_t t[6] = {MTGP_OP_ADDV, MTGP_OP_SUBV, MTGP_OP_RSUBV, MTGP_OP_MULV, MTGP_OP_DIVV, MTGP_OP_RDIVV}; return t[idx]; }
    case FK_S: { const uint32_t t[6] = {MTGP_OP_ADDS, MTGP_OP_SUBS, MTGP_OP_RSUBS, MTGP_OP_MULS, MTGP_OP_DIVS, MTGP_OP_RDIVS}; return t[idx]; }
    case FK_VC: { const uint32_t t[6] = {MTGP_OP_VC_ADD, MTGP_OP_VC_SUB, MTGP_OP_VC_RSUB, MTGP_OP_VC_MUL, MTGP_OP_VC_DIV, MTGP_OP_VC_RDIV}; return t[idx]; }
    default: { const uint32_t t[6] = {MTGP_OP_VCP_ADD, MTGP_OP_VCP_SUB, MTGP_OP_VCP_RSUB, MTGP_OP_VCP_MUL, MTGP_OP_VCP_DIV, MTGP_OP_VCP_RDIV}; return t[idx]; }
  }
}

// family index of a C / V opcode (-1 if op is not one)
MTGP_INLINE MTGP_HD int fam_idx(uint32_t op, int kind) {
  for (int i = 0; i < 6; ++i)
    if (fam_op(kind, i) == op) return i;
  return -1;
}

MTGP_INLINE MTGP_HD bool is_var_op(uint32_t op) {
  return op == MTGP_OP_LDV || op == MTGP_OP_LDVP || fam_idx(op, FK_V) >= 0;
}

MTGP_INLINE MTGP_HD float bits_to_f32(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, sizeof f);
  return f;
}

// Superinstructions (peephole over an emitted program): a leaf load followed by the leaf
// operation or unary that consumes it becomes one instruction.  Exact: the fused handler
// performs the same single fp32 operation on the same operands; the only rewrites swap the
// operands of + and * (commutative in IEEE arithmetic, signed zeros included) or turn
// "c - v" / "c / v" into the reversed VC forms.
MTGP_INLINE MTGP_HD bool fuse_pair(const MtgpInstr& a, const MtgpInstr& b, MtgpInstr* f) {
  const uint32_t oa = a.op >> MTGP_OP_SHIFT, ob = b.op >> MTGP_OP_SHIFT;
  uint32_t ia, ib;
  __builtin_memcpy(&ia, &a.imm, 4);
  __builtin_memcpy(&ib, &b.imm, 4);
  const bool push = (oa == MTGP_OP_LDVP || oa == MTGP_OP_LDCP);
  if (oa == MTGP_OP_LDV || oa == MTGP_OP_LDVP) {  // acc = v_a ...
    const int kc = fam_idx(ob, FK_C);
    if (kc >= 0) {  // ... op c
      f->op = (fam_op(push ? FK_VCP : FK_VC, kc) << MTGP_OP_SHIFT) | ia;
      f->imm = b.imm;
      return true;
    }
    const int kv = fam_idx(ob, FK_V);
    if (kv >= 0) {  // ... op v_b  ->  VV(left, right)
      uint32_t l = ia, r = ib, op;
      switch (kv) {
        case 0: op = push ? MTGP_OP_VVP_ADD : MTGP_OP_VV_ADD; break;
        case 1: op = push ? MTGP_OP_VVP_SUB : MTGP_OP_VV_SUB; break;
        case 2: op = push ? MTGP_OP_VVP_SUB : MTGP_OP_VV_SUB; l = ib; r = ia; break;  // v_b - v_a
        case 3: op = push ? MTGP_OP_VVP_MUL : MTGP_OP_VV_MUL; break;
        case 4: op = push ? MTGP_OP_VVP_DIV : MTGP_OP_VV_DIV; break;
        default: op = push ? MTGP_OP_VVP_DIV : MTGP_OP_VV_DIV; l = ib; r = ia; break;  // v_b / v_a
      }
      f->op = (op << MTGP_OP_SHIFT) | r;
      f->imm = bits_to_f32(l);
      return true;
    }
    if (ob == MTGP_OP_SIN || ob == MTGP_OP_COS) {
      const uint32_t op = ob == MTGP_OP_SIN ? (push ? MTGP_OP_SINVP : MTGP_OP_SINV) : (push ? MTGP_OP_COSVP : MTGP_OP_COSV);
      f->op = op << MTGP_OP_SHIFT;
      f->imm = a.imm;
      return true;
    }
    return false;
  }
  if (oa == MTGP_OP_LDC || oa == MTGP_OP_LDCP) {  // acc = c op v_b
    const int kv = fam_idx(ob, FK_V);
    if (kv < 0) return false;
    const int map[6] = {0, 2, 1, 3, 5, 4};  // c+v = v+c, c-v = RSUB, v-c = SUB, c*v, c/v = RDIV, v/c = DIV
    f->op = (fam_op(push ? FK_VCP : FK_VC, map[kv]) << MTGP_OP_SHIFT) | ib;
    f->imm = a.imm;
    return true;
  }
  return false;
}

// The emitter applies the superinstruction peephole while it writes: the last instruction is
// held back until the next one shows whether the pair fuses (the same greedy left-to-right
// pairing as a second pass over the finished program, without reading it back).  n counts the
// unfused instructions (the length limits are defined on it), j the words written.
struct Emitter {
  MtgpInstr* out;
  int cap;
  int n;
  int pending_push;
  int j;
  bool have;
  MtgpInstr held;
  MTGP_HD void put(uint32_t op, uint32_t slot, float imm) {
    // V opcodes carry the slot as an LDS byte offset (mtgp.h program format)
    if (n < cap) {
      MtgpInstr x;
      x.op = op << MTGP_OP_SHIFT;
      x.imm = is_var_op(op) ? bits_to_f32(slot * MTGP_SLOT_BYTES) : imm;
      if (have) {
        MtgpInstr f;
        if (fuse_pair(held, x, &f)) {
          out[j++] = f;
          have = false;
        } else {
          out[j++] = held;
          held = x;
        }
      } else {
        held = x;
        have = true;
      }
    }
    ++n;
  }
  MTGP_HD int finish() {
    if (have) out[j++] = held;
    have = false;
    return j;
  }
  // load a leaf operand into acc (pushing the previous acc when a push is pending)
  MTGP_HD void load(const Ref& x, const RowInfo* info) {
    const int p = pending_push;
    pending_push = 0;
    if (x.row < 0) put(p ? MTGP_OP_LDCP : MTGP_OP_LDC, 0, x.val);
    else if (info[x.row].isconst) put(p ? MTGP_OP_LDCP : MTGP_OP_LDC, 0, info[x.row].cval);
    else put(p ? MTGP_OP_LDVP : MTGP_OP_LDV, info[x.row].slot, 0.0f);
  }
  // acc = f(acc, leaf) when rev == 0, acc = f(leaf, acc) when rev == 1
  MTGP_HD void op_leaf(int fn, int rev, const Ref& x, const RowInfo* info) {
    const bool isc = (x.row < 0) || info[x.row].isconst;
    const float v = (x.row < 0) ? x.val : info[x.row].cval;
    int base;
    switch (fn) {
      case MTGP_FN_ADD: base = 0; rev = 0; break;
      case MTGP_FN_SUB: base = 1; break;
      case MTGP_FN_MUL: base = 3; rev = 0; break;
      default: base = 4; break;  // DIV
    }
    // family members: ADD, SUB, RSUB, MUL, DIV, RDIV
    int idx = base + ((base == 1 || base == 4) ? rev : 0);
    if (isc) put(fam_op(FK_C, idx), 0, v);
    else put(fam_op(FK_V, idx), info[x.row].slot, 0.0f);
  }
  MTGP_HD void op_stack(int fn, int rev) {
    int idx;
    switch (fn) {
      case MTGP_FN_ADD: idx = 0; break;
      case MTGP_FN_SUB: idx = rev ? 2 : 1; break;
      case MTGP_FN_MUL: idx = 3; break;
      default: idx = rev ? 5 : 4; break;
    }
    put(fam_op(FK_S, idx), 0, 0.0f);
  }
};

// Emit the program computing row `root` into acc. Uses an explicit frame stack.
// Returns the unfused instruction count; *fused = words written (valid when count <= cap).
MTGP_INLINE MTGP_HD int emit_program(int root, const RowInfo* info, MtgpInstr* out, int cap, int* fused) {
  Emitter em;
  em.out = out; em.cap = cap; em.n = 0; em.pending_push = 0; em.j = 0; em.have = false;
  *fused = 0;
  const RowInfo& rr = info[root];
  if (rr.isconst || rr.kind == K_VAR) {
    Ref x; x.row = (int16_t)root; x.val = 0.0f;
    em.load(x, info);
    *fused = em.finish();
    return em.n;
  }
  int16_t fr_row[MTGP_MAX_NODES + 1];
  uint8_t fr_ph[MTGP_MAX_NODES + 1];
  int top = 0;
  fr_row[0] = (int16_t)root; fr_ph[0] = 0;
  while (top >= 0) {
    if (em.n > cap) return em.n;  // runaway (shared sub-DAGs): caller reports too-long
    const int n = fr_row[top];
    const RowInfo& r = info[n];
    const int ph = fr_ph[top];
    const bool al = ref_is_leaf(r.a, info);
    if (r.kind == K_UNARY) {
      if (ph == 0 && al) {
        em.load(r.a, info);
        em.put(unary_op(r.fn), 0, 0.0f);
        --top;
      } else if (ph == 0) {
        fr_ph[top] = 1;
        ++top; fr_row[top] = r.a.row; fr_ph[top] = 0;
      } else {
        em.put(unary_op(r.fn), 0, 0.0f);
        --top;
      }
      continue;
    }
    // binary
    const bool bl = ref_is_leaf(r.b, info);
    if (bl) {
      if (ph == 0 && al) {
        em.load(r.a, info);
        em.op_leaf(r.fn, 0, r.b, info);
        --top;
      } else if (ph == 0) {
        fr_ph[top] = 1;
        ++top; fr_row[top] = r.a.row; fr_ph[top] = 0;
      } else {
        em.op_leaf(r.fn, 0, r.b, info);
        --top;
      }
    } else if (al) {
      if (ph == 0) {
        fr_ph[top] = 1;
        ++top; fr_row[top] = r.b.row; fr_ph[top] = 0;
      } else {
        em.op_leaf(r.fn, 1, r.a, info);  // acc = f(a_leaf, acc)
        --top;
      }
    } else {
      const int first = r.afirst ? r.a.row : r.b.row;
      const int second = r.afirst ? r.b.row : r.a.row;
      if (ph == 0) {
        fr_ph[top] = 1;
        ++top; fr_row[top] = (int16_t)first; fr_ph[top] = 0;
      } else if (ph == 1) {
        fr_ph[top] = 2;
        em.pending_push = 1;
        ++top; fr_row[top] = (int16_t)second; fr_ph[top] = 0;
      } else {
        // a first: stack holds x, acc = y -> acc = f(pop, acc)   (reversed)
        // b first: stack holds y, acc = x -> acc = f(acc, pop)
        em.op_stack(r.fn, r.afirst ? 1 : 0);
        --top;
      }
    }
  }
  if (em.n <= cap) *fused = em.finish();
  return em.n;
}

// Full flatten of one tree: the fused program (unfused length at most cap) -> its length, or
// -MTGP_ERR_*.
MTGP_INLINE MTGP_HD int flatten_tree_body(const float* tree, int N, const MtgpNodeLibrary* lib,
                                          int n_data, uint64_t zero_mask, MtgpInstr* out, int cap,
                                          RowInfo* info, int* stack_need, int gap_at = 0, int gap = 0) {
  uint64_t zrows[(MTGP_MAX_NODES + 63) / 64] = {0};
  for (int i = 0; i < N; ++i) {
    if (i < N - 1 && zero_row(tree, i, lib)) {  // empty rows (most of a reference tree): no RowInfo
      zrows[i >> 6] |= 1ull << (i & 63);
      continue;
    }
    resolve_row(tree, N, i, lib, n_data, zero_mask, info, zrows, gap_at, gap);
    size_row(i, info);
  }
  const int need = info[N - 1].need;
  if (stack_need) *stack_need = need;
  if (need > MTGP_STACK_MAX) return -MTGP_ERR_STACK;
  if (info[N - 1].len > cap) return -MTGP_ERR_PROG_TOO_LONG;
  int fused = 0;
  const int n = emit_program(N - 1, info, out, cap, &fused);
  if (n > cap) return -MTGP_ERR_PROG_TOO_LONG;
  return fused;
}

// Full flatten of one tree into `slots` instructions: the program (at most slots - 1) and
// its MTGP_OP_END.  Returns the program length (>0, END excluded) or -MTGP_ERR_*; on error
// the slot holds a bare END (an empty program), so an evaluator never runs stale words.
MTGP_INLINE MTGP_HD int flatten_tree(const float* tree, int N, const MtgpNodeLibrary* lib,
                                     int n_data, uint64_t zero_mask, MtgpInstr* out, int slots,
                                     RowInfo* info, int* stack_need, int gap_at = 0, int gap = 0) {
  if (slots < 1) return -MTGP_ERR_PROG_TOO_LONG;
  const int n = flatten_tree_body(tree, N, lib, n_data, zero_mask, out, slots - 1, info, stack_need, gap_at, gap);
  const int at = n > 0 ? n : 0;
  out[at].op = (uint32_t)MTGP_OP_END << MTGP_OP_SHIFT;
  out[at].imm = 0.0f;
  return n;
}

MTGP_INLINE MTGP_HD int count_nodes(const float* tree, int N) {
  int c = 0;
  for (int i = 0; i < N; ++i) c += (tree[4 * i] != 0.0f) ? 1 : 0;
  return c;
}

}  // namespace mtgp
