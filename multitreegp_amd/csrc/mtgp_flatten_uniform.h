// mtgp_flatten_uniform.h -- the device flattener with row-uniform control flow.
//
// mtgp_flatten.h's flatten_tree walks one tree per lane with data-dependent control flow: in a
// wave whose lanes hold different trees every branch of the walk is executed for the union of
// the lanes (measured: an 8k-instruction kernel, ~300 us at C3).  Here all lanes step through
// the row indices together and every per-row decision is a select:
//   pass 1 (rows ascending, gp.py:366-376 order): resolve each row -- constant / variable /
//     operator, operand references, constant folding -- and size it (unfused length `len` for the
//     limits, fused length `flen`, Sethi-Ullman need and operand order) into an LDS table laid
//     out [row][lane] (a child lookup is a gather with one lane per bank: conflict-free);
//   pass 2 (rows descending: a parent's row index is above its children's): the postorder
//     position of every reachable node follows from its parent's (first child at the parent's
//     start, second child after the first's code, the node's own word after both), so each node
//     writes its own instruction word directly.  A leaf operand is folded into its parent's word
//     (the fused superinstruction forms, mtgp_flatten.h fuse_pair), so every non-leaf node owns
//     exactly one word.
// The output (program words, lengths, status) is the one flatten_tree produces, word for word
// (tests/test_gpu_build.py compares with the host flattener).  A tree in which one row is reached
// from two parents (a shared sub-DAG, only in arbitrary arrays) needs its subtree emitted twice;
// such a lane re-runs the serial flatten_tree.
#pragma once
#include "mtgp_flatten.h"

namespace mtgp {

// one leaf operand: a constant or a data slot
struct ULeaf {
  bool isc;
  float v;
  uint32_t slot;
};

MTGP_INLINE MTGP_HD MtgpInstr u_instr(uint32_t op, uint32_t slot, float imm) {
  MtgpInstr x;
  x.op = op << MTGP_OP_SHIFT;
  x.imm = is_var_op(op) ? bits_to_f32(slot * MTGP_SLOT_BYTES) : imm;
  return x;
}

MTGP_INLINE MTGP_HD MtgpInstr u_load(const ULeaf& x, bool push) {
  return x.isc ? u_instr(push ? MTGP_OP_LDCP : MTGP_OP_LDC, 0, x.v) : u_instr(push ? MTGP_OP_LDVP : MTGP_OP_LDV, x.slot, 0.0f);
}

// Emitter::op_leaf: acc = f(acc, leaf) (rev 0) or f(leaf, acc) (rev 1)
MTGP_INLINE MTGP_HD MtgpInstr u_op_leaf(int fn, int rev, const ULeaf& x) {
  int base;
  switch (fn) {
    case MTGP_FN_ADD: base = 0; rev = 0; break;
    case MTGP_FN_SUB: base = 1; break;
    case MTGP_FN_MUL: base = 3; rev = 0; break;
    default: base = 4; break;  // DIV
  }
  const int idx = base + ((base == 1 || base == 4) ? rev : 0);
  return x.isc ? u_instr(fam_op(FK_C, idx), 0, x.v) : u_instr(fam_op(FK_V, idx), x.slot, 0.0f);
}

// Emitter::op_stack
MTGP_INLINE MTGP_HD MtgpInstr u_op_stack(int fn, int rev) {
  int idx;
  switch (fn) {
    case MTGP_FN_ADD: idx = 0; break;
    case MTGP_FN_SUB: idx = rev ? 2 : 1; break;
    case MTGP_FN_MUL: idx = 3; break;
    default: idx = rev ? 5 : 4; break;
  }
  return u_instr(fam_op(FK_S, idx), 0, 0.0f);
}

// packed row record: kind 2 | fn 4 | slot 8 | isconst 1 | afirst 1 | need 5 (bits, low to high)
MTGP_INLINE MTGP_HD uint32_t u_pack(uint32_t kind, uint32_t fn, uint32_t slot, uint32_t isc, uint32_t afirst,
                                    uint32_t need) {
  return kind | fn << 2 | slot << 6 | isc << 14 | afirst << 15 | need << 16;
}
MTGP_INLINE MTGP_HD uint32_t u_kind(uint32_t w) { return w & 3u; }
MTGP_INLINE MTGP_HD uint32_t u_fn(uint32_t w) { return (w >> 2) & 15u; }
MTGP_INLINE MTGP_HD uint32_t u_slot(uint32_t w) { return (w >> 6) & 255u; }
MTGP_INLINE MTGP_HD bool u_isc(uint32_t w) { return (w >> 14) & 1u; }
MTGP_INLINE MTGP_HD uint32_t u_afirst(uint32_t w) { return (w >> 15) & 1u; }
MTGP_INLINE MTGP_HD uint32_t u_need(uint32_t w) { return (w >> 16) & 31u; }

// a unary node over a leaf: its word(s) at pos (one fused word for sin / cos, else load + op)
MTGP_INLINE MTGP_HD int u_unary_leaf(int fn, const ULeaf& la, bool push, MtgpInstr* w) {
  const MtgpInstr un = u_instr(unary_op(fn), 0, 0.0f);
  if (unary_fuses(fn)) {
    fuse_pair(u_load(la, push), un, &w[0]);
    return 1;
  }
  w[0] = u_load(la, push);
  w[1] = un;
  return 2;
}
MTGP_INLINE MTGP_HD bool u_leaf(uint32_t w) { return u_isc(w) || u_kind(w) == K_VAR; }

// per-lane bit set over NMAX rows kept in registers (selects, never a dynamic index)
template <int NMAX>
struct UBits {
  static constexpr int W = (NMAX + 63) / 64;
  uint64_t w[W];
  MTGP_HD void clear() {
    for (int k = 0; k < W; ++k) w[k] = 0;
  }
  MTGP_HD bool test(int i) const {
    uint64_t r = 0;
    for (int k = 0; k < W; ++k) r = (k == (i >> 6)) ? w[k] : r;
    return (r >> (i & 63)) & 1ull;
  }
  MTGP_HD void set(int i) {
    for (int k = 0; k < W; ++k) w[k] |= (k == (i >> 6)) ? (1ull << (i & 63)) : 0ull;
  }
};

}  // namespace mtgp
