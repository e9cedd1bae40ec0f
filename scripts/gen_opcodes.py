#!/usr/bin/env python3
"""Generate the program opcode set and the interpreter's dispatch tree.

The evaluator dispatches on the raw instruction word w = opcode << 24 | aux with a binary
tree of `w < K << 24` scalar compares.  Every compare + branch costs scalar issue slots (the
interpreter's bound), so the tree is a Huffman tree over measured dispatch
frequencies (C3 control programs, plus SR programs at a lower weight) instead of the
compiler's balanced tree over opcode values.  Opcodes are numbered by an in-order walk of the
tree, so every internal node splits a contiguous opcode range.

Outputs (committed; tests/test_abi.py checks they are up to date):
  include/mtgp_opcodes.h             enum MTGP_OP_*  (part of the C ABI)
  multitreegp_amd/csrc/mtgp_dispatch.inc   MTGP_DISPATCH(w, ib) for the kernel
  multitreegp_amd/_opcodes.py         names + operand kinds for host-side decoding

Operand conventions in a handler: `imm` = f32 view of the imm word, `ib` = its bits,
`ax` = w & 0xffffff (the aux field), V(x) = the data slot at LDS byte offset x (emitted as
MTGP_LDSV), PUSH pushes
acc, POP pops into `s_`.
"""
import heapq
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (name, handler, kinds, weight) -- kinds: operand layout for host decoding:
#   "-" none, "C" imm = constant, "V" imm = slot, "VC" aux = slot & imm = constant,
#   "VV" imm = slot a & aux = slot b
FAM = [("ADD", "{x} + {y}"), ("SUB", "{x} - {y}"), ("RSUB", "{y} - {x}"), ("MUL", "{x} * {y}"),
       ("DIV", "{x} / {y}"), ("RDIV", "{y} / {x}")]

# dispatch frequencies (% of dispatches) after fusion: C3 (weight 1) + C5 SR mix (weight 0.3),
# measured with scripts/opcode_stats.py; ops absent from both get a floor weight
FREQ_C3 = {'END': 20.12, 'MULC': 8.71, 'ADDC': 8.2, 'ADDV': 6.62, 'MULV': 6.01, 'VC_MUL': 5.33, 'ADDS': 5.14, 'MULS': 5.04, 'VC_ADD': 4.79, 'VCP_MUL': 3.22, 'VCP_ADD': 3.12, 'COS': 2.61, 'SIN': 2.29, 'VV_MUL': 2.07, 'LDC': 2.05, 'VV_ADD': 1.76, 'VVP_ADD': 1.48, 'SINV': 1.42, 'COSV': 1.39, 'VVP_MUL': 0.97, 'RSUBC': 0.95, 'RSUBS': 0.85, 'SUBC': 0.83, 'SINVP': 0.7, 'COSVP': 0.68, 'RSUBV': 0.65, 'SUBV': 0.64, 'VV_SUB': 0.48, 'VC_RSUB': 0.42, 'VC_SUB': 0.38, 'VCP_RSUB': 0.37, 'VCP_SUB': 0.31, 'VVP_SUB': 0.26, 'SUBS': 0.09}
FREQ_SR = {'END': 17.68, 'MULC': 8.85, 'ADDC': 8.71, 'ADDV': 6.8, 'MULV': 6.72, 'ADDS': 5.84, 'MULS': 5.52, 'VC_MUL': 4.99, 'VC_ADD': 4.97, 'VCP_ADD': 3.93, 'VCP_MUL': 3.91, 'VV_MUL': 2.11, 'VV_ADD': 2.0, 'VVP_MUL': 1.74, 'VVP_ADD': 1.69, 'RSUBS': 0.99, 'RDIVC': 0.98, 'LDC': 0.97, 'RDIVS': 0.95, 'RSUBC': 0.89, 'SUBC': 0.85, 'DIVC': 0.85, 'DIVV': 0.75, 'RSUBV': 0.7, 'RDIVV': 0.69, 'SUBV': 0.68, 'VC_RDIV': 0.55, 'VC_SUB': 0.5, 'VCP_RDIV': 0.46, 'VC_DIV': 0.46, 'VCP_RSUB': 0.42, 'VV_DIV': 0.41, 'VC_RSUB': 0.41, 'VCP_DIV': 0.38, 'VVP_DIV': 0.37, 'VVP_SUB': 0.35, 'VCP_SUB': 0.34, 'VV_SUB': 0.31, 'SUBS': 0.14, 'DIVS': 0.14}
FLOOR = 0.15


def ops():
    out = [("LDC", "acc = imm;", "C"), ("LDCP", "PUSH acc = imm;", "C"),
           ("LDV", "acc = V(ib);", "V"), ("LDVP", "PUSH acc = V(ib);", "V")]
    for k, src in (("C", "imm"), ("V", "V(ib)"), ("S", "s_")):
        for f, e in FAM:
            pre = "POP " if k == "S" else ""
            out.append((f + k, pre + "acc = " + e.format(x="acc", y=src) + ";", k if k != "S" else "-"))
    out += [("SIN", "acc = mtgp_sinf(acc);", "-"), ("COS", "acc = mtgp_cosf(acc);", "-")]
    # further unary operators (round 3; include/mtgp_f32math.h specs): acc forms only, at the
    # floor weight (the JIT does not translate them, populations using them are interpreted)
    out += [("EXP", "acc = mtgp_expf(acc);", "-"), ("LOG", "acc = mtgp_logf(acc);", "-"),
            ("SQRT", "acc = mtgp_sqrtf(acc);", "-"), ("TANH", "acc = mtgp_tanhf(acc);", "-"),
            ("ABS", "acc = mtgp_absf(acc);", "-")]
    # superinstructions: a leaf load fused with the leaf operation that follows it
    for p in ("", "P"):
        push = "PUSH " if p else ""
        for f, e in FAM:  # acc = V(a) op c
            out.append(("VC" + p + "_" + f, push + "acc = " + e.format(x="V(ax)", y="imm") + ";", "VC"))
        for f, e in FAM[:2] + FAM[3:5]:  # ADD SUB MUL DIV: acc = V(a) op V(b)
            out.append(("VV" + p + "_" + f, push + "acc = " + e.format(x="V(ib)", y="V(ax)") + ";", "VV"))
        out.append(("SINV" + p, push + "acc = mtgp_sinf(V(ib));", "V"))
        out.append(("COSV" + p, push + "acc = mtgp_cosf(V(ib));", "V"))
    out.append(("END", "goto done;", "-"))
    return out


def weights(names):
    w = {}
    for n in names:
        w[n] = max(FREQ_C3.get(n, 0.0) + 0.3 * FREQ_SR.get(n, 0.0), FLOOR)
    return w


def huffman(names, w, max_depth=8):
    """Huffman tree (nested tuples / leaf names); weights are flattened until depth <= max_depth."""
    ww = dict(w)
    while True:
        heap = [(ww[n], i, n) for i, n in enumerate(names)]
        heapq.heapify(heap)
        cnt = len(heap)
        while len(heap) > 1:
            a = heapq.heappop(heap)
            b = heapq.heappop(heap)
            heapq.heappush(heap, (a[0] + b[0], cnt, (a[2], b[2])))
            cnt += 1
        tree = heap[0][2]

        def depth(t):
            return 0 if isinstance(t, str) else 1 + max(depth(t[0]), depth(t[1]))
        if depth(tree) <= max_depth:
            return tree
        ww = {n: v ** 0.8 for n, v in ww.items()}


def leaves(t):
    return [t] if isinstance(t, str) else leaves(t[0]) + leaves(t[1])


def tree_weight(t, w):
    return w[t] if isinstance(t, str) else tree_weight(t[0], w) + tree_weight(t[1], w)


def generate():
    table = ops()
    names = [n for n, _, _ in table]
    handler = {n: h for n, h, _ in table}
    kinds = {n: k for n, _, k in table}
    w = weights(names)
    tree = huffman(names, w)
    order = leaves(tree)
    code = {n: i for i, n in enumerate(order)}
    exp_depth = 0.0

    def emit(t, ind, d):
        nonlocal exp_depth
        pad = "  " * ind
        if isinstance(t, str):
            exp_depth += w[t] * d
            h = handler[t].replace("PUSH ", "st[sp * kWave] = acc; ++sp; ").replace("POP ", "--sp; const float s_ = st[sp * kWave]; ")
            h = h.replace("V(", "MTGP_LDSV(")
            return [f"{pad}{{ /* {t} */ {h} }}"]
        k = code[leaves(t[1])[0]]
        lw, rw = tree_weight(t[0], w), tree_weight(t[1], w)
        cond = f"w < {k}u << MTGP_OP_SHIFT"
        cond = f"__builtin_expect({cond}, {1 if lw >= rw else 0})"
        return ([f"{pad}if ({cond}) {{"] + emit(t[0], ind + 1, d + 1) + [f"{pad}}} else {{"] +
                emit(t[1], ind + 1, d + 1) + [f"{pad}}}"])

    body = emit(tree, 1, 0)
    exp_depth /= sum(w.values())
    hdr = ["/* GENERATED by scripts/gen_opcodes.py -- do not edit. */",
           "#ifndef MTGP_OPCODES_H", "#define MTGP_OPCODES_H",
           "/* opcode in the top byte of the op word: w = opcode << MTGP_OP_SHIFT | aux */",
           "#define MTGP_OP_SHIFT 24", "enum {"]
    for n in order:
        hdr.append(f"  MTGP_OP_{n} = {code[n]},")
    hdr += [f"  MTGP_OP_COUNT = {len(order)}", "};", "#endif", ""]
    inc = ["// GENERATED by scripts/gen_opcodes.py -- do not edit.",
           f"// Huffman dispatch tree over {len(order)} opcodes, expected depth {exp_depth:.2f} compares",
           "// (a balanced tree needs {:.2f}).  Needs in scope: acc, sp, st, dcol, kWave and a".format(
               math.log2(len(order))),
           "// label `done` (END).",
           "#define MTGP_LDSV(x) (*(const float*)((const char*)dcol + (x)))",
           "#define MTGP_DISPATCH(w_, ib_)                                                       \\",
           "  {                                                                                  \\",
           "    const uint32_t w = (w_), ib = (ib_), ax = w & 0xffffffu;                          \\",
           "    const float imm = __uint_as_float(ib);                                            \\",
           "    (void)ax;                                                                        \\"]
    inc += [line + " \\" for line in body]
    inc += ["  }", ""]
    py = ['"""GENERATED by scripts/gen_opcodes.py -- do not edit."""',
          f"OP_SHIFT = 24",
          f"OP_NAMES = {order!r}",
          f"OP_KINDS = {[kinds[n] for n in order]!r}",
          ""]
    return "\n".join(hdr), "\n".join(inc), "\n".join(py), exp_depth


def targets():
    return {os.path.join(ROOT, "include", "mtgp_opcodes.h"): 0,
            os.path.join(ROOT, "multitreegp_amd", "csrc", "mtgp_dispatch.inc"): 1,
            os.path.join(ROOT, "multitreegp_amd", "_opcodes.py"): 2}


def main():
    out = generate()
    for path, i in targets().items():
        with open(path, "w") as f:
            f.write(out[i])
    print(f"{len(ops())} opcodes, expected dispatch depth {out[3]:.2f}")


if __name__ == "__main__":
    sys.exit(main())
