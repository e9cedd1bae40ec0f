"""Dual-number program JIT (multitreegp_amd/csrc/mtgp_jit_dual.h, ABI v19) checked on the CPU.

The gradient kernels' dual interpreter (csrc/mtgp_grad.hip run_dual_src) is restated here in
numpy float32 (d_add / d_sub / d_mul / d_div, constants with tangent 0, the unary rules of
include/mtgp_dual.h through the oracle's `unary`); the host translation of random programs over
every opcode family, run by a word-level emulator, reproduces it bit for bit in value and tangent
for every lane -- each lane with its own coefficient index, so parameter tangents are 1 in some
lanes and 0 in others.  The emitted words disassemble cleanly (llvm-mc, gfx950) and write only
the registers of the dual call ABI.  The GPU side (the same translation executed) is
tests/test_coefficients.py's bit-exact comparisons plus test_gpu_dual_jit_* there."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from multitreegp_amd import _native as nat
from multitreegp_amd.sampling import sample_population
from oracle import oracle as orc
import multitreegp_amd as mt
from helpers import CONTROL_OPS

from test_jit import BLOBS, DEFS, FN, GETPC_S44, LLVM_MC, SETPC, SUB_AT, TEMPLATE_BYTES, _disassemble

pytestmark = pytest.mark.skipif(not os.path.exists(nat.LIB_PATH), reason="libmtgp_hip.so not built")

EXT = [("/", None, 2, 0.1), ("exp", None, 1, 0.05), ("log", None, 1, 0.05), ("sqrt", None, 1, 0.05),
       ("tanh", None, 1, 0.05), ("abs", None, 1, 0.05)]
FN_ADD, FN_SUB, FN_MUL, FN_DIV = 0, 1, 2, 3
FN_ABS = 12
F32 = np.float32


def _flatten(tree, nl, n_data):
    lib = nat.load()
    t = np.ascontiguousarray(tree, np.float32)
    L = 2 * t.shape[0] + 8
    out = (nat.MtgpInstr * L)()
    need = ctypes.c_int32(0)
    n = lib.mtgp_flatten_tree_host(t.ctypes.data, t.shape[0], ctypes.byref(nl), n_data, 0, L, ctypes.addressof(out),
                                   ctypes.byref(need))
    assert n > 0
    return np.frombuffer(bytes(out), dtype=np.uint32).reshape(-1, 2)[: n + 1].copy()


def _translate(prog, D, theta):
    lib = nat.load()
    p = np.ascontiguousarray(prog, np.uint32)
    th = np.ascontiguousarray(theta, np.float32)
    L = p.shape[0]
    n = lib.mtgp_jit_dual_translate_host(p.ctypes.data, L, D, th.ctypes.data, len(th), TEMPLATE_BYTES, None, 0)
    assert n > 0, n
    out = np.zeros(n, np.uint32)
    assert lib.mtgp_jit_dual_translate_host(p.ctypes.data, L, D, th.ctypes.data, len(th), TEMPLATE_BYTES,
                                            out.ctypes.data, n) == n
    return [int(w) for w in out]


# ---- the dual interpreter, restated (run_dual_src) --------------------------------------------
def _fam(f, a, b):
    """d_fam: 0 ADD, 1 SUB (a - b), 2 RSUB (b - a), 3 MUL, 4 DIV (a / b), 5 RDIV (b / a)."""
    if f == 2:
        a, b = b, a
        f = 1
    if f == 5:
        a, b = b, a
        f = 4
    (av, ad), (bv, bd) = a, b
    with np.errstate(all="ignore"):
        if f == 0:
            return av + bv, ad + bd
        if f == 1:
            return av - bv, ad - bd
        if f == 3:
            return av * bv, ad * bv + av * bd
        q = av / bv
        return q, (ad - q * bd) / bv


def _unary(fn, a):
    y, dy = orc.unary(fn, a[0], a[1])
    return y.astype(F32), dy.astype(F32)


def _run_dual(prog, D, theta, vals, tans, kk):
    """prog [n, 2] (op word, imm bits); vals / tans [D, M]; theta [K]; kk [M] -> (v, d) [M]."""
    M = vals.shape[1]
    zero = np.zeros(M, F32)
    ops = {name: i for i, name in enumerate(nat.OP_NAMES)}
    inv = {i: name for name, i in ops.items()}

    def V(slot):
        if slot < D:
            return vals[slot].copy(), tans[slot].copy()
        j = slot - D
        return np.full(M, theta[j], F32), np.where(kk == j, F32(1.0), F32(0.0)).astype(F32)

    acc = (zero.copy(), zero.copy())
    stack = []
    for w, imm in prog:
        code, ax = int(w) >> 24, int(w) & 0xFFFFFF
        immf = np.array([imm], np.uint32).view(np.float32)[0]
        C = (np.full(M, immf, F32), zero.copy())
        ib = int(imm) // nat.SLOT_BYTES
        axs = ax // nat.SLOT_BYTES
        name = inv[code]
        if name == "END":
            return acc
        if name == "LDC":
            acc = C
        elif name == "LDCP":
            stack.append(acc); acc = C
        elif name == "LDV":
            acc = V(ib)
        elif name == "LDVP":
            stack.append(acc); acc = V(ib)
        elif name in ("SIN", "COS", "EXP", "LOG", "SQRT", "TANH", "ABS"):
            acc = _unary(FN[name] if name in FN else FN_ABS, acc)
        elif name in ("SINV", "COSV", "SINVP", "COSVP"):
            if name.endswith("P"):
                stack.append(acc)
            acc = _unary(FN["SIN" if name.startswith("SIN") else "COS"], V(ib))
        else:
            m = re.fullmatch(r"(VCP?|VVP?)_(\w+)|(R?SUB|ADD|MUL|R?DIV)([CVS])", name)
            assert m, name
            fams = {"ADD": 0, "SUB": 1, "RSUB": 2, "MUL": 3, "DIV": 4, "RDIV": 5}
            if m.group(1):
                kind, f = m.group(1), fams[m.group(2)]
                if kind.endswith("P"):
                    stack.append(acc)
                if kind.startswith("VC"):
                    acc = _fam(f, V(axs), C)
                else:
                    acc = _fam(f, V(ib), V(axs))
            else:
                f, src = fams[m.group(3)], m.group(4)
                o = C if src == "C" else (V(ib) if src == "V" else stack.pop())
                acc = _fam(f, acc, o)
        acc = (acc[0].astype(F32), acc[1].astype(F32))
    raise AssertionError("no END")


# ---- word-level emulator of the dual code ------------------------------------------------------
def _src(v, s, words, i, M):
    """(value [M] as float32, words consumed) of a 9-bit source field (VGPR, inline, literal)."""
    if s >= 256:
        return v[s - 256].view(np.float32).copy(), 0
    if s == 255:
        return np.full(M, np.array([words[i]], np.uint32).view(np.float32)[0], F32), 1
    if s == 128:
        return np.zeros(M, F32), 0
    if 129 <= s <= 192:
        return np.full(M, s - 128, np.uint32).view(np.float32), 0
    return np.full(M, {240: 0.5, 241: -0.5, 242: 1.0, 243: -1.0, 244: 2.0, 245: -2.0, 246: 4.0, 247: -4.0}[s], F32), 0


def _emulate_dual(words, vals, tans, kk):
    M = vals.shape[1]
    v = np.zeros((72, M), np.uint32)
    v[: vals.shape[0]] = vals.view(np.uint32)
    v[48: 48 + tans.shape[0]] = tans.view(np.uint32)
    v[25] = kk.astype(np.int32).view(np.uint32)
    vcc = np.zeros(M, bool)
    i = 0

    def setf(d, x):
        v[d] = np.asarray(x, F32).view(np.uint32)

    while True:
        w = words[i]
        if w == SETPC:
            return v[8].view(np.float32).copy(), v[56].view(np.float32).copy()
        if w == GETPC_S44:
            assert words[i + 1] == 0x802CFF2C and words[i + 4] == 0xBEA81E2C
            rel = int(np.array(words[i + 2], np.uint32).view(np.int32))
            target = TEMPLATE_BYTES + 4 * (i + 1) + rel
            assert target in SUB_AT, target
            x = v[17].view(np.float32)
            name = SUB_AT[target]
            if name in ("SIN", "COS"):
                s, c = orc.sincos(x)
                setf(8, s if name == "SIN" else c)
            else:
                setf(8, orc.unary(FN[name], x))
            # the subroutines may clobber v17-v24 (v8 aside): poison them
            v[17:25] = 0x7FC00001
            i += 5
            continue
        if words[i:i + len(BLOBS["DIV"])] == BLOBS["DIV"]:
            with np.errstate(all="ignore"):
                setf(8, v[17].view(np.float32) / v[18].view(np.float32))
            v[19:24] = 0x7FC00001
            i += len(BLOBS["DIV"])
            continue
        if words[i:i + len(BLOBS["ABS"])] == BLOBS["ABS"]:
            setf(8, orc.unary(FN_ABS, v[8].view(np.float32)))
            i += len(BLOBS["ABS"])
            continue
        if (w >> 25) == 0x3F:  # VOP1: v_mov_b32
            assert ((w >> 9) & 0xFF) == 1, hex(w)
            a, n = _src(v, w & 0x1FF, words, i + 1, M)
            setf((w >> 17) & 0xFF, a)
            i += 1 + n
            continue
        if (w >> 25) == 0x3E:  # VOPC e32 -> vcc
            a, n = _src(v, w & 0x1FF, words, i + 1, M)
            b = v[(w >> 9) & 0xFF]
            op = (w >> 17) & 0xFF
            if op == 0xCA:  # v_cmp_eq_u32
                vcc = a.view(np.uint32) == b
            elif op == 0x44:  # v_cmp_gt_f32: a > b
                vcc = a > b.view(np.float32)
            elif op == 0x41:  # v_cmp_lt_f32: a < b
                vcc = a < b.view(np.float32)
            else:
                raise AssertionError(hex(w))
            i += 1 + n
            continue
        if (w & 0xFFFFFF00) == 0xD1000000:  # v_cndmask_b32_e64 vdst, src0, src1, vcc
            w1 = words[i + 1]
            assert (w1 >> 18) & 0x1FF == 106, hex(w1)
            a, _ = _src(v, w1 & 0x1FF, words, i + 2, M)
            b, _ = _src(v, (w1 >> 9) & 0x1FF, words, i + 2, M)
            setf(w & 0xFF, np.where(vcc, b, a))
            i += 2
            continue
        assert (w >> 31) == 0, hex(w)  # VOP2
        a, n = _src(v, w & 0x1FF, words, i + 1, M)
        b = v[(w >> 9) & 0xFF].view(np.float32)
        op, d = w >> 25, (w >> 17) & 0xFF
        with np.errstate(all="ignore"):
            if op == 1:
                setf(d, a + b)
            elif op == 2:
                setf(d, a - b)
            elif op == 3:
                setf(d, b - a)
            elif op == 5:
                setf(d, a * b)
            elif op == 21:
                v[d] = a.view(np.uint32) ^ b.view(np.uint32)
            elif op == 19:
                v[d] = a.view(np.uint32) & b.view(np.uint32)
            else:
                raise AssertionError(hex(w))
        i += 1 + n


def _case(seed, D, K, n_trees=24, depth=6, ops=None):
    names = [f"x{i}" for i in range(D + K)]
    lib = mt.NodeLibrary((ops or CONTROL_OPS) + EXT, [names], [1])
    pop = sample_population(seed, lib, n_trees, 1, max_init_depth=depth, max_nodes=64)[0]
    nl = lib.native()
    return [_flatten(pop[p, 0], nl, D + K) for p in range(pop.shape[0])]


def _lanes(rng, D, K, M=64):
    scale = rng.choice([0.1, 1.0, 3.0, 50.0], size=(D, 1)).astype(F32)
    vals = (rng.standard_normal((D, M)) * scale).astype(F32)
    if D:  # a +0 and a -0 lane
        vals[:, 0] = 0.0
        vals[:, 1] = -0.0
    tans = rng.standard_normal((D, M)).astype(F32)
    kk = rng.integers(-1, K, size=M).astype(np.int32)
    theta = (rng.standard_normal(K) * 2).astype(F32)
    return vals, tans, kk, theta


@pytest.mark.parametrize("seed,D,K", [(1, 4, 3), (2, 7, 1), (3, 2, 6), (4, 8, 2), (5, 0, 4)])
def test_dual_units_emulate_to_the_dual_interpreter(seed, D, K):
    rng = np.random.default_rng(seed)
    progs = _case(seed, D, K)
    vals, tans, kk, theta = _lanes(rng, D, K)
    n_ok = 0
    for prog in progs:
        words = _translate(prog, D, theta)
        gv, gd = _emulate_dual(words, vals, tans, kk)
        rv, rd = _run_dual(prog, D, theta, vals, tans, kk)
        np.testing.assert_array_equal(gv.view(np.uint32), rv.view(np.uint32))
        np.testing.assert_array_equal(gd.view(np.uint32), rd.view(np.uint32))
        n_ok += 1
    assert n_ok == len(progs)


def _asm(rows):
    """A program from (opcode name, imm float or slot, aux slot) rows (hand-made: forms the random
    trees rarely produce)."""
    out = []
    for name, imm, aux in rows:
        code = nat.OP_NAMES.index(name)
        if isinstance(imm, float):
            ib = int(np.array([imm], F32).view(np.uint32)[0])
        else:
            ib = int(imm) * nat.SLOT_BYTES
        out.append((code << 24 | int(aux) * nat.SLOT_BYTES, ib))
    out.append((nat.OP_NAMES.index("END") << 24, 0))
    return np.array(out, np.uint32)


HAND = [
    [("LDV", 0, 0), ("LDCP", 1.5, 0), ("ADDS", 0, 0)],
    [("LDV", 4, 0), ("LDCP", -0.0, 0), ("RDIVS", 0, 0), ("LDCP", 2.0, 0), ("MULS", 0, 0)],
    [("LDV", 1, 0), ("LDVP", 5, 0), ("RSUBS", 0, 0), ("SINVP", 6, 0), ("DIVS", 0, 0)],
    [("VV_DIV", 5, 6), ("VVP_MUL", 4, 4), ("SUBS", 0, 0), ("ABS", 0, 0), ("COSVP", 2, 0), ("MULS", 0, 0)],
    [("VC_RDIV", 0.25, 5), ("VCP_RSUB", 1.0, 4), ("RSUBS", 0, 0), ("LOG", 0, 0), ("SQRT", 0, 0), ("TANH", 0, 0),
     ("EXP", 0, 0)],
    [("LDC", 0.0, 0), ("ABS", 0, 0), ("ADDV", 5, 0), ("RDIVV", 6, 0), ("MULC", -3.0, 0), ("DIVC", 0.5, 0)],
]


@pytest.mark.parametrize("rows", HAND)
def test_dual_hand_programs_emulate_to_the_dual_interpreter(rows):
    """Stack forms, parameter operands on both sides, -0 constants, chains of unary operators."""
    D, K = 4, 3
    rng = np.random.default_rng(len(rows))
    vals, tans, kk, theta = _lanes(rng, D, K)
    prog = _asm(rows)
    words = _translate(prog, D, theta)
    gv, gd = _emulate_dual(words, vals, tans, kk)
    rv, rd = _run_dual(prog, D, theta, vals, tans, kk)
    np.testing.assert_array_equal(gv.view(np.uint32), rv.view(np.uint32))
    np.testing.assert_array_equal(gd.view(np.uint32), rd.view(np.uint32))


def test_dual_units_cover_every_opcode_family():
    """The random programs and the hand-made ones above exercise every opcode."""
    seen = set()
    for seed in range(1, 40):
        for prog in _case(seed, 4, 3, n_trees=12):
            seen |= {nat.OP_NAMES[int(w) >> 24] for w, _ in prog}
    for rows in HAND:
        seen |= {n for n, _, _ in rows}
    missing = set(nat.OP_NAMES) - seen
    assert not missing, missing


def test_dual_units_disassemble_and_respect_the_abi():
    rng = np.random.default_rng(7)
    vals, tans, kk, theta = _lanes(rng, 6, 3)
    allowed = set(range(8, 30)) - {25} | set(range(56, 65))
    for prog in _case(7, 6, 3, n_trees=10):
        lines = _disassemble(_translate(prog, 6, theta))
        assert lines[-1] == "s_setpc_b64 s[30:31]", lines[-1]
        for ln in lines[:-1]:
            assert "invalid" not in ln.lower() and "exec" not in ln, ln
            op, _, rest = ln.partition(" ")
            dst = rest.split(",")[0].strip()
            if op.startswith("v_cmp"):
                assert dst == "vcc", ln
                continue
            m = re.fullmatch(r"v(\d+)|v\[(\d+):(\d+)\]", dst)
            if m:
                assert all(int(x) in allowed for x in m.groups() if x is not None), ln
                continue
            assert re.fullmatch(r"s\[(\d+):(\d+)\]|s(\d+)", dst), ln
            assert all(30 <= int(x) <= 45 for x in re.findall(r"\d+", dst)), ln


def test_dual_word_bound_and_rejections():
    """Every instruction stays within MTGP_GRAD_JIT_WORDS_PER_INSTR words (the buffer bound of
    MTGP_GRAD_JIT_BYTES); a slot past the coefficients and more than 8 data slots do not translate."""
    rng = np.random.default_rng(3)
    for D, K in ((4, 3), (8, 8)):
        theta = rng.standard_normal(K).astype(F32)
        for prog in _case(11, D, K, n_trees=30, depth=8):
            n = len(_translate(prog, D, theta))
            assert n <= len(prog) * nat.GRAD_JIT_WORDS_PER_INSTR
    lib = nat.load()
    prog = _case(12, 4, 3, n_trees=1)[0]
    th = np.zeros(3, F32)
    p = np.ascontiguousarray(prog, np.uint32)
    assert lib.mtgp_jit_dual_translate_host(p.ctypes.data, p.shape[0], 9, th.ctypes.data, 3, TEMPLATE_BYTES,
                                            None, 0) < 0
    reads_param = any((int(w) >> 24) != 11 and (int(i) // nat.SLOT_BYTES) >= 4 for w, i in prog)
    if reads_param:
        assert lib.mtgp_jit_dual_translate_host(p.ctypes.data, p.shape[0], 4, th.ctypes.data, 0, TEMPLATE_BYTES,
                                                None, 0) < 0
