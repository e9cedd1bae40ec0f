"""Program JIT (multitreegp_amd/csrc/mtgp_jit.h) checked on the CPU before any GPU runs it.

* the committed templates (mtgp_jit_blobs.h) are what scripts/gen_jit_templates.py assembles;
* every translated program disassembles cleanly with llvm-mc (gfx950), ends in
  s_setpc_b64 s[30:31] and writes only the registers the call-site ABI allows
  (v8-v24, s[32:39], vcc; never v0-v7, exec or other SGPRs);
* a word-level emulator of the emitted subset (v_mov / v_add / v_sub / v_subrev / v_mul, the
  templates and subroutine calls as black boxes) reproduces the row-order oracle bit for bit on
  random trees and data, which pins operand order and the compile-time operand stack;
* instruction-level emulators of the templates themselves (sin / cos hot path, exp / log / tanh /
  sqrt) reproduce the include/mtgp_f32math.h specs bit for bit on edge and random inputs."""
import os
import ctypes
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETPC_S40 = 0xBE801D28  # s_setpc_b64 s[40:41] (the sin/cos subroutine return)
LLVM_MC = "/opt/rocm/lib/llvm/bin/llvm-mc"

from multitreegp_amd import _native as nat  # noqa: E402
from multitreegp_amd.sampling import sample_population  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from helpers import CONTROL_OPS, SR_OPS  # noqa: E402
import multitreegp_amd as mt  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(nat.LIB_PATH), reason="libmtgp_hip.so not built")


def _blobs():
    text = open(os.path.join(ROOT, "multitreegp_amd", "csrc", "mtgp_jit_blobs.h")).read()
    out = {}
    for name, body in re.findall(r"mtgp_jit_(\w+)_blob\[\d+\] = \{(.*?)\};", text):
        out[name.upper()] = [int(x.rstrip("u"), 16) for x in body.split(",")]
    return out


BLOBS = _blobs()
SETPC = 0xBE801D1E
GETPC_S44 = 0xBEAC1C00  # s_getpc_b64 s[44:45] -- starts a call of a shared subroutine


def _defines():
    text = open(os.path.join(ROOT, "multitreegp_amd", "csrc", "mtgp_jit_blobs.h")).read()
    return {k: int(v) for k, v in re.findall(r"#define MTGP_JIT_(\w+) (\d+)u?", text)}


DEFS = _defines()
TEMPLATE_BYTES = DEFS["SUB_WORDS"] * 4  # host translations start right after the subroutine area
FN = {"SIN": 6, "COS": 7, "EXP": 8, "LOG": 9, "SQRT": 10, "TANH": 11}  # include/mtgp.h MTGP_FN_*
SUB_AT = {DEFS[name + "_OFFSET"]: name for name in FN}  # byte offset -> subroutine


def test_templates_up_to_date():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_jit_templates.py"), "--check"])
    assert r.returncode == 0, "mtgp_jit_blobs.h is stale: rerun scripts/gen_jit_templates.py"


def _programs(lib, pop, n_data, masks):
    nl = lib.native()
    progs = []
    for p in range(pop.shape[0]):
        for t in range(pop.shape[1]):
            for zm in masks:
                instrs, _ = nat.flatten_tree_host(pop[p, t], nl, n_data, zm)
                raw = _raw_program(pop[p, t], nl, n_data, zm)
                progs.append((p, t, zm, raw))
    return progs


def _raw_program(tree, nl, n_data, zm):
    import ctypes
    lib = nat.load()
    t = np.ascontiguousarray(tree, np.float32)
    L = 2 * t.shape[0] + 8
    out = (nat.MtgpInstr * L)()
    need = ctypes.c_int32(0)
    n = lib.mtgp_flatten_tree_host(t.ctypes.data, t.shape[0], ctypes.byref(nl), n_data, zm, L, ctypes.addressof(out),
                                   ctypes.byref(need))
    assert n > 0
    return np.frombuffer(bytes(out), dtype=np.uint32).reshape(-1, 2)[: n + 1].copy()


def _disassemble(words):
    text = " ".join(f"0x{(w >> (8 * b)) & 0xff:02x}" for w in words for b in range(4))
    r = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "--disassemble"], input=text.encode(),
                       capture_output=True)
    assert r.returncode == 0 and not r.stderr.strip(), r.stderr.decode()[:500]
    return [ln.strip() for ln in r.stdout.decode().splitlines() if ln.strip()]


ALLOWED_V = set(range(8, 26))
ALLOWED_S = set(range(30, 46))
EXEC_OK = ("s_mov_b64 s[40:41], exec", "s_mov_b64 exec, s[40:41]", "s_mov_b64 exec, s[36:37]")


def _check_abi(lines):
    assert lines[-1] == "s_setpc_b64 s[30:31]", lines[-1]
    for ln in lines[:-1]:
        if ln in EXEC_OK or ln.startswith("s_mov_b32 exec_lo, ") or ln.startswith("s_mov_b32 exec_hi, ") or \
                ln.startswith("s_and_saveexec_b64 s[36:37]") or ln.startswith("s_cbranch_execz"):
            continue
        assert "exec" not in ln and "invalid" not in ln.lower(), ln
        op, _, rest = ln.partition(" ")
        dst = rest.split(",")[0].strip()
        if op.startswith("s_nop"):
            continue
        if op.startswith("v_cmp") and op.endswith("_e32"):
            assert dst == "vcc", ln
            continue
        m = re.fullmatch(r"v(\d+)|v\[(\d+):(\d+)\]", dst)
        if m:
            assert all(int(x) in ALLOWED_V for x in m.groups() if x is not None), ln
            # the vcc / sgpr written by v_div_scale / v_cmp_e64 (second operand) is checked below
            if op.startswith("v_div_scale"):
                sd = rest.split(",")[1].strip()
                assert sd == "vcc" or re.fullmatch(r"s\[(\d+):(\d+)\]", sd) and \
                    all(int(x) in ALLOWED_S for x in re.findall(r"\d+", sd)), ln
            continue
        m = re.fullmatch(r"s\[(\d+):(\d+)\]|s(\d+)", dst)
        assert m, ln
        regs = [int(x) for x in m.groups() if x is not None]
        assert all(r in ALLOWED_S for r in regs), ln


def _setup(kind):
    if kind == "dynamic":
        lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
        pop = sample_population(5, lib, 40, 1, max_init_depth=8, max_nodes=64)[0]
        return lib, pop, 7, [0, 0b1001111]
    if kind == "sr":
        lib = mt.NodeLibrary(SR_OPS, [["x0", "x1", "x2", "x3"]], [4])
        pop = sample_population(6, lib, 30, 1, max_init_depth=7, max_nodes=64)[0]
        return lib, pop, 4, [0]
    if kind == "ext":  # the round-3 unary operators: subroutine calls / inline abs since round 4
        ext = [("exp", None, 1, 0.2), ("log", None, 1, 0.2), ("sqrt", None, 1, 0.2), ("tanh", None, 1, 0.2),
               ("abs", None, 1, 0.2)]
        lib = mt.NodeLibrary(SR_OPS + ext, [["x0", "x1", "x2", "x3"]], [4])
        pop = sample_population(16, lib, 40, 1, max_init_depth=7, max_nodes=64)[0]
        return lib, pop, 4, [0]
    lib = mt.NodeLibrary(CONTROL_OPS + [("/", None, 2, 0.1)], [["y1", "y2", "y3", "y4"]], [1])
    pop = sample_population(7, lib, 60, 1, max_init_depth=6, max_nodes=40)[0]
    return lib, pop, 4, [0]


class FellThrough(Exception):
    """The emulated unit ended without returning (a role-chain member falls into the next unit)."""

    def __init__(self, regs):
        super().__init__("fell through")
        self.regs = regs


def _emulate(words, data, full=False, lds=False, regs=None, s46=0, lds_out=None):
    """Run emitted code on data [n_data, M] (float32 lanes, M <= 64); returns v8 (or all VGPRs).
    Honours the exec moves of per-wave units (VALU results only land in exec lanes).  lds: the
    data vector is the LDS stage vector (LDS-data mode: ds_read_b32 from v0 + slot * 256).
    regs: VGPRs to start from (a chain's next unit); s46: the chain-continuation flag; a unit that
    ends without returning raises FellThrough(regs)."""
    M = data.shape[1]
    if regs is not None:
        v = regs
    else:
        v = np.zeros((64, M), np.float32)
        if not lds:
            v[: data.shape[0]] = data
    i = 0
    lit = lambda k: np.full(M, np.array(words[k], np.uint32).view(np.float32), np.float32)  # noqa: E731
    exec_ = np.ones(M, bool)
    saved = None
    sel = [0, 0]

    def put(dst, val):
        v[dst] = np.where(exec_, val, v[dst])

    while True:
        if i >= len(words):
            raise FellThrough(v)
        w = words[i]
        if w == SETPC:
            return v if full else v[8]
        if words[i:i + 3] == [0xBF06802E, 0xBF840001, SETPC]:  # s_cmp_eq_u32 s46, 0; s_cbranch_scc0 +1; s_setpc
            if s46 == 0:
                return v if full else v[8]
            i += 3
            continue
        if (w & 0xFFFF0000) == 0xD8700000:  # ds_read2st64_b32 v[d:d+1], v0 offset0:s0 offset1:s1 (slots)
            assert lds and (words[i + 1] & 0xFF) == 0 and (words[i + 1] >> 24) % 2 == 0, hex(words[i + 1])
            put(words[i + 1] >> 24, data[w & 0xFF])
            put((words[i + 1] >> 24) + 1, data[(w >> 8) & 0xFF])
            i += 2
            continue
        if (w & 0xFFFF0000) == 0xD86C0000:  # ds_read_b32 vdst, v0 offset:slot*256
            assert lds and (words[i + 1] & 0xFF) == 0, hex(words[i + 1])
            put(words[i + 1] >> 24, data[(w & 0xFFFF) // 256])
            i += 2
            continue
        if (w & 0xFFFFF0FF) == 0xBF8CC07F:  # s_waitcnt lgkmcnt(n) (the emulator's loads complete at once)
            i += 1
            continue
        if (w & 0xFFFF0000) == 0xD81A0000 and words[i + 1] == 0x00000801:  # ds_write_b32 v1, v8 offset:j*256
            lds_out[(w & 0xFFFF) // 256] = v[8].copy()
            i += 2
            continue
        if w == GETPC_S44:  # getpc; s_add_u32 s44, lit; s_addc_u32 s45; s_swappc_b64 s[40:41], s[44:45]
            assert words[i + 1] == 0x802CFF2C and words[i + 4] == 0xBEA81E2C, [hex(x) for x in words[i:i + 5]]
            rel = int(np.array(words[i + 2], np.uint32).view(np.int32))
            target = TEMPLATE_BYTES + 4 * (i + 1) + rel
            assert target in SUB_AT, target
            put(8, orc.unary(FN[SUB_AT[target]], v[17]))
            i += 5
            continue
        if (w >> 23) == 0x17D:  # SOP1: the exec save / restore / set of per-wave units
            sdst, op, ssrc = (w >> 16) & 0x7F, (w >> 8) & 0xFF, w & 0xFF
            if (sdst, op, ssrc) == (40, 1, 126):
                saved = exec_.copy()
                i += 1
            elif (sdst, op, ssrc) == (126, 1, 40):
                exec_ = saved.copy()
                i += 1
            elif op == 0 and ssrc == 255 and sdst in (126, 127):
                bits = words[i + 1]
                lo = 0 if sdst == 126 else 32
                for lane in range(lo, min(lo + 32, M)):
                    exec_[lane] = bool(bits >> (lane - lo) & 1)
                i += 2
            elif op == 0 and ssrc == 255 and sdst in (42, 43):  # lane mask of a wave unit's select
                sel[sdst - 42] = words[i + 1]
                i += 2
            else:
                raise AssertionError(hex(w))
            continue
        if (w & 0xFFFF0000) == 0x91AA0000:  # s_bfm_b64 s[42:43], width, offset: group 1's lane mask
            width, off = (w & 0xFF) - 128, ((w >> 8) & 0xFF) - 128
            m64 = (((1 << width) - 1) << off) & 0xFFFFFFFFFFFFFFFF
            sel = [m64 & 0xFFFFFFFF, m64 >> 32]
            i += 1
            continue
        if (w & 0xFFFF00FF) == 0x8EAA002A:  # s_lshl_b64 s[42:43], s[42:43], n: the next group's lane mask
            m64 = ((sel[0] | sel[1] << 32) << (((w >> 8) & 0xFF) - 128)) & 0xFFFFFFFFFFFFFFFF
            sel = [m64 & 0xFFFFFFFF, m64 >> 32]
            i += 1
            continue
        if words[i:i + 2] == [0xD1000019, 0x00AA1119]:  # v_cndmask_b32_e64 v25, v25, v8, s[42:43] (running result)
            m64 = sel[0] | sel[1] << 32
            lanes = np.array([bool(m64 >> lane & 1) for lane in range(M)])
            put(25, np.where(lanes, v[8], v[25]))
            i += 2
            continue
        if words[i:i + 2] == [0xD1000008, 0x00AA1119]:  # v_cndmask_b32_e64 v8, v25, v8, s[42:43]
            m64 = sel[0] | sel[1] << 32
            lanes = np.array([bool(m64 >> lane & 1) for lane in range(M)])
            put(8, np.where(lanes, v[8], v[25]))
            i += 2
            continue
        hit = None
        for name, b in BLOBS.items():
            if words[i:i + len(b)] == b:
                hit = name
                break
        if hit == "DIV":
            with np.errstate(all="ignore"):
                put(8, v[17] / v[18])
            i += len(BLOBS["DIV"])
            continue
        if hit in ("SIN", "COS"):
            s, c = orc.sincos(v[17])
            put(8, s if hit == "SIN" else c)
            i += len(BLOBS[hit])
            continue
        if hit == "ABS":
            put(8, orc.unary(12, v[8]))
            i += len(BLOBS[hit])
            continue
        src0 = w & 0x1FF
        if src0 == 255:
            a = lit(i + 1)
            step = 2
        else:
            assert src0 >= 256, hex(w)
            a = v[src0 - 256].copy()
            step = 1
        vdst = (w >> 17) & 0xFF
        if (w >> 25) == 0x3F:  # VOP1
            assert ((w >> 9) & 0xFF) == 1, hex(w)  # v_mov_b32
            put(vdst, a)
        else:
            assert (w >> 31) == 0, hex(w)
            b = v[(w >> 9) & 0xFF]
            op = w >> 25
            with np.errstate(all="ignore"):
                put(vdst, {1: lambda: a + b, 2: lambda: a - b, 3: lambda: b - a, 5: lambda: a * b}[op]())
        i += step


@pytest.mark.parametrize("kind", ["dynamic", "static_div", "sr", "ext"])
def test_translation_disassembles_and_respects_abi(kind):
    lib, pop, n_data, masks = _setup(kind)
    progs = _programs(lib, pop[:12], n_data, masks)
    words_all = []
    for (_, _, _, raw) in progs:
        words = nat.jit_translate_host(raw)
        words_all.append(words)
        lines = _disassemble([int(w) for w in words])
        _check_abi(lines)
    assert len(words_all) >= 12


@pytest.mark.parametrize("kind", ["dynamic", "static_div", "sr", "ext"])
def test_emulated_code_matches_row_order_oracle(kind):
    lib, pop, n_data, masks = _setup(kind)
    rng = np.random.default_rng(3)
    data = (rng.standard_normal((n_data, 33)) * 2.5).astype(np.float32)
    data[:, 0] = 0.0
    data[:, 1] = [1e6, -3e5, 2.0, 0.5, -0.0, 7.0, 1e-30][:n_data]  # large / tiny / signed-zero lanes
    checked = 0
    for (p, t, zm, raw) in _programs(lib, pop, n_data, masks):
        words = [int(w) for w in nat.jit_translate_host(raw)]
        got = _emulate(words, data)
        d = data.copy()
        for k in range(n_data):
            if zm >> k & 1:
                d[k] = 0.0
        want = np.array([orc.eval_tree(pop[p, t], lib.fn_codes, lib.n_funcs, lib.var_start, d[:, m])
                         for m in range(d.shape[1])], np.float32)
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (p, t, zm, got[~same][:4], want[~same][:4])
        checked += 1
    assert checked >= 30


def test_translation_rejects_wide_slots():
    raw = np.array([[nat.OP_NAMES.index("LDV") << nat.OP_SHIFT, 9 * nat.SLOT_BYTES],
                    [nat.OP_NAMES.index("END") << nat.OP_SHIFT, 0]], np.uint32)
    with pytest.raises(ValueError):
        nat.jit_translate_host(raw)


def _host_flatten(ff, lib, pop):
    """Programs [P, n_prog, L, 2] of a population as the device flattener lays them out."""
    specs, roles = ff.program_specs()
    nl = lib.native()
    P, T, N, _ = pop.shape
    L = (2 * N + 8 + 3) // 4 * 4
    prog = np.zeros((P, len(specs), L, 2), np.uint32)
    for p in range(P):
        for j, (t, nd, zm) in enumerate(sp[:3] for sp in specs):
            raw = _raw_program(pop[p, t], nl, nd, zm)
            prog[p, j, : raw.shape[0]] = raw
    return prog, specs, roles, L


@pytest.mark.parametrize("kind,R", [("dynamic", 32), ("dynamic", 8), ("static", 16), ("sr", 16), ("sr", 64)])
def test_wave_units_emulate_to_oracle(kind, R):
    """(wave, program) units: the G individuals' programs back to back, merged per lane group
    with v_cndmask, checked lane by lane against the oracle of each lane's own individual."""
    import ctypes
    if kind == "dynamic":
        lib, pop, n_data, _ = _setup("dynamic")
        ff = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05)
    elif kind == "static":
        lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1])
        pop = sample_population(8, lib, 40, 1, max_init_depth=6, max_nodes=40)[0]
        ff = mt.FeedforwardEvaluator(mt.Acrobot(0, 0), 0.05)
        n_data = 4
    else:
        lib, pop, n_data, _ = _setup("sr")
        ff = mt.SREvaluator(dt0=0.05)
        ff._n_var = 4
    prog, specs, roles, L = _host_flatten(ff, lib, pop)
    P, n_prog = prog.shape[:2]
    order = np.random.default_rng(1).permutation(P).astype(np.int32)
    lib_n = nat.load()
    units = lib_n.mtgp_jit_units(P, n_prog, R)
    Rp = 1 << max(R - 1, 0).bit_length()
    G = 64 // Rp
    assert units == -(-P // G) * n_prog
    rng = np.random.default_rng(2)
    out = np.zeros(1 << 16, np.uint32)
    for u in range(units):
        n = lib_n.mtgp_jit_unit_host(prog.ctypes.data, P, n_prog, L, R, order.ctypes.data, u, out.ctypes.data,
                                     out.size)
        assert n > 0, n
        words = [int(x) for x in out[:n]]
        _check_abi(_disassemble(words))
        data = (rng.standard_normal((8, 64)) * 2).astype(np.float32)
        regs = _emulate(words, data, full=True)
        wave, j = divmod(u, n_prog)
        t, nd, zm = specs[j][:3]
        for lane in range(64):
            g = lane // Rp
            q = wave * G + g
            if q >= P:
                continue
            d = data[:n_data, lane].copy()
            for b in range(nd):
                if zm >> b & 1:
                    d[b] = 0.0
            want = orc.eval_tree(pop[order[q], t], lib.fn_codes, lib.n_funcs, lib.var_start, d)
            got = regs[8, lane]
            assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32) or \
                (np.isnan(got) and np.isnan(want)), (u, lane, got, want)


def test_trig_templates_hot_path_and_slow_blocks():
    """The sin/cos templates (spec v2): a straight-line hot path up to the return whose only
    branch is the (normally not taken) jump to the out-of-line slow blocks; those blocks mask
    exec, restore it and branch back; no lane is ever sent to the interpreter (s[32:33])."""
    for name in ("SIN", "COS"):
        w = BLOBS[name]
        ret = w.index(SETPC_S40)
        hot = _disassemble(w[:ret + 1])
        assert [ln.split()[0] for ln in hot if ln.startswith("s_cbranch")] == ["s_cbranch_vccnz"]
        assert not any("exec" in ln and not ln.startswith("s_and_b64 vcc, exec") for ln in hot)
        cold = _disassemble(w[ret + 1:])
        assert any(ln.startswith("s_and_saveexec_b64") for ln in cold)
        assert cold[-1].startswith("s_branch")
        assert not any("s[32:33]" in ln for ln in hot + cold)


def _emulate_trig_template(text, x):
    """Instruction-level float32 emulation of the HOT path of a sin/cos template (up to its
    s_setpc) on lanes x -> (v8, lanes that branch to the out-of-line slow blocks).  The slow
    blocks (double Cody-Waite, Payne-Hanek) are checked on the GPU (scripts/micro/jit_smoke.hip,
    test_gpu_parity slow-lane tests).  fma via float64 (exact product, one rounding)."""
    f32 = np.float32
    v = {17: x.astype(f32)}
    sg = {}
    vcc = None
    slow = np.zeros(x.shape, bool)
    u = lambda a: a.view(np.uint32)  # noqa: E731

    def val(o):
        if o.startswith("v"):
            return v[int(o[1:])]
        if o.startswith("s") and o[1:].isdigit():
            return np.full(x.shape, np.array(sg[int(o[1:])], np.uint32).view(f32))
        if o.startswith("0x"):
            return np.full(x.shape, np.array(int(o, 16), np.uint32).view(f32))
        return np.full(x.shape, f32(float(o)))

    def fma(a, b, c):
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)

    masks = {}
    for ln in text.strip().splitlines():
        if ln.endswith(":"):
            continue
        op, *rest = ln.split(None, 1)
        a = [t.strip() for t in rest[0].split(",")] if rest else []
        d = int(a[0][1:]) if a and a[0][:1] == "v" and a[0][1:].isdigit() else None
        with np.errstate(all="ignore"):
            if op == "v_and_b32":
                v[d] = (np.uint32(int(a[1], 16)) & u(val(a[2]))).view(f32)
            elif op == "s_mov_b32":
                sg[int(a[0][1:])] = int(a[1], 16) if a[1].startswith("0x") else int(a[1])
            elif op == "v_cmp_gt_f32_e64":
                masks[a[0]] = val(a[1]) > val(a[2])
            elif op == "v_subrev_u32":  # vdst = src1 - src0
                v[d] = (u(val(a[2])) - u(val(a[1]))).view(f32)
            elif op == "v_cmp_gt_u32_e32":
                vcc = u(val(a[1])) > u(val(a[2]))
            elif op == "s_and_b64":
                pass  # vcc &= exec (full)
            elif op == "s_cbranch_vccnz":
                slow = vcc.copy()
            elif op == "v_mul_f32":
                v[d] = (val(a[1]) * val(a[2])).astype(f32)
            elif op == "v_add_f32":
                v[d] = (val(a[1]) + val(a[2])).astype(f32)
            elif op == "v_rndne_f32":
                v[d] = np.rint(val(a[1]))
            elif op in ("v_fma_f32", "v_fmamk_f32", "v_fmaak_f32"):
                v[d] = fma(val(a[1]), val(a[2]), val(a[3]))
            elif op == "v_cvt_i32_f32":  # saturating, NaN -> 0
                t = val(a[1]).astype(np.float64)
                t = np.where(np.isnan(t), 0, np.clip(t, -2.0 ** 31, 2.0 ** 31 - 1))
                v[d] = t.astype(np.int64).astype(np.int32).view(f32)
            elif op == "v_add_u32":
                v[d] = (val(a[2]).view(np.int32) + np.int32(int(a[1]))).astype(np.int32).view(f32)
            elif op == "v_lshlrev_b32":
                v[d] = (u(val(a[2])) << np.uint32(int(a[1]))).view(f32)
            elif op == "v_xor_b32":
                v[d] = (u(val(a[1])) ^ u(val(a[2]))).view(f32)
            elif op == "v_mov_b32":
                v[d] = val(a[1])
            elif op == "v_cndmask_b32_e64":
                v[d] = np.where(masks[a[3]], val(a[2]), val(a[1]))
            elif op == "s_setpc_b64":
                return v[8], slow
            elif op != "s_nop":
                raise AssertionError(op)
    raise AssertionError("no s_setpc")


def test_trig_templates_emulate_to_spec():
    """Every hot-path lane of the sin/cos templates equals the spec (oracle) bit for bit --
    NaN, infinities, signed zeros, denormals, tiny, the 2^17 edge and random arguments; the
    lanes sent to the out-of-line slow blocks are exactly the finite |x| >= 2^17."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_jit_templates", os.path.join(ROOT, "scripts",
                                                                                     "gen_jit_templates.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-200, 200, 100000), rng.uniform(-2e5, 2e5, 50000),
                        [np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-30, -1e-40, 2.44e-4, 131071.99, 131072.0,
                         -131072.0, 1e-3, np.pi / 2, -np.pi, 3e38]]).astype(np.float32)
    s_ref, c_ref = orc.sincos(x)
    for name, ref in (("SIN", s_ref), ("COS", c_ref)):
        got, flag = _emulate_trig_template(g.TEMPLATES[name], x)
        same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
        assert np.all(same | flag), (name, x[~(same | flag)][:5], got[~(same | flag)][:5])
        assert np.array_equal(flag, ~(np.abs(x) < 131072.0) & np.isfinite(x)), name


def _lds_setup():
    lib = mt.NodeLibrary(SR_OPS, [[f"x{i}" for i in range(24)]], [24])
    pop = sample_population(9, lib, 30, 1, max_init_depth=9, max_nodes=96)[0]
    return lib, pop, 24


def test_lds_mode_translation_disassembles_and_emulates_to_oracle():
    """LDS-data mode (the wide-state SR kernel): every program preloads its first 16 distinct data
    slots from v0 + slot * 256 (pairs with ds_read2st64_b32, an odd last one with ds_read_b32; one
    s_waitcnt), loads the rest at their use, and
    computes the row-order oracle's value bit for bit; registers stay within v8-v43 / the ABI."""
    import ctypes
    lib, pop, n_data = _lds_setup()
    nl = lib.native()
    lib_n = nat.load()
    rng = np.random.default_rng(4)
    data = (rng.standard_normal((n_data, 17)) * 2.0).astype(np.float32)
    out = np.zeros(1 << 15, np.uint32)
    checked = beyond = 0
    allowed = set(range(8, 44))
    for p in range(pop.shape[0]):
        for t in range(n_data):
            raw = _raw_program(pop[p, t], nl, n_data, 0)
            n = lib_n.mtgp_jit_translate_host_ex(raw.ctypes.data, raw.shape[0], out.ctypes.data, out.size, 1)
            assert n > 0, n
            words = [int(w) for w in out[:n]]
            lines = _disassemble(words)
            assert lines[-1] == "s_setpc_b64 s[30:31]"
            for ln in lines[:-1]:
                if ln.startswith("ds_read_b32"):
                    dst = int(re.match(r"ds_read_b32 v(\d+), v0", ln).group(1))
                    assert dst in allowed, ln
                    beyond += dst >= 42
                    continue
                if ln.startswith("ds_read2st64_b32"):  # a preload pair (round 4): even-aligned, v26..v41
                    lo, hi = (int(x) for x in re.match(r"ds_read2st64_b32 v\[(\d+):(\d+)\], v0", ln).groups())
                    assert lo % 2 == 0 and hi == lo + 1 and 26 <= lo and hi <= 41, ln
                    continue
                if ln.startswith("s_waitcnt"):
                    continue
                dst = ln.partition(" ")[2].split(",")[0].strip()
                m = re.fullmatch(r"v(\d+)", dst)
                assert m and int(m.group(1)) in allowed, ln
            got = _emulate(words, data, lds=True)
            want = np.array([orc.eval_tree(pop[p, t], lib.fn_codes, lib.n_funcs, lib.var_start, data[:, m])
                             for m in range(data.shape[1])], np.float32)
            same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
            assert same.all(), (p, t, got[~same][:4], want[~same][:4])
            checked += 1
    assert checked >= 600


def _chain_model(kind):
    m = nat.MtgpModel()
    if kind == "dynamic":
        m.model, m.state_size, m.n_var = nat.MODEL_ACROBOT_DYNAMIC, 2, 4
        m.prog_state, m.prog_readout, m.prog_readout_save, m.readout_save_same = 1, 0, 3, -1
    else:
        m.model, m.n_var, m.prog_state = nat.MODEL_SR, 4, 0
    m.solver = nat.SOLVER_RK4
    return m


def test_chain_masks():
    """mtgp_jit_chain: the dynamic policy chains its state programs, register-resident SR its n_var
    trees; wide SR and static policies have no chain.  (ABI v18: no save-point continuation -- the
    save readout reads the dense-output state, so no solver asks for one; the emitter keeps the
    conditional form, tested below with an explicit chain.)"""
    lib_n = nat.load()
    ch = nat.MtgpJitChain()
    m = _chain_model("dynamic")
    assert lib_n.mtgp_jit_chain(ctypes.byref(m), 4, ctypes.byref(ch)) == 0
    # fixed step (ABI v18): readout -> u into data slot n_var + state_size -> the state programs
    assert (ch.next, ch.cond, ch.put, ch.put_slot) == (0b011, 0, 0b001, 6)
    m.solver = nat.SOLVER_DOPRI5
    lib_n.mtgp_jit_chain(ctypes.byref(m), 4, ctypes.byref(ch))
    assert (ch.next, ch.cond, ch.put) == (0b010, 0, 0)
    m = _chain_model("sr")
    lib_n.mtgp_jit_chain(ctypes.byref(m), 4, ctypes.byref(ch))
    assert (ch.next, ch.cond) == (0b0111, 0)
    m.n_var = 12
    lib_n.mtgp_jit_chain(ctypes.byref(m), 12, ctypes.byref(ch))
    assert (ch.next, ch.cond) == (0, 0)
    m.model, m.n_var, m.prog_state, m.prog_readout = nat.MODEL_ACROBOT_STATIC, 4, -1, 0
    lib_n.mtgp_jit_chain(ctypes.byref(m), 1, ctypes.byref(ch))
    assert (ch.next, ch.cond) == (0, 0)


@pytest.mark.parametrize("kind,R", [("dynamic", 32), ("dynamic", 4), ("sr", 16)])
def test_role_chain_units_emulate_to_oracle(kind, R):
    """Role chains (ABI v13): the state programs of a wave run as one call -- each chain member
    copies its result to v26 + k and falls into the next unit, the last returns, or (dynamic,
    s46 != 0) continues into the save-point readout, which returns in v8.  Emulated unit by unit
    and checked lane by lane against the oracle; the code disassembles and writes only v8-v29 /
    the template SGPRs."""
    if kind == "dynamic":
        lib, pop, n_data, _ = _setup("dynamic")
        ff = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05)
    else:
        lib, pop, n_data, _ = _setup("sr")
        ff = mt.SREvaluator(dt0=0.05)
        ff._n_var = 4
    prog, specs, roles, L = _host_flatten(ff, lib, pop[:24])
    P, n_prog = prog.shape[:2]
    order = np.random.default_rng(4).permutation(P).astype(np.int32)
    lib_n = nat.load()
    ch = nat.MtgpJitChain()
    lib_n.mtgp_jit_chain(ctypes.byref(_chain_model(kind)), n_prog, ctypes.byref(ch))
    if kind == "dynamic":  # the conditional continuation into the save-point readout (ABI v13 form)
        ch.next, ch.cond, ch.put, ch.put_slot = 0b110, 0b100, 0, 0
    first = roles["prog_state"]
    members = [j for j in range(n_prog) if ch.next >> j & 1] + [j for j in range(n_prog) if
                                                                 j > 0 and ch.next >> (j - 1) & 1 and
                                                                 not ch.next >> j & 1]
    members = sorted(set(members))
    Rp = 1 << max(R - 1, 0).bit_length()
    G = 64 // Rp
    rng = np.random.default_rng(5)
    out = np.zeros(1 << 16, np.uint32)
    for wave in range(-(-P // G)):
        data = (rng.standard_normal((8, 64)) * 2).astype(np.float32)
        codes = {}
        for j in members:
            n = lib_n.mtgp_jit_unit_host_chain(prog.ctypes.data, P, n_prog, L, R, order.ctypes.data,
                                               ctypes.byref(ch), wave * n_prog + j, out.ctypes.data, out.size, 0)
            assert n > 0, n
            codes[j] = [int(x) for x in out[:n]]
            for ln in _disassemble(codes[j]):
                assert "invalid" not in ln.lower() and "exec" not in ln, ln
                m = re.fullmatch(r"v_\w+ v(\d+),.*", ln)
                if m:
                    assert 8 <= int(m.group(1)) <= 29, ln
        for s46 in ((0, 1) if ch.cond else (0,)):
            regs = None
            for j in members:
                try:
                    regs = _emulate(codes[j], data, full=True, regs=regs, s46=s46)
                    break
                except FellThrough as e:
                    regs = e.regs
            else:
                raise AssertionError("the chain never returned")
            n_state = len(members) - (1 if ch.cond else 0)
            for lane in range(64):
                q = wave * G + lane // Rp
                if q >= P:
                    continue
                outs = [(26 + k, first + k) for k in range(n_state)]
                if s46:
                    outs.append((8, roles["prog_readout_save"]))
                for reg, j in outs:
                    t, nd, zm = specs[j][:3]
                    d = data[:n_data, lane].copy()
                    for b in range(nd):
                        if zm >> b & 1:
                            d[b] = 0.0
                    want = orc.eval_tree(pop[order[q], t], lib.fn_codes, lib.n_funcs, lib.var_start, d)
                    got = regs[reg, lane]
                    assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32) or \
                        (np.isnan(got) and np.isnan(want)), (wave, lane, reg, got, want)


@pytest.mark.parametrize("R", [32, 4, 64])
def test_merged_readout_chain_emulates_to_oracle(R):
    """The fixed-step dynamic policy's put chain (ABI v18, MtgpJitChain.put): the readout unit
    computes u on [y, a, u, tar] with y and u folded to 0 and leaves it in v26 (its chain slot);
    the state units it falls into read their data slot 6 (u) from v26 instead of v6 and return in
    v27 / v28.  Emulated per wave against the oracle: u = readout([0, a, 0]), state_j =
    tree_j([y, a, u]); v6 itself is never written (the call site's data registers are inputs)."""
    lib, pop, n_data, _ = _setup("dynamic")
    ff = mt.DynamicEvaluator(mt.Acrobot(0, 0), 2, 0.05, solver=mt.RK4())
    prog, specs, roles, L = _host_flatten(ff, lib, pop[:24])
    P, n_prog = prog.shape[:2]
    order = np.random.default_rng(7).permutation(P).astype(np.int32)
    lib_n = nat.load()
    ch = nat.MtgpJitChain()
    lib_n.mtgp_jit_chain(ctypes.byref(_chain_model("dynamic")), n_prog, ctypes.byref(ch))
    assert ch.put == 1 and ch.put_slot == 6 and roles["prog_readout"] == 0 and roles["prog_state"] == 1
    Rp = 1 << max(R - 1, 0).bit_length()
    G = 64 // Rp
    rng = np.random.default_rng(8)
    out = np.zeros(1 << 16, np.uint32)
    for wave in range(-(-P // G)):
        data = (rng.standard_normal((8, 64)) * 2).astype(np.float32)
        codes = []
        for j in (0, 1, 2):
            n = lib_n.mtgp_jit_unit_host_chain(prog.ctypes.data, P, n_prog, L, R, order.ctypes.data,
                                               ctypes.byref(ch), wave * n_prog + j, out.ctypes.data, out.size, 0)
            assert n > 0, n
            codes.append([int(x) for x in out[:n]])
            for ln in _disassemble(codes[-1]):
                assert "invalid" not in ln.lower() and "exec" not in ln, ln
                mm = re.fullmatch(r"v_\w+ v(\d+),.*", ln)
                if mm:
                    assert 8 <= int(mm.group(1)) <= 29, ln
        regs = None
        for c in codes:
            try:
                regs = _emulate(c, data, full=True, regs=regs)
                break
            except FellThrough as e:
                regs = e.regs
        else:
            raise AssertionError("the chain never returned")
        for lane in range(64):
            q = wave * G + lane // Rp
            if q >= P:
                continue
            d = data[:n_data, lane].copy()
            t, nd, zm = specs[0][:3]
            dz = d.copy()
            for b in range(nd):
                if zm >> b & 1:
                    dz[b] = 0.0
            u = orc.eval_tree(pop[order[q], t], lib.fn_codes, lib.n_funcs, lib.var_start, dz)
            d[6] = u
            got = [regs[26, lane], regs[27, lane], regs[28, lane]]
            want = [u] + [orc.eval_tree(pop[order[q], specs[1 + k][0]], lib.fn_codes, lib.n_funcs, lib.var_start, d)
                             for k in range(2)]
            for g_, w_ in zip(got, want):
                assert np.float32(g_).view(np.uint32) == np.float32(w_).view(np.uint32) or \
                    (np.isnan(g_) and np.isnan(w_)), (wave, lane, got, want)


@pytest.mark.parametrize("R", [8, 64])
def test_lds_store_chain_units_emulate_to_oracle(R):
    """LDS store chains (ABI v14, the wide-state SR kernels): each unit writes its result to the
    output vector (ds_write_b32 v1, v8 offset:j*256) and falls into the next unit except at the
    kWideComp boundaries, where it waits and returns; one call per wave runs its components.
    Emulated per wave, every slot written equals the oracle of its lane's own individual."""
    lib, pop, n_data = _lds_setup()
    ff = mt.SREvaluator(dt0=0.05)
    ff._n_var = n_data
    prog, specs, roles, L = _host_flatten(ff, lib, pop[:20])
    P, n_prog = prog.shape[:2]
    order = np.random.default_rng(6).permutation(P).astype(np.int32)
    lib_n = nat.load()
    m = nat.MtgpModel()
    m.model, m.n_var, m.prog_state, m.solver = nat.MODEL_SR, n_data, 0, nat.SOLVER_RK4
    ch = nat.MtgpJitChain()
    assert lib_n.mtgp_jit_chain(ctypes.byref(m), n_prog, ctypes.byref(ch)) == 0
    assert (ch.next, ch.cond, ch.store) == (0, 0, 8)
    Rp = 1 << max(R - 1, 0).bit_length()
    G = 64 // Rp
    rng = np.random.default_rng(7)
    out = np.zeros(1 << 16, np.uint32)
    for wave in range(-(-P // G)):
        data = (rng.standard_normal((n_data, 64)) * 2).astype(np.float32)
        for c0 in range(0, n_prog, 8):
            lds_out, regs = {}, None
            for j in range(c0, min(c0 + 8, n_prog)):
                n = lib_n.mtgp_jit_unit_host_chain(prog.ctypes.data, P, n_prog, L, R, order.ctypes.data,
                                                   ctypes.byref(ch), wave * n_prog + j, out.ctypes.data, out.size, 1)
                assert n > 0, n
                words = [int(x) for x in out[:n]]
                last = j == min(c0 + 8, n_prog) - 1
                assert (words[-2:] == [0xBF8CC07F, SETPC]) == last, (j, [hex(x) for x in words[-3:]])
                try:
                    regs = _emulate(words, data, full=True, lds=True, regs=regs, lds_out=lds_out)
                    assert last
                except FellThrough as e:
                    assert not last
                    regs = e.regs
            assert sorted(lds_out) == list(range(c0, min(c0 + 8, n_prog)))
            for lane in range(64):
                q = wave * G + lane // Rp
                if q >= P:
                    continue
                for j, vals in lds_out.items():
                    want = orc.eval_tree(pop[order[q], j], lib.fn_codes, lib.n_funcs, lib.var_start, data[:, lane])
                    got = vals[lane]
                    assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32) or \
                        (np.isnan(got) and np.isnan(want)), (wave, lane, j, got, want)


# ---- the exp / log / tanh / sqrt subroutines (round 4), instruction by instruction -------------
class _Tmpl:
    """Float32 / uint32 lane emulator of the straight-line subroutine templates (every gfx950
    instruction they use).  IEEE basic operations are numpy float32 (correctly rounded); fma via
    float64 (exact product, one rounding); the v_div_scale .. v_div_fixup sequence is the IEEE
    division (its temporaries are poisoned with NaN, so a template that read one after the
    sequence would fail); v_sqrt_f32 is the correctly rounded root moved by a random -1 / 0 / +1
    ulp (the hardware's approximation is within one ulp: the template's correction must undo it)."""

    def __init__(self, x, seed=0):
        self.n = x.size
        self.v = {17: x.astype(np.float32).view(np.uint32).copy()}
        self.s = {}
        self.rng = np.random.default_rng(seed)

    def f(self, o):
        return self.u(o, float_ctx=True).view(np.float32)

    def u(self, o, float_ctx=False):
        o = o.strip()
        neg = absm = False
        if o.startswith("-") and o[1:2] in ("v", "|", "s"):
            neg, o = True, o[1:]
        if o.startswith("|"):
            absm, o = True, o.strip("|")
        if o.startswith("v") and o[1:].isdigit():
            r = self.v[int(o[1:])].copy()
        elif o.startswith("s") and o[1:].isdigit():
            r = np.full(self.n, self.s[int(o[1:])], np.uint32)
        elif o.startswith("0x"):
            r = np.full(self.n, int(o, 16), np.uint32)
        elif "." in o:
            r = np.full(self.n, np.float32(float(o)).view(np.uint32), np.uint32)
        else:  # integer inline constant (-16 .. 64): in a float operation the integer's value as a float
            k = int(o)
            r = np.full(self.n, (np.float32(k).view(np.uint32) if float_ctx else np.uint32(k & 0xFFFFFFFF)), np.uint32)
        if absm:
            r = r & np.uint32(0x7FFFFFFF)
        if neg:
            r = r ^ np.uint32(0x80000000)
        return r

    def mask(self, o):
        o = o.strip()
        return self.vcc if o == "vcc" else self.s_mask[o]

    def setf(self, d, val):
        self.v[int(d[1:])] = np.asarray(val, np.float32).view(np.uint32).copy()

    def setu(self, d, val):
        self.v[int(d[1:])] = np.asarray(val).astype(np.uint32)

    @staticmethod
    def _class(x, bits):
        u = x.view(np.uint32)
        neg = (u >> 31) == 1
        e, m = (u >> 23) & 0xFF, u & 0x7FFFFF
        cls = np.select([(e == 255) & (m != 0) & ((m >> 22) == 0), (e == 255) & (m != 0), (e == 255) & neg,
                         (e == 0) & (m == 0) & neg, (e == 0) & neg, neg,
                         (e == 255), (e == 0) & (m == 0), (e == 0)],
                        [0, 1, 2, 5, 4, 3, 9, 6, 7], 8)
        return ((bits >> cls.astype(np.uint32)) & 1) == 1

    def run(self, text):
        """-> (v8, whether the out-of-line slow path ran)"""
        f32, f64 = np.float32, np.float64
        self.vcc = np.zeros(self.n, bool)
        self.s_mask = {}
        in_div = []
        lines = [ln.strip() for ln in text.strip().splitlines()]
        labels = {ln[:-1]: k for k, ln in enumerate(lines) if ln.endswith(":")}
        pc, slow = 0, False
        while pc < len(lines):
            ln = lines[pc]
            pc += 1
            if ln.endswith(":"):
                continue
            op, _, rest = ln.partition(" ")
            a = [t.strip() for t in rest.split(",")] if rest else []
            if op == "s_cbranch_vccnz":
                if self.vcc.any():
                    pc, slow = labels[a[0]], True
                continue
            if op == "s_and_b64" and a == ["vcc", "exec", "vcc"]:
                continue  # (exec: all lanes)
            with np.errstate(all="ignore"):
                if op in ("v_div_scale_f32",) or (in_div and op != "v_div_fixup_f32"):
                    in_div.append(a[0])
                    if op == "v_div_scale_f32" and a[1] == "vcc":
                        self.vcc = np.zeros(self.n, bool)
                    continue
                if op == "v_div_fixup_f32":  # = IEEE n / d, temporaries poisoned
                    for r in in_div:
                        self.setf(r, np.full(self.n, np.nan, f32))
                    in_div = []
                    self.setf(a[0], self.f(a[3]) / self.f(a[2]))
                elif op == "v_mul_f32":
                    self.setf(a[0], self.f(a[1]) * self.f(a[2]))
                elif op in ("v_add_f32", "v_add_f32_e64"):
                    self.setf(a[0], self.f(a[1]) + self.f(a[2]))
                elif op == "v_sub_f32":
                    self.setf(a[0], self.f(a[1]) - self.f(a[2]))
                elif op == "v_rndne_f32":
                    self.setf(a[0], np.rint(self.f(a[1])))
                elif op in ("v_fma_f32", "v_fmamk_f32", "v_fmaak_f32"):
                    self.setf(a[0], (self.f(a[1]).astype(f64) * self.f(a[2]).astype(f64) +
                                     self.f(a[3]).astype(f64)).astype(f32))
                elif op == "v_fmac_f32":
                    self.setf(a[0], (self.f(a[1]).astype(f64) * self.f(a[2]).astype(f64) +
                                     self.f(a[0]).astype(f64)).astype(f32))
                elif op == "v_mov_b32":
                    self.setu(a[0], self.u(a[1]))
                elif op == "v_cvt_i32_f32":  # saturating, NaN -> 0
                    t = self.f(a[1]).astype(f64)
                    t = np.where(np.isnan(t), 0, np.clip(np.trunc(t), -2.0 ** 31, 2.0 ** 31 - 1))
                    self.setu(a[0], t.astype(np.int64).astype(np.int32).view(np.uint32))
                elif op == "v_cvt_f32_i32":
                    self.setf(a[0], self.u(a[1]).view(np.int32).astype(f32))
                elif op == "v_lshrrev_b32":
                    self.setu(a[0], self.u(a[2]) >> (self.u(a[1]) & 31))
                elif op == "v_ashrrev_i32":
                    self.setu(a[0], (self.u(a[2]).view(np.int32) >> (self.u(a[1]) & 31).astype(np.int32)).view(np.uint32))
                elif op == "v_add_u32":
                    self.setu(a[0], self.u(a[1]).astype(np.uint64) + self.u(a[2]))
                elif op == "v_subrev_u32":
                    self.setu(a[0], self.u(a[2]).astype(np.int64) - self.u(a[1]).astype(np.int64))
                elif op == "v_rcp_f32":  # within one ulp of 1/x: a random -1 / 0 / +1 ulp move of the rounded value
                    x = self.f(a[1])
                    r = (np.float64(1.0) / x.astype(f64)).astype(f32)
                    step = self.rng.integers(-1, 2, self.n).astype(np.int64)
                    ok = np.isfinite(r) & (r != 0) & (np.abs(r) < f32(3e38))
                    self.setu(a[0], np.where(ok, (r.view(np.uint32).astype(np.int64) + step).astype(np.uint32),
                                             r.view(np.uint32)))
                elif op == "v_sub_u32":
                    self.setu(a[0], self.u(a[1]).astype(np.int64) - self.u(a[2]).astype(np.int64))
                elif op == "v_lshl_add_u32":
                    self.setu(a[0], ((self.u(a[1]).astype(np.uint64) << (self.u(a[2]).astype(np.uint64) & 31))
                                     + self.u(a[3])) & 0xFFFFFFFF)
                elif op == "v_and_b32":
                    self.setu(a[0], self.u(a[1]) & self.u(a[2]))
                elif op == "v_or_b32":
                    self.setu(a[0], self.u(a[1]) | self.u(a[2]))
                elif op == "v_xor_b32":
                    self.setu(a[0], self.u(a[1]) ^ self.u(a[2]))
                elif op.startswith("v_cmp_"):
                    kind = op[6:].replace("_e64", "").replace("_e32", "")
                    dst = a[0]
                    if kind == "class_f32":
                        m = self._class(self.f(a[1]), self.u(a[2]))
                    elif kind.endswith("_u32"):
                        x, y = self.u(a[1]), self.u(a[2])
                        m = {"gt_u32": x > y, "le_u32": x <= y}[kind]
                    else:
                        x, y = self.f(a[1]), self.f(a[2])
                        m = {"lt_f32": x < y, "gt_f32": x > y, "ge_f32": x >= y, "nge_f32": ~(x >= y),
                             "u_f32": np.isnan(x) | np.isnan(y)}[kind]
                    if dst == "vcc":
                        self.vcc = m
                    else:
                        self.s_mask[dst] = m
                elif op in ("v_cndmask_b32", "v_cndmask_b32_e64"):
                    m = self.mask(a[3]) if len(a) > 3 else self.vcc
                    self.setu(a[0], np.where(m, self.u(a[2]), self.u(a[1])))
                elif op == "v_sqrt_f32":
                    x = self.f(a[1])
                    r = np.sqrt(x.astype(f64)).astype(f32)
                    step = self.rng.integers(-1, 2, self.n).astype(np.int64)
                    moved = (r.view(np.uint32).astype(np.int64) + step).astype(np.uint32)
                    ok = np.isfinite(r) & (r > 0) & (r.view(np.uint32) < 0x7F7FFFFF)
                    self.setu(a[0], np.where(ok, moved, r.view(np.uint32)))
                elif op == "s_mov_b32":
                    self.s[int(a[0][1:])] = self.u(a[1])[0]
                elif op == "s_setpc_b64":
                    return self.v[8].view(np.float32), slow
                elif op != "s_nop":
                    raise AssertionError(ln)
        raise AssertionError("no s_setpc")


def _gen_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_jit_templates", os.path.join(ROOT, "scripts",
                                                                                     "gen_jit_templates.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def _edge_inputs(rng):
    f32 = np.float32
    special = [np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 1e-40, -1e-40, 1.1754942e-38, 1.17549435e-38,
               2.3509886e-38, 1e-30, 1e-7, 0.5, 0.625, -0.625, 0.62499994, 0.62500006, 1.0, -1.0, 2.0, 44.361416,
               44.36142, 88.7228394, 88.72284, 88.72283, -103.972084, -103.97209, -87.33655, -88.0, 3.4e38, -3.4e38,
               1e10, -1e10, 2.0 ** 24, 0.70710677, 1.4142135, 1.4142137]
    parts = [np.array(special, f32), rng.uniform(-120, 100, 60000).astype(f32),
             rng.uniform(-3, 3, 60000).astype(f32), (np.exp(rng.uniform(-100, 88, 60000))).astype(f32),
             np.exp(rng.uniform(-103, 0, 20000)).astype(f32) * rng.choice([-1, 1], 20000).astype(f32),
             rng.integers(0, 2 ** 32, 60000, dtype=np.uint64).astype(np.uint32).view(f32)]
    x = np.concatenate(parts)
    with np.errstate(invalid="ignore"):
        return np.concatenate([x, np.nextafter(x, np.float32(np.inf)), np.nextafter(x, np.float32(-np.inf))])


# the hot range of subroutines with an out-of-line slow path (lanes that never take it); none since
# the straight-line versions measured faster (the machinery stays for a future branchy template)
HOT = {}


@pytest.mark.parametrize("name", ["EXP", "LOG", "TANH", "SQRT"])
def test_unary_templates_emulate_to_spec(name):
    """The exp / log / tanh / sqrt subroutines equal the include/mtgp_f32math.h specs (the oracle)
    bit for bit on every lane: NaN, infinities, signed zeros, subnormals, the range limits and
    branch points and their neighbours, random bit patterns."""
    g = _gen_module()
    x = _edge_inputs(np.random.default_rng(7))
    batches = [(x, name in HOT)]
    if name in HOT:
        batches.append((x[HOT[name](x)], False))
    for batch, want_slow in batches:
        got, slow = _Tmpl(batch, seed=1).run(g.TEMPLATES[name])
        ref = orc.unary(FN[name], batch)
        same = got.view(np.uint32) == ref.view(np.uint32)
        assert same.all(), (name, want_slow, batch[~same][:6], got[~same][:6], ref[~same][:6])
        assert slow == want_slow, (name, want_slow)
    if name in HOT:
        for i in np.nonzero(~HOT[name](x))[0][:50]:  # one outside lane is enough
            assert _Tmpl(np.array([1.25, x[i]], np.float32)).run(g.TEMPLATES[name])[1], (name, x[i])


def test_unary_subroutines_abi_clean():
    """Straight-line (a branchy template: one s_cbranch_vccnz to its slow path, which has its own
    return and no branch).  Nothing writes exec; only
    v8 / v18-v24, s[34:35], s38 and vcc are written (v17, the argument, is read to the end: the
    special-case selects need it)."""
    for name in ("EXP", "LOG", "TANH", "SQRT"):
        w = BLOBS[name]
        ret = w.index(SETPC_S40)
        hot, cold = _disassemble(w[:ret + 1]), _disassemble(w[ret + 1:]) if ret + 1 < len(w) else []
        assert hot[-1] == "s_setpc_b64 s[40:41]", name
        branches = [ln.split()[0] for ln in hot if ln.startswith(("s_cbranch", "s_branch"))]
        if name in HOT:
            assert branches == ["s_cbranch_vccnz"] and cold[-1] == "s_setpc_b64 s[40:41]", name
        else:
            assert branches == [] and cold == [], name
        assert not any(ln.startswith(("s_cbranch", "s_branch")) for ln in cold), name
        for ln in hot[:-1] + cold[:-1]:
            op, _, rest = ln.partition(" ")
            assert "exec" not in ln or ln == "s_and_b64 vcc, exec, vcc", (name, ln)
            if op.startswith(("s_nop", "s_cbranch")) or ln == "s_and_b64 vcc, exec, vcc":
                continue
            dst = rest.split(",")[0].strip()
            if op.startswith("v_cmp") and op.endswith("_e32"):
                assert dst == "vcc", ln
                continue
            m = re.fullmatch(r"v(\d+)", dst)
            if m:
                assert int(m.group(1)) in {8} | set(range(18, 25)), (name, ln)
                if op.startswith("v_div_scale"):
                    assert rest.split(",")[1].strip() in ("vcc", "s[34:35]"), ln
                continue
            assert dst in ("vcc", "s[34:35]", "s38"), (name, ln)
    assert _disassemble(BLOBS["ABS"]) == ["v_and_b32_e32 v8, 0x7fffffff, v8"]


def test_subroutine_cost_counts_match_blobs():
    """The schedule's per-call cost (mtgp_jit.h kJit*Exec = WORDS - SKIPPABLE_WORDS) counts exactly
    the words up to each subroutine's return: sin / cos keep their Payne-Hanek reduction after the
    return (skippable), exp / log / tanh / sqrt are branch-free (no s_cbranch; 0 skippable)."""
    text = open(os.path.join(ROOT, "multitreegp_amd", "csrc", "mtgp_jit_blobs.h")).read()
    for name in ("SIN", "COS", "EXP", "LOG", "TANH", "SQRT"):
        words = int(re.search(rf"#define MTGP_JIT_{name}_WORDS (\d+)", text).group(1))
        skip = int(re.search(rf"#define MTGP_JIT_{name}_SKIPPABLE_WORDS (\d+)", text).group(1))
        blob = re.search(rf"mtgp_jit_{name.lower()}_blob\[\d+\] = \{{(.*?)\}};", text).group(1)
        ws = [int(w.strip().rstrip("u"), 16) for w in blob.split(",")]
        assert len(ws) == words
        ret = ws.index(0xBE801D28)  # s_setpc_b64 s[40:41]
        assert skip == words - ret - 1
        listing = text[text.index(f"// {name}:"):text.index(f"#define MTGP_JIT_{name}_WORDS")]
        if name in ("SIN", "COS"):
            assert skip > 100 and "s_cbranch" in listing
        else:
            assert skip == 0 and "s_cbranch" not in listing
