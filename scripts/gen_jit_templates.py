#!/usr/bin/env python3
"""Assemble the fixed machine-code templates of the program JIT (gfx950) into
multitreegp_amd/csrc/mtgp_jit_blobs.h.

The JIT (csrc/mtgp_jit.h) translates each flattened program into straight-line gfx950 code;
simple operations are encoded directly (VOP1/VOP2 words), while sin, cos, exp, log, tanh, sqrt,
abs and the IEEE fp32 division come from the templates below.  Register ABI of the generated code
(csrc/mtgp_jit.h): v0-v7 data slots (read only), v8 accumulator, v9-v16 operand stack,
v17-v24 template temporaries, s[30:31] return address, s[32:33] fallback lane mask
(OR-accumulated), s[34:39] template temporaries, vcc clobbered, exec never written.

  SIN / COS  : subroutines (one shared copy at the start of the code buffer, called with
               s_swappc_b64 s[40:41], returning with s_setpc_b64 s[40:41]): x in v17 -> v8.
               include/mtgp_f32math.h mtgp_trig_pi (spec v2: reduction onto the pi grid, one
               odd polynomial, sign from bit 0 of k + odd) op for op: the float Cody-Waite hot
               path (|x| < 2^17) straight-line; finite |x| >= 2^17 lanes take a branch (not
               taken in the common case) to out-of-line exec-masked blocks -- the spec's double
               Cody-Waite below 2^28, its Payne-Hanek reduction beyond -- and come back.  exec
               is restored; s[32:33] is never set (the evaluator's fallback stays for safety).
  EXP / LOG /: subroutines like SIN / COS (x in v17 -> v8), straight-line: include/mtgp_f32math.h
  TANH / SQRT  mtgp_expf / mtgp_logf / mtgp_tanhf op for op on every lane, their special cases
               (NaN, infinities, zeros, range limits) by selects at the end; sqrt is the
               compiler's correctly rounded gfx950 sequence (= HIP's sqrtf, the spec's).  Temps
               v18-v24 and v8; v17 (x) is kept until the final selects.
  DIV        : v17 / v18 -> v8, the compiler's own IEEE-exact sequence for gfx950
               (v_div_scale / v_rcp / fma refinement / v_div_fmas / v_div_fixup).
  ABS        : v8 = |v8| inline (v_and_b32 with 0x7fffffff).
Hazards: VALU-written SGPR/VCC read by a VALU mask operand gets `s_nop 1` in between; the
division keeps the compiler's instruction order (v_div_fmas >= 4 wait states after VCC); the
local branch of the sin/cos double block is a relative SOPP offset resolved by llvm-mc.
Run with --check to verify the committed header is current (tests/test_jit.py)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "multitreegp_amd", "csrc", "mtgp_jit_blobs.h")
LLVM_MC = os.environ.get("LLVM_MC", "/opt/rocm/lib/llvm/bin/llvm-mc")

# Payne-Hanek window selection and 96-bit product for finite |x| >= 2^28 (|x| in v24): leaves
# hi_lo32 in v18, mid_lo32 in v22, lo_lo32 in v20 (include/mtgp_f32math.h
# mtgp_reduce_payne_hanek_pi: b = e - 2, k = b >> 5, s = b & 31, W = 2/pi bits [b+1, b+96])
_PH_PRODUCT = """
v_lshrrev_b32 v18, 23, v24
v_add_u32 v18, 0xffffff68, v18
v_lshrrev_b32 v19, 5, v18
v_and_b32 v18, 31, v18
v_sub_u32 v18, 32, v18
v_mov_b32 v23, 0xf534ddc0
v_mov_b32 v22, 0xdb629599
v_mov_b32 v21, 0x3c439041
v_mov_b32 v20, 0xfe5163ab
v_cmp_ne_u32_e32 vcc, 2, v19
s_nop 1
v_mov_b32 v8, 0xfc2757d1
v_cndmask_b32_e32 v23, v8, v23, vcc
v_mov_b32 v8, 0xf534ddc0
v_cndmask_b32_e32 v22, v8, v22, vcc
v_mov_b32 v8, 0xdb629599
v_cndmask_b32_e32 v21, v8, v21, vcc
v_mov_b32 v8, 0x3c439041
v_cndmask_b32_e32 v20, v8, v20, vcc
v_cmp_ne_u32_e32 vcc, 1, v19
s_nop 1
v_mov_b32 v8, 0x4e441529
v_cndmask_b32_e32 v23, v8, v23, vcc
v_mov_b32 v8, 0xfc2757d1
v_cndmask_b32_e32 v22, v8, v22, vcc
v_mov_b32 v8, 0xf534ddc0
v_cndmask_b32_e32 v21, v8, v21, vcc
v_mov_b32 v8, 0xdb629599
v_cndmask_b32_e32 v20, v8, v20, vcc
v_cmp_ne_u32_e32 vcc, 0, v19
s_nop 1
v_mov_b32 v8, 0xa2f9836e
v_cndmask_b32_e32 v23, v8, v23, vcc
v_mov_b32 v8, 0x4e441529
v_cndmask_b32_e32 v22, v8, v22, vcc
v_mov_b32 v8, 0xfc2757d1
v_cndmask_b32_e32 v21, v8, v21, vcc
v_mov_b32 v8, 0xf534ddc0
v_cndmask_b32_e32 v20, v8, v20, vcc
v_and_b32 v8, 0x7fffff, v24
v_or_b32 v8, 0x800000, v8
v_cmp_eq_u32_e32 vcc, 32, v18
v_alignbit_b32 v19, v23, v22, v18
s_nop 1
v_cndmask_b32_e32 v19, v19, v23, vcc
v_alignbit_b32 v23, v22, v21, v18
v_cndmask_b32_e32 v23, v23, v22, vcc
v_alignbit_b32 v22, v21, v20, v18
v_cndmask_b32_e32 v22, v22, v21, vcc
v_mad_u64_u32 v[20:21], s[34:35], v8, v22, 0
v_mov_b32 v18, v23
v_mov_b32 v22, v21
v_mov_b32 v23, 0
v_mad_u64_u32 v[22:23], s[34:35], v8, v18, v[22:23]
v_mov_b32 v21, v19
v_mov_b32 v18, v23
v_mov_b32 v19, 0
v_mad_u64_u32 v[18:19], s[34:35], v8, v21, v[18:19]
"""


def _trig(odd):
    """sin (odd = 0) / cos (odd = 1) of include/mtgp_f32math.h mtgp_trig_pi (spec v2) op for op.
    Hot path (|x| < 2^17): t = x * f32(1/pi); k = rint(t [- 0.5]); j = 2k [+ 1]; r = x - j pi/2
    by the 3-constant fma Cody-Waite; sin_poly(r), sign bit = bit 0 of (k + odd); |x| < 2^-12
    override (mask kept in s[44:45]).  Finite |x| >= 2^17 lanes branch (not taken in the common
    case) to out-of-line blocks after the return: the spec's double Cody-Waite for |x| < 2^28
    and its Payne-Hanek reduction beyond, each under its own exec mask, then back to the
    polynomial.  v23 carries the sign source (k + odd, or (j + odd) >> 1 on the Payne-Hanek
    path); NaN / +-inf give NaN on the hot path.  s[32:33] is never set."""
    t = """
v_and_b32 v24, 0x7fffffff, v17
s_mov_b32 s38, 0x39800000
v_cmp_gt_f32_e64 s[44:45], s38, v24
v_mul_f32 v18, 0x3ea2f983, v17
"""
    if odd:
        t += """v_add_f32 v18, -0.5, v18
v_rndne_f32 v18, v18
v_cvt_i32_f32 v23, v18
v_fma_f32 v18, v18, 2.0, 1.0
v_add_u32 v23, 1, v23
"""
    else:
        t += """v_rndne_f32 v18, v18
v_cvt_i32_f32 v23, v18
v_add_f32 v18, v18, v18
"""
    t += """v_fmamk_f32 v19, v18, 0xbfc90fdb, v17
v_fmamk_f32 v19, v18, 0x333bbd2e, v19
v_fmamk_f32 v19, v18, 0x26f72ced, v19
v_subrev_u32 v20, 0x48000000, v24
v_cmp_gt_u32_e32 vcc, 0x37800000, v20
s_and_b64 vcc, exec, vcc
s_cbranch_vccnz .Lslow
.Lpoly:
v_lshlrev_b32 v23, 31, v23
v_mul_f32 v20, v19, v19
v_mov_b32 v21, {C9}
v_fmaak_f32 v21, v21, v20, {C7}
v_fmaak_f32 v21, v21, v20, {C5}
v_fmaak_f32 v21, v21, v20, {C3}
v_mul_f32 v22, v19, v20
v_fma_f32 v21, v22, v21, v19
v_xor_b32 v21, v21, v23
"""
    t += ("v_cndmask_b32_e64 v8, v21, 1.0, s[44:45]\n" if odd else "v_cndmask_b32_e64 v8, v21, v17, s[44:45]\n")
    t += "s_setpc_b64 s[40:41]\n"
    # ---- out of line: finite |x| >= 2^17 (vcc = those lanes)
    t += """.Lslow:
s_mov_b64 s[34:35], vcc
v_cmp_gt_u32_e32 vcc, 0x5800000, v20
s_and_b64 vcc, vcc, s[34:35]
s_and_saveexec_b64 s[36:37], vcc
s_cbranch_execz .Lph
v_cvt_f64_f32 v[20:21], v17
s_mov_b32 s38, 0x6dc9c883
s_mov_b32 s39, 0x3fd45f30
v_mul_f64 v[18:19], v[20:21], s[38:39]
""" + ("v_add_f64 v[18:19], v[18:19], -0.5\n" if odd else "") + """v_rndne_f64 v[18:19], v[18:19]
v_cvt_i32_f64 v8, v[18:19]
""" + ("v_fma_f64 v[18:19], v[18:19], 2.0, 1.0\nv_add_u32 v8, 1, v8\n" if odd else
       "v_add_f64 v[18:19], v[18:19], v[18:19]\n") + """s_mov_b32 s38, 0x40000000
s_mov_b32 s39, 0x3ff921fb
v_mul_f64 v[22:23], v[18:19], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[22:23]
s_mov_b32 s38, 0
s_mov_b32 s39, 0x3e74442d
v_mul_f64 v[22:23], v[18:19], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[22:23]
s_mov_b32 s38, 0x98cc5170
s_mov_b32 s39, 0x3cf84698
v_mul_f64 v[22:23], v[18:19], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[22:23]
v_cvt_f32_f64 v19, v[20:21]
v_mov_b32 v23, v8
.Lph:
s_mov_b64 exec, s[36:37]
v_subrev_u32 v20, 0x4d800000, v24
v_cmp_gt_u32_e32 vcc, 0x32000000, v20
s_and_saveexec_b64 s[36:37], vcc
s_cbranch_execz .Ldone
""" + _PH_PRODUCT + """v_lshrrev_b32 v21, 30, v18
v_and_b32 v23, 0x3fffffff, v18
v_lshlrev_b32 v23, 2, v23
v_lshrrev_b32 v8, 30, v22
v_or_b32 v23, v23, v8
v_lshrrev_b32 v20, 30, v20
v_lshlrev_b32 v22, 2, v22
v_or_b32 v22, v22, v20
v_cvt_f64_u32 v[18:19], v23
v_ldexp_f64 v[18:19], v[18:19], 32
v_cvt_f64_u32 v[22:23], v22
v_add_f64 v[18:19], v[18:19], v[22:23]
s_mov_b32 s38, 0
s_mov_b32 s39, 0x3bf00000
v_mul_f64 v[18:19], v[18:19], s[38:39]
v_and_b32 v20, 1, v21
""" + ("v_xor_b32 v20, 1, v20\n" if odd else "") + """v_add_u32 v21, v21, v20
v_cmp_ne_u32_e32 vcc, 0, v20
v_add_f64 v[22:23], v[18:19], -1.0
s_nop 1
v_cndmask_b32_e32 v18, v18, v22, vcc
v_cndmask_b32_e32 v19, v19, v23, vcc
s_mov_b32 s38, 0x54442d18
s_mov_b32 s39, 0x3ff921fb
v_mul_f64 v[18:19], v[18:19], s[38:39]
v_cvt_f32_f64 v19, v[18:19]
v_cmp_gt_f32_e32 vcc, 0, v17
v_xor_b32 v20, 0x80000000, v19
v_sub_u32 v22, 4, v21
s_nop 1
v_cndmask_b32_e32 v19, v19, v20, vcc
v_cndmask_b32_e32 v21, v21, v22, vcc
""" + ("v_add_u32 v21, 1, v21\n" if odd else "") + """v_lshrrev_b32 v23, 1, v21
.Ldone:
s_mov_b64 exec, s[36:37]
s_branch .Lpoly
"""
    return t.format(**_sin_coefficients())


def _sin_coefficients():
    """the polynomial's f32 coefficients, read from the spec header (one source of truth)"""
    import struct
    text = open(os.path.join(ROOT, "include", "mtgp_f32math.h")).read()
    out = {}
    for name in ("C3", "C5", "C7", "C9"):
        m = re.search(r"#define MTGP_SIN_%s ([-+0-9.eE]+)f" % name, text)
        out[name] = "0x%08x" % struct.unpack("<I", struct.pack("<f", float(m.group(1))))[0]
    return out


def _f32(v):
    """the f32 bit pattern of a decimal constant (rounded as the C compiler rounds `v f`)"""
    import struct
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", float(v)))[0]


def _spec_consts(fn, count):
    """the float literals of one spec function of include/mtgp_f32math.h, in source order"""
    text = open(os.path.join(ROOT, "include", "mtgp_f32math.h")).read()
    a = text.index("MTGP_INLINE MTGP_HD float %s(" % fn)
    b = text.index("\n}\n", a)
    vals = re.findall(r"(?<![\w.])(-?[0-9]+\.[0-9]+(?:e[-+]?[0-9]+)?)f", text[a:b])
    assert len(vals) == count, (fn, vals)
    return vals


def _exp_body(x, out, tmp_inf, select=True):
    """mtgp_expf of v{x} into v{out} op for op (fma Cody-Waite, degree-6 polynomial, two
    power-of-two scalings; n1 = ni / 2 truncated), then (select) x > 88.7228394 -> +inf.  Temps
    v18-v21 (and v{tmp_inf}); v{x} is kept.  (The x < -103.972084 -> 0 and NaN cases are the
    caller's.)  Returns (code, the lower limit's literal)."""
    v = _spec_consts("mtgp_expf", 13)
    lim_hi, lim_lo, zero, log2e, ln2hi, ln2lo, c6, c5, c4, c3, c2, c1, one = v
    assert _f32(c1) == _f32(0.5) and _f32(zero) == _f32(0.0) and _f32(one) == _f32(1.0), v  # inline constants
    code = f"""v_mul_f32 v18, {_f32(log2e)}, v{x}
v_rndne_f32 v18, v18
v_fmamk_f32 v19, v18, {_f32(-float(ln2hi))}, v{x}
v_fmamk_f32 v19, v18, {_f32(-float(ln2lo))}, v19
v_mov_b32 v20, {_f32(c5)}
v_fmac_f32 v20, {_f32(c6)}, v19
v_fmaak_f32 v20, v20, v19, {_f32(c4)}
v_fmaak_f32 v20, v20, v19, {_f32(c3)}
v_fmaak_f32 v20, v20, v19, {_f32(c2)}
v_fma_f32 v20, v20, v19, 0.5
v_mul_f32 v21, v19, v19
v_fmac_f32 v19, v20, v21
v_add_f32 v19, 1.0, v19
v_cvt_i32_f32 v18, v18
v_lshrrev_b32 v20, 31, v18
v_add_u32 v20, v18, v20
v_ashrrev_i32 v20, 1, v20
v_sub_u32 v18, v18, v20
v_lshl_add_u32 v20, v20, 23, 1.0
v_mul_f32 v19, v19, v20
v_lshl_add_u32 v18, v18, 23, 1.0
v_mul_f32 v{out}, v19, v18
"""
    if select:
        code += f"""v_cmp_lt_f32 vcc, {_f32(lim_hi)}, v{x}
v_mov_b32 v{tmp_inf}, 0x7f800000
s_nop 1
v_cndmask_b32 v{out}, v{out}, v{tmp_inf}, vcc
"""
    return code, lim_lo


# The subroutines are straight-line: every lane runs the spec's main path and the special cases
# are selects at the end.  (Hot paths with an out-of-line slow path for the special ranges
# measured slower at C3 -- 2.48-2.50 vs 2.37 ms with the extended library, profiles/r04/v8, v9:
# negative log / sqrt arguments, |x| >= 0.625 for tanh and the inf / NaN states of diverged
# rollouts occur in some lane of most waves, and a unit's other groups' lanes run every program
# too, so the branch was usually taken and only added work.)
_RET = "s_setpc_b64 s[40:41]\n"


def _div_body(q, n, d, t):
    """the IEEE division n / d into v{q}, the compiler's own gfx950 sequence (as DIV), temps
    v{t[0..4]}; n may be an inline constant"""
    a, r, s_, e, f = t
    return f"""v_div_scale_f32 v{a}, s[34:35], v{d}, v{d}, {n}
v_rcp_f32 v{r}, v{a}
v_div_scale_f32 v{s_}, vcc, {n}, v{d}, {n}
v_fma_f32 v{e}, -v{a}, v{r}, 1.0
v_fmac_f32 v{r}, v{e}, v{r}
v_mul_f32 v{e}, v{s_}, v{r}
v_fma_f32 v{f}, -v{a}, v{e}, v{s_}
v_fmac_f32 v{e}, v{f}, v{r}
v_fma_f32 v{a}, -v{a}, v{e}, v{s_}
v_div_fmas_f32 v{a}, v{a}, v{r}, v{e}
v_div_fixup_f32 v{q}, v{a}, v{d}, {n}
"""


def _exp():
    """EXP subroutine: mtgp_expf(v17) -> v8, straight-line on every lane: the spec's hot path, then
    NaN -> x, x > 88.72 -> +inf, x < -103.97 -> +0 by selects.  (An out-of-line slow path for
    |x| > 88.72 or NaN measured slower: diverged rollouts carry inf / NaN states, so some lane of
    most waves needs it.)"""
    full, lim_lo = _exp_body(17, 8, 18)
    return full + f"""v_cmp_gt_f32 vcc, {_f32(lim_lo)}, v17
s_nop 1
v_cndmask_b32_e64 v8, v8, 0, vcc
v_cmp_u_f32 vcc, v17, v17
s_nop 1
v_cndmask_b32 v8, v8, v17, vcc
""" + _RET


def _log():
    """LOG subroutine: mtgp_logf(v17) -> v8: mtgp_logf_pos op for op on every lane (subnormal
    scaling by a select, s = f / (2 + f) by the IEEE division), then the special cases by
    class selects: -inf/-normal/-subnormal -> NaN, +-0 -> -inf, NaN/+inf -> x."""
    v = _spec_consts("mtgp_logf_pos", 10)
    scale, m1, two, c3, c4, c5, c6, half, ln2hi, ln2lo = v
    assert _f32(scale) == "0x4c000000" and _f32(m1) == _f32(1.0) and _f32(two) == _f32(2.0), v
    assert _f32(half) == _f32(0.5), v
    return _log_text(scale, c3, c4, c5, c6, ln2hi, ln2lo)


def _log_text(scale, c3, c4, c5, c6, ln2hi, ln2lo):
    """Straight-line on every lane.  s = f / (2 + f) by the division's fast path -- rcp,
    one Newton step, two fma corrections: the compiler's IEEE sequence with v_div_scale and
    v_div_fixup identities, as they are on EVERY lane, special ones included: m is built with a
    fixed exponent, so f = m - 1 is +0 or in [2^-24, 0.42] in magnitude and 2 + f in [1.7, 2.42]
    (the scale flag could only be set by the zero numerator, whose quotient is +0 either way)."""
    def tail(dst):
        return f"""v_mul_f32 v22, v21, v21
v_mul_f32 v23, v22, v22
v_mul_f32 v24, {_f32(c4)}, v23
v_add_f32 v24, {_f32(c3)}, v24
v_mul_f32 v24, v23, v24
v_mul_f32 v23, {_f32(c6)}, v23
v_add_f32 v23, {_f32(c5)}, v23
v_mul_f32 v23, v22, v23
v_add_f32 v23, v23, v24
v_mul_f32 v22, 0.5, v18
v_mul_f32 v22, v22, v18
v_add_f32 v23, v22, v23
v_mul_f32 v23, v21, v23
v_cvt_f32_i32 v24, v19
v_mul_f32 v21, {_f32(ln2lo)}, v24
v_add_f32 v23, v23, v21
v_sub_f32 v23, v22, v23
v_sub_f32 v23, v23, v18
v_mul_f32 v24, {_f32(ln2hi)}, v24
v_sub_f32 v{dst}, v24, v23
"""
    mant = """v_and_b32 v18, 0x7fffff, v18
v_add_u32 v20, 0x4afb20, v18
v_and_b32 v20, 0x800000, v20
v_xor_b32 v21, 0x3f800000, v20
v_or_b32 v18, v18, v21
v_lshrrev_b32 v20, 23, v20
v_add_u32 v19, v19, v20
v_add_f32 v18, -1.0, v18
v_add_f32 v20, 2.0, v18
"""
    fast_div = """v_rcp_f32 v22, v20
s_nop 0
v_fma_f32 v24, -v20, v22, 1.0
v_fmac_f32 v22, v24, v22
v_mul_f32 v24, v18, v22
v_fma_f32 v8, -v20, v24, v18
v_fmac_f32 v24, v8, v22
v_fma_f32 v8, -v20, v24, v18
v_fma_f32 v21, v8, v22, v24
"""
    return f"""v_cmp_gt_u32 vcc, 0x800000, v17
v_mul_f32 v18, {_f32(scale)}, v17
v_mov_b32 v19, 0xffffff81
v_mov_b32 v20, 0xffffff68
v_cndmask_b32 v18, v17, v18, vcc
v_cndmask_b32 v19, v19, v20, vcc
v_lshrrev_b32 v20, 23, v18
v_add_u32 v19, v19, v20
""" + mant + fast_div + tail(23) + """v_mov_b32 v21, 0x1c
v_cmp_class_f32 vcc, v17, v21
v_mov_b32 v22, 0x7fc00000
s_nop 1
v_cndmask_b32 v23, v23, v22, vcc
v_mov_b32 v21, 0x60
v_cmp_class_f32 vcc, v17, v21
v_mov_b32 v22, 0xff800000
s_nop 1
v_cndmask_b32 v23, v23, v22, vcc
v_mov_b32 v21, 0x203
v_cmp_class_f32 vcc, v17, v21
s_nop 1
v_cndmask_b32 v8, v23, v17, vcc
""" + _RET


def _tanh():
    """TANH subroutine: mtgp_tanhf(v17) -> v8, straight-line on every lane: the odd polynomial
    x + x^3 P(x^2) (|x| < 0.625) into v23, then sign(x) (1 - 2 / (exp(2|x|) + 1)) with the EXP
    body (2|x| > 88.72 -> +inf) and the IEEE division; |x| >= 0.625 selects the second;
    NaN and +-0 -> x."""
    v = _spec_consts("mtgp_tanhf", 11)
    cut, one, two, one2, z1, z2, p0, p1, p2, p3, p4 = v
    assert _f32(one) == _f32(one2) == _f32(1.0) and _f32(two) == _f32(2.0) and _f32(z1) == _f32(z2) == _f32(0.0), v
    body, _ = _exp_body(24, 19, 18)
    return f"""v_mul_f32 v18, v17, v17
v_mov_b32 v19, {_f32(p1)}
v_fmac_f32 v19, {_f32(p0)}, v18
v_fmaak_f32 v19, v19, v18, {_f32(p2)}
v_fmaak_f32 v19, v19, v18, {_f32(p3)}
v_fmaak_f32 v19, v19, v18, {_f32(p4)}
v_mul_f32 v19, v19, v18
v_fma_f32 v23, v19, v17, v17
v_add_f32_e64 v24, |v17|, |v17|
""" + body + """v_add_f32 v19, 1.0, v19
""" + _div_body(18, "2.0", 19, (18, 20, 21, 22, 24)) + f"""v_sub_f32 v18, 1.0, v18
v_cmp_gt_f32 vcc, 0, v17
s_nop 1
v_cndmask_b32_e64 v18, v18, -v18, vcc
s_mov_b32 s38, {_f32(cut)}
v_cmp_ge_f32_e64 vcc, |v17|, s38
s_nop 1
v_cndmask_b32 v8, v23, v18, vcc
v_mov_b32 v18, 0x63
v_cmp_class_f32 vcc, v17, v18
s_nop 1
v_cndmask_b32 v8, v8, v17, vcc
""" + _RET


# SQRT subroutine: the compiler's correctly rounded f32 square root for gfx950 (HIP's default
# sqrtf = include/mtgp_f32math.h mtgp_sqrtf): scale x < 2^-96 by 2^32, v_sqrt_f32, one-ulp
# correction from the two fma residuals, rescale by 2^-16; +-0 / +inf (class 0x260) pass through.
_SQRT = """v_mul_f32 v18, 0x4f800000, v17
v_cmp_gt_f32 vcc, 0xf800000, v17
s_nop 1
v_cndmask_b32 v19, v17, v18, vcc
v_sqrt_f32 v18, v19
s_nop 0
v_add_u32 v20, -1, v18
v_add_u32 v21, 1, v18
v_fma_f32 v22, -v20, v18, v19
v_fma_f32 v23, -v21, v18, v19
v_cmp_ge_f32_e64 s[34:35], 0, v22
s_nop 1
v_cndmask_b32_e64 v18, v18, v20, s[34:35]
v_cmp_lt_f32_e64 s[34:35], 0, v23
s_nop 1
v_cndmask_b32_e64 v18, v18, v21, s[34:35]
v_mul_f32 v20, 0x37800000, v18
v_cndmask_b32 v18, v18, v20, vcc
v_mov_b32 v20, 0x260
v_cmp_class_f32 vcc, v19, v20
s_nop 1
v_cndmask_b32 v8, v18, v19, vcc
""" + _RET

TEMPLATES = {
    "SIN": _trig(0),
    "COS": _trig(1),
    "DIV": """
v_div_scale_f32 v19, s[34:35], v18, v18, v17
v_rcp_f32 v20, v19
v_div_scale_f32 v21, vcc, v17, v18, v17
v_fma_f32 v22, -v19, v20, 1.0
v_fmac_f32 v20, v22, v20
v_mul_f32 v22, v21, v20
v_fma_f32 v23, -v19, v22, v21
v_fmac_f32 v22, v23, v20
v_fma_f32 v19, -v19, v22, v21
v_div_fmas_f32 v19, v19, v20, v22
v_div_fixup_f32 v8, v19, v18, v17
""",
    "EXP": _exp(),
    "LOG": _log(),
    "TANH": _tanh(),
    "SQRT": _SQRT,
    "ABS": "v_and_b32 v8, 0x7fffffff, v8\n",
}



def assemble(text):
    """Machine words from an object file (branch fixups resolved by the assembler) plus the
    instruction listing from -show-encoding (for the header comments)."""
    import tempfile
    r = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"], input=text.encode(),
                       capture_output=True, check=True)
    lines, n_bytes = [], 0
    for ln in r.stdout.decode().splitlines():
        m = re.search(r"^\s*(.*?)\s*; encoding: \[(.*)\]", ln)
        if m:
            lines.append(m.group(1))
            n_bytes += len(m.group(2).split(","))
    with tempfile.TemporaryDirectory() as d:
        obj, raw = os.path.join(d, "t.o"), os.path.join(d, "t.bin")
        subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-filetype=obj", "-o", obj], input=text.encode(),
                       check=True)
        objcopy = os.path.join(os.path.dirname(LLVM_MC), "llvm-objcopy")
        subprocess.run([objcopy, "-O", "binary", "--only-section=.text", obj, raw], check=True)
        b = open(raw, "rb").read()
    assert len(b) == n_bytes and len(b) % 4 == 0, (len(b), n_bytes)
    words = [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]
    return words, lines


# The shared subroutines, laid out in this order at the start of every code buffer, each at a
# 64-byte boundary (padding: s_nop 0); the rest of TEMPLATES (DIV, ABS) are copied inline.
SUBROUTINES = ("SIN", "COS", "EXP", "LOG", "TANH", "SQRT")
_ALIGN = 64
_PAD = 0xBF800000  # s_nop 0


def generate():
    out = ["// GENERATED by scripts/gen_jit_templates.py -- do not edit.",
           "// gfx950 machine-code templates of the program JIT (register ABI: csrc/mtgp_jit.h).",
           "#ifndef MTGP_JIT_BLOBS_H", "#define MTGP_JIT_BLOBS_H", "#include <stdint.h>", ""]
    area, offs = [], {}
    for name, text in TEMPLATES.items():
        words, lines = assemble(text)
        out.append(f"// {name}:")
        out += [f"//   {ln}" for ln in lines]
        body = ", ".join(f"0x{w:08x}u" for w in words)
        out.append(f"#define MTGP_JIT_{name}_WORDS {len(words)}")
        # out-of-line words after the return (only run when some lane needs a slow reduction)
        ret = words.index(0xBE801D28) if 0xBE801D28 in words else len(words) - 1  # s_setpc_b64 s[40:41]
        skip = len(words) - ret - 1
        out.append(f"#define MTGP_JIT_{name}_SKIPPABLE_WORDS {skip}")
        out.append(f"static const uint32_t mtgp_jit_{name.lower()}_blob[{len(words)}] = {{{body}}};")
        out.append("")
        if name in SUBROUTINES:
            assert 0xBE801D28 in words, name  # a subroutine returns with s_setpc_b64 s[40:41]
            while len(area) * 4 % _ALIGN:
                area.append(_PAD)
            offs[name] = len(area) * 4
            area += words
    while len(area) * 4 % _ALIGN:
        area.append(_PAD)
    out.append("// The subroutine area at the start of every JIT code buffer (byte offsets of each entry).")
    for name in SUBROUTINES:
        out.append(f"#define MTGP_JIT_{name}_OFFSET {offs[name]}u")
    out.append(f"#define MTGP_JIT_SUB_WORDS {len(area)}")
    rows = [", ".join(f"0x{w:08x}u" for w in area[i:i + 8]) for i in range(0, len(area), 8)]
    out.append("static const uint32_t mtgp_jit_sub_blob[MTGP_JIT_SUB_WORDS] = {\n    " + ",\n    ".join(rows) + "};")
    out.append("")
    out.append("#endif")
    return "\n".join(out) + "\n"


def main():
    text = generate()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        sys.exit(0 if cur == text else 1)
    open(OUT, "w").write(text)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
