#!/usr/bin/env python3
"""Assemble the fixed machine-code templates of the program JIT (gfx950) into
multitreegp_amd/csrc/mtgp_jit_blobs.h.

The JIT (csrc/mtgp_jit.h) translates each flattened program into straight-line gfx950 code;
simple operations are encoded directly (VOP1/VOP2 words), while sin, cos and the IEEE fp32
division are copied from the templates below.  Register ABI of the generated code
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
  DIV        : v17 / v18 -> v8, the compiler's own IEEE-exact sequence for gfx950
               (v_div_scale / v_rcp / fma refinement / v_div_fmas / v_div_fixup).
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


def generate():
    out = ["// GENERATED by scripts/gen_jit_templates.py -- do not edit.",
           "// gfx950 machine-code templates of the program JIT (register ABI: csrc/mtgp_jit.h).",
           "#ifndef MTGP_JIT_BLOBS_H", "#define MTGP_JIT_BLOBS_H", "#include <stdint.h>", ""]
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
