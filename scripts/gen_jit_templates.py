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
               s_swappc_b64 s[40:41], returning with s_setpc_b64 s[40:41]): x in v17 -> v8.  include/mtgp_f32math.h mtgp_sinf/mtgp_cosf op for op: float
               Cody-Waite for |x| < 2^17; for finite |x| >= 2^28 the spec's Payne-Hanek
               reduction (96-bit window of 2/pi selected per lane, three 32x32->64 products,
               int64 -> double, times pi/2), for 2^17 <= |x| < 2^28 the spec's double
               Cody-Waite -- each behind an exec-masked block that is branched over when no
               lane needs it; both Taylor polynomials, quadrant selects, |x| < 2^-12 override.
               No lane needs the interpreter any more (s[32:33] is never set; the evaluator's
               fallback stays for safety).  exec is saved in s[36:37] around each block.
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

REDUCE = """
v_mul_f32 v18, 0x3f22f983, v17
v_rndne_f32 v18, v18
v_fmamk_f32 v19, v18, 0xbfc90fdb, v17
v_fmamk_f32 v19, v18, 0x333bbd2e, v19
v_fmamk_f32 v19, v18, 0x26f72ced, v19
v_cvt_i32_f32 v18, v18
v_and_b32 v24, 0x7fffffff, v17
s_mov_b32 s38, 0x4d800000
s_mov_b32 s39, 0x7f800000
v_cmp_le_f32_e64 s[34:35], s38, v24
v_cmp_gt_f32_e64 s[36:37], s39, v24
s_and_b64 s[34:35], s[34:35], s[36:37]
s_and_saveexec_b64 s[36:37], s[34:35]
s_cbranch_execz .Lnoph
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
v_lshrrev_b32 v21, 30, v18
v_and_b32 v23, 0x3fffffff, v18
v_lshlrev_b32 v23, 2, v23
v_lshrrev_b32 v8, 30, v22
v_or_b32 v23, v23, v8
v_lshrrev_b32 v20, 30, v20
v_lshlrev_b32 v22, 2, v22
v_or_b32 v22, v22, v20
v_lshrrev_b32 v8, 31, v23
v_add_u32 v21, v21, v8
v_cvt_f64_i32 v[18:19], v23
v_ldexp_f64 v[18:19], v[18:19], 32
v_cvt_f64_u32 v[22:23], v22
v_add_f64 v[18:19], v[18:19], v[22:23]
s_mov_b32 s38, 0
s_mov_b32 s39, 0x3bf00000
v_mul_f64 v[18:19], v[18:19], s[38:39]
s_mov_b32 s38, 0x54442d18
s_mov_b32 s39, 0x3ff921fb
v_mul_f64 v[18:19], v[18:19], s[38:39]
v_cvt_f32_f64 v19, v[18:19]
v_cmp_gt_f32_e32 vcc, 0, v17
v_xor_b32 v20, 0x80000000, v19
v_sub_u32 v22, 4, v21
s_nop 1
v_cndmask_b32_e32 v19, v19, v20, vcc
v_cndmask_b32_e32 v18, v21, v22, vcc
.Lnoph:
s_mov_b64 exec, s[36:37]
s_mov_b32 s38, 0x4d800000
s_mov_b32 s39, 0x48000000
v_cmp_le_f32_e64 s[34:35], s39, v24
v_cmp_gt_f32_e64 s[36:37], s38, v24
s_and_b64 s[34:35], s[34:35], s[36:37]
s_and_saveexec_b64 s[36:37], s[34:35]
s_cbranch_execz .Lfast
v_cvt_f64_f32 v[20:21], v17
s_mov_b32 s38, 0x6dc9c883
s_mov_b32 s39, 0x3fe45f30
v_mul_f64 v[22:23], v[20:21], s[38:39]
v_rndne_f64 v[22:23], v[22:23]
s_mov_b32 s38, 0x40000000
s_mov_b32 s39, 0x3ff921fb
v_mul_f64 v[18:19], v[22:23], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[18:19]
s_mov_b32 s38, 0
s_mov_b32 s39, 0x3e74442d
v_mul_f64 v[18:19], v[22:23], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[18:19]
s_mov_b32 s38, 0x98cc5170
s_mov_b32 s39, 0x3cf84698
v_mul_f64 v[18:19], v[22:23], s[38:39]
v_add_f64 v[20:21], v[20:21], -v[18:19]
v_cvt_i32_f64 v18, v[22:23]
v_cvt_f32_f64 v19, v[20:21]
.Lfast:
s_mov_b64 exec, s[36:37]
v_mul_f32 v20, v19, v19
v_mov_b32 v21, 0x3638ef1d
v_fmaak_f32 v21, v21, v20, 0xb9500d01
v_fmaak_f32 v21, v21, v20, 0x3c088889
v_fmaak_f32 v21, v21, v20, 0xbe2aaaab
v_mul_f32 v22, v19, v20
v_fma_f32 v21, v22, v21, v19
v_mov_b32 v22, 0xb493f27e
v_fmaak_f32 v22, v22, v20, 0x37d00d01
v_fmaak_f32 v22, v22, v20, 0xbab60b61
v_fmaak_f32 v22, v22, v20, 0x3d2aaaab
v_fmaak_f32 v22, v22, v20, 0xbf000000
v_fma_f32 v22, v20, v22, 1.0
v_and_b32 v23, 1, v18
v_cmp_ne_u32_e32 vcc, 0, v23
s_nop 1
"""

TEMPLATES = {
    # v21 = sin poly(r), v22 = cos poly(r), v18 = quadrant, v24 = |x|; v8 is scratch until the end
    "SIN": REDUCE + """
v_cndmask_b32_e32 v23, v21, v22, vcc
v_and_b32 v18, 2, v18
v_lshlrev_b32 v18, 30, v18
v_xor_b32 v23, v23, v18
v_cmp_gt_f32_e32 vcc, 0x39800000, v24
s_nop 1
v_cndmask_b32_e32 v8, v23, v17, vcc
s_setpc_b64 s[40:41]
""",
    "COS": REDUCE + """
v_cndmask_b32_e32 v23, v22, v21, vcc
v_add_u32 v18, 1, v18
v_and_b32 v18, 2, v18
v_lshlrev_b32 v18, 30, v18
v_xor_b32 v23, v23, v18
v_cmp_ngt_f32_e32 vcc, 0x39800000, v24
s_nop 1
v_cndmask_b32_e32 v8, 1.0, v23, vcc
s_setpc_b64 s[40:41]
""",
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
        # words inside the exec-masked blocks (skipped by s_cbranch_execz when no lane needs them)
        skip = sum(x & 0xFFFF for x in words if (x >> 16) == 0xBF88)
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
