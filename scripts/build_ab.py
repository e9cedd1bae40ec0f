#!/usr/bin/env python3
"""Build diagnostic A/B variants of the kernel library (mtgp_ab.h knobs) for scripts/kvariants.py
and PMC passes.  Only one translation unit (MTGP_AB_TU, default 7 = the fixed-step Acrobot kernels)
is recompiled with the variant's defines; the other units' objects are the product build's.  Output:
multitreegp_amd/lib/abrun/libmtgp_hip_<name>.so (delete the directory after the GPU run: it is
pushed with the tree).

usage: build_ab.py name=DEF[,DEF...] [name=...]      e.g. notrig=MTGP_AB_NOTRIG=1"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

TU = int(os.environ.get("MTGP_AB_TU", "7"))


def build(name, defines):
    g.build_hip()  # product objects up to date
    objdir = os.path.join(g.LIBDIR, "obj")
    vdir = os.path.join(g.LIBDIR, "obj", "ab_" + name)
    os.makedirs(vdir, exist_ok=True)
    obj0 = os.path.join(vdir, f"mtgp_kernels_tu{TU}.o")
    cflags = [f for f in g.HIPCC_FLAGS if f != "-shared"]
    cmd = ["/opt/rocm/bin/hipcc", *cflags, "-c", f"-DMTGP_TU={TU}", *[f"-D{d}" for d in defines],
           "-I", os.path.join(ROOT, "include"), "-I", g.CSRC, os.path.join(g.CSRC, "mtgp_kernels.hip"), "-o", obj0]
    return subprocess.Popen(cmd), obj0, objdir


def main():
    jobs = []
    for arg in sys.argv[1:]:
        name, defs = arg.split("=", 1)
        jobs.append((name, defs.split(",")) )
    procs = [(name, *build(name, defs)) for name, defs in jobs]
    out_dir = os.path.join(g.LIBDIR, "abrun")
    os.makedirs(out_dir, exist_ok=True)
    for name, p, obj0, objdir in procs:
        if p.wait() != 0:
            raise SystemExit(f"hipcc failed for {name}")
        objs = [obj0] + [os.path.join(objdir, f"mtgp_kernels_tu{tu}.o") for tu in g.HIP_TUS if tu != TU] + \
               [os.path.join(objdir, "mtgp_grad.o"), os.path.join(objdir, "mtgp_build_info.o")]  # (the
        # product's build info: a variant reports the product's sources hash)
        out = os.path.join(out_dir, f"libmtgp_hip_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-fPIC", "-shared", *objs, "-o", out,
                        "-L/opt/rocm/lib", "-lhsa-runtime64"], check=True)
        print("built", out)


if __name__ == "__main__":
    main()
