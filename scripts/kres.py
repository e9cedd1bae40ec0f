"""Per-kernel resource usage (VGPRs, SGPRs, spills, scratch) of a hipcc -c object or a .so:
python scripts/kres.py OBJ [name-filter].  Unbundles the gfx950 code object and reads its notes."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path, tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", path], check=True)
    co = os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def kernels(path):
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(path, tmp)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"private_segment_fixed_size|agpr_count):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name":
            cur = {"name": v}
            out.append(cur)
        else:
            cur[k] = int(v)
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    dem = lambda n: subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()  # noqa: E731
    for k in kernels(sys.argv[1]):
        name = dem(k["name"])
        if flt in name:
            print(f"vgpr {k.get('vgpr_count', 0):4d} agpr {k.get('agpr_count', 0):3d} sgpr {k.get('sgpr_count', 0):3d} "
                  f"vspill {k.get('vgpr_spill_count', 0):3d} sspill {k.get('sgpr_spill_count', 0):3d} "
                  f"scratch {k.get('private_segment_fixed_size', 0):4d}  {name[:150]}")
