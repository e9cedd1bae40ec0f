"""The C ABI library: loads without a GPU, exports every declared symbol, struct layouts match."""
import ctypes
import os
import re
import subprocess

import numpy as np

from multitreegp_amd import _native as nat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mtgp.h")


def test_declared_symbols_exported():
    text = open(HDR).read()
    declared = set(re.findall(r"^\s*(?:int|float)\s+(mtgp_\w+)\s*\(", text, re.M))
    assert declared == set(nat.EXPORTED_SYMBOLS)
    lib = nat.load()
    for sym in declared:
        assert hasattr(lib, sym)
    assert lib.mtgp_abi_version() == nat.ABI_VERSION


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mtgp.h"\nint main(){printf("%zu %zu %zu %zu %zu %zu %zu\\n",'
                   'sizeof(MtgpNodeLibrary), sizeof(MtgpProgramSpec), sizeof(MtgpInstr), sizeof(MtgpModel),'
                   'sizeof(MtgpRollouts), sizeof(MtgpOutputs), offsetof(MtgpModel, readout_save_same));'
                   'printf("%zu %zu %zu %zu %zu\\n", offsetof(MtgpRollouts, lanes), offsetof(MtgpModel, dp_budget),'
                   'sizeof(MtgpGradJit), offsetof(MtgpGradJit, info), offsetof(MtgpOutputs, traj_layout));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(t) for t in (nat.MtgpNodeLibrary, nat.MtgpProgramSpec, nat.MtgpInstr, nat.MtgpModel,
                                       nat.MtgpRollouts, nat.MtgpOutputs)] + [nat.MtgpModel.readout_save_same.offset,
                                                                              nat.MtgpRollouts.lanes.offset,
                                                                              nat.MtgpModel.dp_budget.offset,
                                                                              ctypes.sizeof(nat.MtgpGradJit),
                                                                              nat.MtgpGradJit.info.offset,
                                                                              nat.MtgpOutputs.traj_layout.offset]
    assert got == want


def test_argument_validation_without_gpu():
    """Bad arguments are rejected before any device call (no GPU needed)."""
    lib = nat.load()
    nl = nat.MtgpNodeLibrary()
    assert lib.mtgp_flatten(None, 1, 1, 1, ctypes.byref(nl), None, 1, 8, None, None, None, None, None) == nat.ERR_ARG
    m = nat.MtgpModel()
    ro = nat.MtgpRollouts()
    out = nat.MtgpOutputs()
    assert lib.mtgp_eval_rk4(ctypes.byref(m), None, None, 1, 1, None, 1, ctypes.byref(ro), ctypes.byref(out),
                             None) == nat.ERR_ARG
    one = np.zeros(4, np.int32)
    m.n_steps, m.save_every, m.n_save = 10, 3, 4  # n_steps not a multiple of save_every
    ro.R = 4
    out.fitness = one.ctypes.data
    assert lib.mtgp_eval_rk4(ctypes.byref(m), one.ctypes.data, one.ctypes.data, 1, 1, one.ctypes.data, 1,
                             ctypes.byref(ro), ctypes.byref(out), None) == nat.ERR_ARG
    m.save_every = 2
    m.n_save = 6

    def rk4():
        return lib.mtgp_eval_rk4(ctypes.byref(m), one.ctypes.data, one.ctypes.data, 1, 4, one.ctypes.data, 1,
                                 ctypes.byref(ro), ctypes.byref(out), None)
    ro.R = 65  # lane set over two waves: the mean is formed from rollout_fitness, which is missing
    assert rk4() == nat.ERR_ARG
    ro.R, ro.lanes = 8, 4  # lane set narrower than R
    assert rk4() == nat.ERR_ARG
    ro.lanes = 24  # not a power of two
    assert rk4() == nat.ERR_ARG
    ro.R, ro.lanes = nat.MAX_ROLLOUTS + 1, 0
    assert rk4() == nat.ERR_ARG
    # launch geometry (sizes of the Dopri5 parked-state buffers)
    assert lib.mtgp_eval_waves(8192, 32, 0) == 4096  # C3: two individuals per wave
    assert lib.mtgp_eval_waves(1024, 16, 64) == 1024  # C2 lane set widened: one per wave
    assert lib.mtgp_eval_waves(10, 128, 0) == 20      # R > 64: two waves per individual
    assert lib.mtgp_eval_waves(7, 100, 0) == 14
    assert lib.mtgp_eval_waves(5, 8, 4) == nat.ERR_ARG and lib.mtgp_eval_waves(5, 8, 12) == nat.ERR_ARG
    ro.R, ro.lanes = 8, 0
    ro.x0 = ro.ts = ro.params = one.ctypes.data
    m.solver, m.dp_budget, m.max_steps, m.h, m.n_save = 1, 16, 10, 0.1, 4  # Dopri5 in two launches:
    out.dp_state = None                                                     # the parked-state buffer is required
    m.model, m.n_var, m.n_obs, m.n_control, m.state_size = 1, 4, 4, 1, 2  # otherwise a valid Acrobot model
    assert rk4() == nat.ERR_ARG
    # lane-major trajectory rows (ABI v20) only for the adaptive solve; unknown layouts rejected
    m.solver, m.dp_budget, m.max_steps, m.n_save = 0, 0, 0, 4
    out.xs, out.traj_layout = one.ctypes.data, nat.TRAJ_LANE_MAJOR
    assert rk4() == nat.ERR_ARG
    out.traj_layout = 7
    assert rk4() == nat.ERR_ARG


def _define(text, name):
    m = re.search(rf"#define\s+{name}\s+\(?([0-9]+)u?\s*(?:\*\s*(\w+))?\)?", text)
    assert m, name
    v = int(m.group(1))
    return v * _define(text, m.group(2)) if m.group(2) else v


def test_constants_match_header():
    text = open(HDR).read()
    assert _define(text, "MTGP_ABI_VERSION") == nat.ABI_VERSION
    assert _define(text, "MTGP_SLOT_BYTES") == nat.SLOT_BYTES
    assert _define(text, "MTGP_SCHED_BINS") == nat.SCHED_BINS
    assert _define(text, "MTGP_SCHED_SCRATCH") == nat.SCHED_SCRATCH
    assert _define(text, "MTGP_MAX_PROGRAMS") == nat.MAX_PROGRAMS
    assert _define(text, "MTGP_STACK_MAX") == nat.STACK_MAX
    assert _define(text, "MTGP_MAX_ROLLOUTS") == nat.MAX_ROLLOUTS
    assert _define(text, "MTGP_DP_STATE_WORDS") == nat.DP_STATE_WORDS
    assert _define(text, "MTGP_GRAD_JIT_WORDS_PER_INSTR") == nat.GRAD_JIT_WORDS_PER_INSTR
    assert _define(text, "MTGP_TRAJ_TIME_MAJOR") == nat.TRAJ_TIME_MAJOR
    assert _define(text, "MTGP_TRAJ_LANE_MAJOR") == nat.TRAJ_LANE_MAJOR
    ops = open(os.path.join(ROOT, "include", "mtgp_opcodes.h")).read()
    pairs = re.findall(r"MTGP_OP_(\w+) = (\d+),", ops)
    assert [n for n, _ in pairs] == nat.OP_NAMES and [int(v) for _, v in pairs] == list(range(len(pairs)))


def test_generated_opcode_files_up_to_date():
    """include/mtgp_opcodes.h, csrc/mtgp_dispatch.inc and _opcodes.py match scripts/gen_opcodes.py."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_opcodes", os.path.join(ROOT, "scripts", "gen_opcodes.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    out = gen.generate()
    for path, i in gen.targets().items():
        assert open(path).read() == out[i], f"{path} is stale: run scripts/gen_opcodes.py"


def test_unaligned_program_stride_rejected():
    """The evaluators fetch four instructions per scalar load: L % 4 != 0 is an argument error."""
    lib = nat.load()
    one = np.zeros(8, np.int32)
    m = nat.MtgpModel()
    m.n_steps, m.save_every, m.n_save = 4, 1, 5
    ro = nat.MtgpRollouts()
    ro.R, ro.x0, ro.ts = 4, one.ctypes.data, one.ctypes.data
    out = nat.MtgpOutputs()
    out.fitness = one.ctypes.data
    assert lib.mtgp_eval_rk4(ctypes.byref(m), one.ctypes.data, one.ctypes.data, 1, 6, one.ctypes.data, 1,
                             ctypes.byref(ro), ctypes.byref(out), None) == nat.ERR_ARG
    assert lib.mtgp_eval_programs(one.ctypes.data, one.ctypes.data, 1, 6, 1, one.ctypes.data, 1, 1,
                                  one.ctypes.data, None) == nat.ERR_ARG


def _local_includes(path, seen):
    """Every quoted #include reachable from path, resolved in csrc/ then include/."""
    import __graft_entry__ as ge
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', open(path).read(), re.M):
        for d in (ge.CSRC, os.path.join(ge.ROOT, "include")):
            p = os.path.join(d, name)
            if os.path.exists(p):
                if p not in seen:
                    seen.add(p)
                    _local_includes(p, seen)
                break
        else:
            raise AssertionError(f"{path}: include {name} not found in csrc/ or include/")
    return seen


def test_hip_sources_cover_every_included_header():
    """HIP_SOURCES decides when libmtgp_hip.so is rebuilt and what its sources hash covers: every
    header a kernel source includes (transitively) must be listed (mtgp_jit_dual.h was not)."""
    import __graft_entry__ as ge
    listed = {os.path.realpath(p) for p in ge.HIP_SOURCES}
    for src in [p for p in ge.HIP_SOURCES if p.endswith(".hip")]:
        for h in _local_includes(src, set()):
            assert os.path.realpath(h) in listed, f"{h} (included by {src}) is missing from HIP_SOURCES"


def test_build_info_matches_tree():
    """Build provenance by content: the library embeds the SHA-256 of the sources it was built from."""
    import __graft_entry__ as ge
    info = nat.build_info()
    assert info.get("sources_sha256") == ge.sources_hash(), \
        "libmtgp_hip.so was built from other sources than this tree: run __graft_entry__.build()"
