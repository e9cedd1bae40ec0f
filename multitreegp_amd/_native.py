"""ctypes binding of the C ABI declared in ``include/mtgp.h``.

The HIP library ``multitreegp_amd/lib/libmtgp_hip.so`` is built in-tree by
``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).  There is no fallback: if the
library is missing or a GPU is absent, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmtgp_hip.so")

MAX_FUNCS = 128
MAX_NODES = 256
MAX_DATA = 64
STACK_MAX = 8
MAX_PROGRAMS = 64
SCHED_BINS = 4096
SCHED_SCRATCH = 2 * SCHED_BINS
ABI_VERSION = 3

OK = 0
ERR_ARG = -1
ERR_LAUNCH = -2
ERR_PROG_TOO_LONG = 3
ERR_STACK = 4

FN_ZERO, FN_VAR, FN_ADD, FN_SUB, FN_MUL, FN_DIV, FN_SIN, FN_COS = range(8)

MODEL_ACROBOT_DYNAMIC = 1
MODEL_ACROBOT_STATIC = 2
MODEL_SR = 3

OP_NAMES = [
    "LDC", "LDCP", "LDV", "LDVP",
    "ADDC", "SUBC", "RSUBC", "MULC", "DIVC", "RDIVC",
    "ADDV", "SUBV", "RSUBV", "MULV", "DIVV", "RDIVV",
    "ADDS", "SUBS", "RSUBS", "MULS", "DIVS", "RDIVS",
    "SIN", "COS", "END",
]
SLOT_BYTES = 256  # V opcodes carry slot * SLOT_BYTES in the imm bits (mtgp.h program format)


def decode_instr(op: int, imm_bits: int):
    """(name, slot, imm) of one MtgpInstr; slot is 0 except for V opcodes."""
    name = OP_NAMES[op]
    if name[-1] == "V" or name in ("LDV", "LDVP"):
        return name, imm_bits // SLOT_BYTES, 0.0
    return name, 0, float(np.array(imm_bits, dtype=np.uint32).view(np.float32))


class MtgpNodeLibrary(ctypes.Structure):
    _fields_ = [("n_funcs", ctypes.c_int32), ("var_start", ctypes.c_int32),
                ("fn", ctypes.c_int8 * MAX_FUNCS)]


class MtgpProgramSpec(ctypes.Structure):
    _fields_ = [("tree", ctypes.c_int32), ("n_data", ctypes.c_int32),
                ("zero_mask", ctypes.c_uint64)]


class MtgpInstr(ctypes.Structure):
    _fields_ = [("op", ctypes.c_uint32), ("imm", ctypes.c_float)]


class MtgpModel(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32), ("n_var", ctypes.c_int32), ("state_size", ctypes.c_int32),
        ("n_obs", ctypes.c_int32), ("n_control", ctypes.c_int32), ("n_targets", ctypes.c_int32),
        ("n_steps", ctypes.c_int32), ("save_every", ctypes.c_int32), ("n_save", ctypes.c_int32),
        ("h", ctypes.c_float), ("max_fitness", ctypes.c_float), ("parsimony", ctypes.c_float),
        ("prog_state", ctypes.c_int32), ("prog_readout", ctypes.c_int32),
        ("prog_readout_save", ctypes.c_int32), ("readout_save_same", ctypes.c_int32),
    ]


class MtgpRollouts(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_void_p), ("params", ctypes.c_void_p), ("targets", ctypes.c_void_p),
                ("ts", ctypes.c_void_p), ("ys_true", ctypes.c_void_p), ("R", ctypes.c_int32),
                ("order", ctypes.c_void_p)]


class MtgpOutputs(ctypes.Structure):
    _fields_ = [("fitness", ctypes.c_void_p), ("rollout_fitness", ctypes.c_void_p),
                ("xs", ctypes.c_void_p), ("ys", ctypes.c_void_p), ("us", ctypes.c_void_p),
                ("acts", ctypes.c_void_p)]


# every symbol include/mtgp.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "mtgp_abi_version",
    "mtgp_flatten",
    "mtgp_flatten_tree_host",
    "mtgp_eval_programs",
    "mtgp_eval_rk4",
    "mtgp_schedule",
    "mtgp_last_kernel_ms",
    "mtgp_set_timing",
)

_lib: Optional[ctypes.CDLL] = None


class NativeLibraryMissing(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the HIP library (cached).  Raises NativeLibraryMissing if it is not built."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.mtgp_abi_version.restype = ctypes.c_int
    lib.mtgp_flatten.argtypes = [vp, i32, i32, i32, ctypes.POINTER(MtgpNodeLibrary), vp, i32, i32,
                                 vp, vp, vp, vp, vp]
    lib.mtgp_flatten.restype = ctypes.c_int
    lib.mtgp_flatten_tree_host.argtypes = [vp, i32, ctypes.POINTER(MtgpNodeLibrary), i32,
                                           ctypes.c_uint64, i32, vp, ctypes.POINTER(i32)]
    lib.mtgp_flatten_tree_host.restype = ctypes.c_int
    lib.mtgp_eval_programs.argtypes = [vp, vp, i32, i32, i32, vp, i32, i32, vp, vp]
    lib.mtgp_eval_programs.restype = ctypes.c_int
    lib.mtgp_eval_rk4.argtypes = [ctypes.POINTER(MtgpModel), vp, vp, i32, i32, vp, i32,
                                  ctypes.POINTER(MtgpRollouts), ctypes.POINTER(MtgpOutputs), vp]
    lib.mtgp_eval_rk4.restype = ctypes.c_int
    lib.mtgp_schedule.argtypes = [vp, i32, i32, ctypes.POINTER(i32), i32, vp, vp, vp]
    lib.mtgp_schedule.restype = ctypes.c_int
    lib.mtgp_last_kernel_ms.restype = ctypes.c_float
    lib.mtgp_set_timing.argtypes = [ctypes.c_int]
    lib.mtgp_set_timing.restype = ctypes.c_int
    if lib.mtgp_abi_version() != ABI_VERSION:
        raise RuntimeError("libmtgp_hip ABI version mismatch")
    if path == LIB_PATH:
        _lib = lib
    return lib


def node_library_struct(n_funcs: int, var_start: int, fn_codes) -> MtgpNodeLibrary:
    lib = MtgpNodeLibrary()
    lib.n_funcs = int(n_funcs)
    lib.var_start = int(var_start)
    for i, c in enumerate(fn_codes):
        lib.fn[i] = int(c)
    return lib


def flatten_tree_host(tree: np.ndarray, node_lib: MtgpNodeLibrary, n_data: int, zero_mask: int = 0,
                      L: Optional[int] = None):
    """Host-side flatten of one [N, 4] tree (same code as the device kernel).

    Returns (instructions as list of (opname, slot, imm), stack_need).  Raises ValueError on
    flatten errors."""
    lib = load()
    t = np.ascontiguousarray(tree, dtype=np.float32)
    N = t.shape[0]
    L = L or 2 * N + 8
    out = (MtgpInstr * L)()
    need = ctypes.c_int32(0)
    n = lib.mtgp_flatten_tree_host(t.ctypes.data, N, ctypes.byref(node_lib), n_data, zero_mask, L,
                                   ctypes.addressof(out), ctypes.byref(need))
    if n <= 0:
        raise ValueError(f"flatten failed with code {n}")
    raw = np.frombuffer(bytes(out), dtype=np.uint32).reshape(-1, 2)
    assert raw[n, 0] == OP_NAMES.index("END")
    prog = [decode_instr(int(raw[i, 0]), int(raw[i, 1])) for i in range(n)]
    return prog, int(need.value)
