"""Pure-Python executor of the flattened program format (test helper).

Executes MtgpInstr programs with float32 numpy scalars; SIN/COS go through the oracle's
shared fp32 math so results are comparable bit-for-bit with the oracle and the kernel."""
import numpy as np

from oracle import oracle as orc

f32 = np.float32


def _sin(x):
    return orc.sincos(np.array([x], np.float32))[0][0]


def _cos(x):
    return orc.sincos(np.array([x], np.float32))[1][0]


_UNARY = {"EXP": 8, "LOG": 9, "SQRT": 10, "TANH": 11, "ABS": 12}  # MTGP_FN_* of the round-3 operators


def _unary(name, x):
    return orc.unary(_UNARY[name], np.array([x], np.float32))[0]


_FAM = {"ADD": lambda x, y: x + y, "SUB": lambda x, y: x - y, "RSUB": lambda x, y: y - x,
        "MUL": lambda x, y: x * y, "DIV": lambda x, y: x / y, "RDIV": lambda x, y: y / x}


def run(prog, data):
    """prog: decoded instructions (name, a, b) from _native.decode_instr."""
    acc = f32(0)
    st = []
    d = [f32(v) for v in np.asarray(data, np.float32).reshape(-1)]
    with np.errstate(all="ignore"):
        for name, a, b in prog:
            if name in ("LDCP", "LDVP", "SINVP", "COSVP") or name.startswith(("VCP_", "VVP_")):
                st.append(acc)
            if name in ("LDC", "LDCP"):
                acc = f32(b)
            elif name in ("LDV", "LDVP"):
                acc = d[a]
            elif name == "SIN":
                acc = _sin(acc)
            elif name == "COS":
                acc = _cos(acc)
            elif name in _UNARY:
                acc = _unary(name, acc)
            elif name in ("SINV", "SINVP"):
                acc = _sin(d[a])
            elif name in ("COSV", "COSVP"):
                acc = _cos(d[a])
            elif name.startswith(("VC_", "VCP_")):
                acc = f32(_FAM[name.split("_")[1]](d[a], f32(b)))
            elif name.startswith(("VV_", "VVP_")):
                acc = f32(_FAM[name.split("_")[1]](d[a], d[b]))
            else:
                fam, kind = name[:-1], name[-1]
                opnd = f32(b) if kind == "C" else (d[a] if kind == "V" else st.pop())
                acc = f32(_FAM[fam](acc, opnd))
    assert not st, "stack not empty at program end"
    return f32(acc)
