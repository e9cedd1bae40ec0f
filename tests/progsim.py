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


def run(prog, data):
    acc = f32(0)
    st = []
    d = [f32(v) for v in np.asarray(data, np.float32).reshape(-1)]
    with np.errstate(all="ignore"):
        for name, slot, imm in prog:
            imm = f32(imm)
            fam = name[:-1] if name[-1] in "CVS" and name not in ("LDC", "LDV") else name
            if name in ("LDCP", "LDVP"):
                st.append(acc)
            if name in ("LDC", "LDCP"):
                acc = imm
                continue
            if name in ("LDV", "LDVP"):
                acc = d[slot]
                continue
            if name == "SIN":
                acc = _sin(acc)
                continue
            if name == "COS":
                acc = _cos(acc)
                continue
            kind = name[-1]
            opnd = imm if kind == "C" else (d[slot] if kind == "V" else st.pop())
            fam = name[:-1]
            if fam == "ADD":
                acc = f32(acc + opnd)
            elif fam == "SUB":
                acc = f32(acc - opnd)
            elif fam == "RSUB":
                acc = f32(opnd - acc)
            elif fam == "MUL":
                acc = f32(acc * opnd)
            elif fam == "DIV":
                acc = f32(acc / opnd)
            elif fam == "RDIV":
                acc = f32(opnd / acc)
            else:
                raise ValueError(name)
    assert not st, "stack not empty at program end"
    return f32(acc)
