#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

The reference (JAX + diffrax) cannot be imported in this container (ModuleNotFoundError,
SURVEY.md §8c) and its repository holds no golden vectors, so these fixtures are produced by
oracle/mtgp_oracle.c (itself pinned by tests/test_oracle.py: float64 restatement, sympy on the
reference's printer, analytic RK4 known answers, and -- for the fixed-step solve -- a literal float32
restatement of diffrax's ConstantStepSize loop).  They freeze oracle outputs for regression
and give the GPU parity tests fixed targets.  Parity vs the JAX reference: UNPINNED.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from helpers import dynamic_setup, oracle_model, oracle_rollouts, sr_setup, static_setup  # noqa: E402
from oracle import oracle as orc  # noqa: E402

def _notebook_grid():
    """C3 trees on the notebooks' save grid ts = arange(0, T, 0.2) with dt0 0.05 (DynamicPolicy.ipynb:55):
    diffrax's accumulated step ends never coincide with the save times (ABI v18 dense output)."""
    env, lib, ff, data, pop = dynamic_setup(P=16, R=8, n_steps=40, depth=10, N=64, seed=14)
    data = (data[0], np.arange(0, 6, 0.2).astype(np.float32)) + tuple(data[2:])
    return env, lib, ff, data, pop


def _sr_euler_nonuniform():
    """SR with the reference's default Euler solver on a non-uniform save grid."""
    import multitreegp_amd as mt
    env, lib, ff, data, pop = sr_setup(P=16, R=4, n_save=21, save_every=4, depth=5, N=30, seed=15)
    ts = np.sort(np.random.default_rng(15).uniform(0.0, 4.0, 21)).astype(np.float32)
    ts[0] = 0.0
    x0 = data[0]
    ys = mt.ground_truth(env, x0, ts)
    ff = mt.SREvaluator(solver=mt.Euler(), dt0=0.05)
    return env, lib, ff, (x0, ts, ys, data[3]), pop


CASES = {
    "c1_sr_vanderpol": lambda: sr_setup(P=16, R=4, n_save=21, save_every=4, depth=5, N=30, seed=11),
    "c2_static_acrobot": lambda: static_setup(P=16, R=4, n_steps=50, depth=4, N=30, seed=12),
    "c3_dynamic_acrobot": lambda: dynamic_setup(P=16, R=8, n_steps=50, depth=10, N=64, seed=13),
    "c3_dynamic_acrobot_notebook_grid": _notebook_grid,
    "c1_sr_euler_nonuniform": _sr_euler_nonuniform,
}


def main():
    for name, make in CASES.items():
        env, lib, ff, data, pop = make()
        d = ff.prepare(data)
        model = oracle_model(ff, d, parsimony=0.25)
        ro = oracle_rollouts(d)
        out = orc.evaluate(model, pop, lib, ro, trajectories=True)
        arrays = {"pop": pop, "x0": d["x0"], "ts": d["ts"]}
        if d.get("params") is not None:
            arrays["params"] = d["params"]
        if ro.get("ys_true") is not None:
            arrays["ys_true"] = ro["ys_true"]
        for k, v in model.items():
            arrays[f"model_{k}"] = np.asarray(v)
        for k, v in out.items():
            arrays[f"out_{k}"] = v
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        print(name, {k: v.shape for k, v in arrays.items() if v.ndim})


if __name__ == "__main__":
    main()
