#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

The reference (JAX + diffrax) cannot be imported in this container (ModuleNotFoundError,
SURVEY.md §8c) and its repository holds no golden vectors, so these fixtures are produced by
oracle/mtgp_oracle.c (itself pinned by tests/test_oracle.py: float64 restatement, sympy on the
reference's printer, analytic RK4 known answers).  They freeze oracle outputs for regression
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

CASES = {
    "c1_sr_vanderpol": lambda: sr_setup(P=16, R=4, n_save=21, save_every=4, depth=5, N=30, seed=11),
    "c2_static_acrobot": lambda: static_setup(P=16, R=4, n_steps=50, depth=4, N=30, seed=12),
    "c3_dynamic_acrobot": lambda: dynamic_setup(P=16, R=8, n_steps=50, depth=10, N=64, seed=13),
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
