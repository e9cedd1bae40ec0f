#!/usr/bin/env python3
"""Marginal cost of one interpreted instruction in the C3 kernel: every tree of the population
is a chain of k additions (y1 + c + c + ... -> VC_ADD, (k-1) x ADDC, END), timed for several k
with trajectories on (no early exit).  slope = ns per (wave x dispatch)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402


def chain_tree(lib, k, N, var="y1", op="+"):
    rows = np.tile(np.array([0.0, -1.0, -1.0, 0.0], np.float32), (N, 1))
    r = N - 1 - 2 * k
    rows[r] = [lib.string_to_node[var], -1, -1, 0.0]
    prev = r
    for i in range(k):
        c, a = r + 1 + 2 * i, r + 2 + 2 * i
        rows[c] = [1, -1, -1, 1e-3]
        rows[a] = [lib.string_to_node[op], prev, c, 0.0]
        prev = a
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="0,1,2,4,8,16,31")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    env, lib, ff, data, _ = bench.setup_workload(argparse.Namespace(pop=8, rollouts=32, ode_steps=200, config="c3"), 0)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    P, N = 8192, 64
    for k in [int(x) for x in a.ks.split(",")]:
        t = chain_tree(lib, k, N)
        pop = np.broadcast_to(t, (P, 3, N, 4)).copy()
        pd = torch.from_numpy(pop).cuda()
        fl = eng.flatten(pd)
        eng.check_status(fl)
        ms = []
        for r in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.evaluate(pd, data, trajectories=True, flattened=fl, check=False)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ms.append(e0.elapsed_time(e1))
        plen = int(fl.plen[0, 0].item())
        print(json.dumps({"k": k, "prog_len": plen, "median_ms": float(np.median(ms))}), flush=True)


if __name__ == "__main__":
    main()
