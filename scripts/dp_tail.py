#!/usr/bin/env python3
"""Where the C3 Dopri5 kernel time goes: the evaluator timed on the full population, on only the
individuals whose slowest rollout needs >= --tail attempts, on the slowest individual alone, and on
the population without the tail.  If the tail-only times match the full one, the kernel is bound by
the serial attempt latency of its slowest waves, not by throughput.  One JSON line per case."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multitreegp_amd import _native as nat  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tail", type=int, default=900)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--obs-noise", type=float, default=0.0)
ap.add_argument("--budget", type=int, default=0)
a = ap.parse_args()
args = bench.apply_config_defaults(argparse.Namespace(config="c3", pop=None, rollouts=None, ode_steps=200,
                                                      solver="dopri5", obs_noise=a.obs_noise))
env, lib, ff, data, pop = bench.setup_workload(args, 0)
eng = DeviceEngine(ff, lib, 0.0, "cuda:0", dp_budget=a.budget)
L = nat.load()
L.mtgp_set_timing(1)


def timed(p, rounds):
    pd = torch.from_numpy(np.ascontiguousarray(p)).cuda()
    ts = []
    res = None
    for r in range(rounds + 1):
        res = eng.evaluate(pd, data, trajectories=True, step_counts=True, check=r == 0)
        torch.cuda.synchronize()
        h = (ctypes.c_float * 1)()
        L.mtgp_kernel_ms_history(h, 1)
        if r > 0:
            ts.append(h[0])
    return float(np.median(ts)), res


t_full, res = timed(pop, a.rounds)
steps = res["steps"].cpu().numpy().reshape(pop.shape[0], -1)
per_ind = steps.max(axis=1)
tail = np.nonzero(per_ind >= a.tail)[0]
rest = np.nonzero(per_ind < a.tail)[0]
worst = int(np.argmax(per_ind))
hist = np.histogram(per_ind, bins=[0, 50, 100, 200, 400, 600, 800, 999, 1001])[0].tolist()
print(json.dumps({"case": "full", "P": int(pop.shape[0]), "kernel_ms": t_full,
                  "individual_max_attempts_hist": hist, "hist_edges": [0, 50, 100, 200, 400, 600, 800, 999, 1001],
                  "tail_individuals": int(tail.size), "lane_attempts_mean": float(steps.mean())}), flush=True)
cases = [("tail_only", tail), ("worst_x2", np.array([worst, worst])), ("no_tail", rest)]
for name, idx in cases:
    if idx.size == 0:
        continue
    t, r = timed(pop[idx], a.rounds)
    s = r["steps"].cpu().numpy().reshape(idx.size, -1)
    print(json.dumps({"case": name, "P": int(idx.size), "kernel_ms": t, "max_attempts": int(s.max()),
                      "us_per_attempt_of_slowest": 1e3 * t / max(1, int(s.max()))}), flush=True)
