#!/usr/bin/env python3
"""Dopri5 in two launches (MtgpModel.dp_budget): A/B of the first launch's attempt budget on the
C3 Dopri5 workload, interleaved rounds in ONE process; every budget must give the same bits.
Prints one JSON line per budget (median evaluator time over rounds, both launches)."""
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
ap.add_argument("--budgets", default="0,64,128,256,512")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--obs-noise", type=float, default=0.0)
ap.add_argument("--config", default="c3", choices=["c2", "c3"])
ap.add_argument("--legacy-pop", action="store_true",
                help="the round-2 population: per-tree sampler (sampling.sample_tree), same seed -- A/B against "
                     "round-2 measurements")
a = ap.parse_args()
args = bench.apply_config_defaults(argparse.Namespace(config=a.config, pop=None, rollouts=None, ode_steps=200,
                                                      solver="dopri5", obs_noise=a.obs_noise))
env, lib, ff, data, pop = bench.setup_workload(args, 0)
if a.legacy_pop:
    from multitreegp_amd.sampling import create_map_b_to_d, sample_tree
    rng = np.random.default_rng(1000)
    m = create_map_b_to_d(10)
    pop = np.stack([np.stack([sample_tree(rng, lib, lib.variable_array[t], 10, 64, 1.0, m) for t in range(3)])
                    for _ in range(pop.shape[0])]).astype(np.float32)
budgets = [int(b) for b in a.budgets.split(",")]
engs = {b: DeviceEngine(ff, lib, 0.0, "cuda:0", dp_budget=b) for b in budgets}
pd = torch.from_numpy(pop).cuda()
L = nat.load()
L.mtgp_set_timing(1)
times = {b: [] for b in budgets}
ref = None
for rnd in range(a.rounds + 1):
    for b in budgets:
        res = engs[b].evaluate(pd, data, trajectories=True, step_counts=True, check=rnd == 0)
        torch.cuda.synchronize()
        h = (ctypes.c_float * 1)()
        L.mtgp_kernel_ms_history(h, 1)
        if rnd > 0:
            times[b].append(h[0])
        fit = res["fitness"].cpu().numpy().view(np.uint32)
        if ref is None:
            ref = fit
            steps = res["steps"].cpu().numpy()
        assert np.array_equal(fit, ref), f"budget {b}: fitness differs"
pend = {}
for b in budgets:
    if b > 0:
        pend[b] = int(engs[b]._dp_bufs[1][0].item())
for b in budgets:
    print(json.dumps({"config": a.config, "obs_noise": a.obs_noise, "budget": b,
                      "kernel_ms_median": float(np.median(times[b])), "kernel_ms": times[b],
                      "parked_waves": pend.get(b), "attempts_mean": float(steps.mean()),
                      "attempts_max": int(steps.max())}), flush=True)
