#!/usr/bin/env python3
"""Design study (CPU, oracle): how far apart in save index are the lanes of one wave in the C3
Dopri5 workload?  The Dopri5 kernel writes each lane's save point k when that lane's accepted step
passes ts[k]; lanes of one wave reach k at different attempt iterations, so the rows are written
piecemeal (write amplification).  A per-wave LDS ring of W rows can collect a
row and flush it whole once every lane of the wave is past it; a lane more than W rows ahead of
the wave's oldest open row falls back to a direct store.  This replays the kernel's lock-step
attempt loop from the oracle's per-save attempt indices (oracle_set_save_trace) and reports, for
several W, the fraction of save writes the ring would take.

    python scripts/dp_save_spread.py --pop 256"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from helpers import oracle_model, oracle_rollouts  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pop", type=int, default=256)
ap.add_argument("--obs-noise", type=float, default=0.0)
ap.add_argument("--rings", default="2,4,6,8,12,16,32")
a = ap.parse_args()
args = bench.apply_config_defaults(argparse.Namespace(pop=None, rollouts=None, ode_steps=200, config="c3",
                                                      solver="dopri5", obs_noise=a.obs_noise))
env, lib, ff, data, pop = bench.setup_workload(args, 0)
pop = pop[: a.pop]
d = ff.prepare(data)
model, ro = oracle_model(ff, d), oracle_rollouts(d)
P, R, S = pop.shape[0], d["R"], d["n_save"]
trace = np.full((P, R, S), -1, np.int32)
L = orc.lib()
L.oracle_set_save_trace.argtypes = [ctypes.c_void_p]
L.oracle_set_save_trace(trace.ctypes.data)
try:
    out = orc.evaluate(model, pop, lib, ro, steps=True)
finally:
    L.oracle_set_save_trace(None)
steps = out["steps"].reshape(P, R)
# waves: 64 lanes = 2 individuals x 32 rollouts (consecutive individuals)
G = 64 // R
rings = [int(x) for x in a.rings.split(",")]
took = {w: 0 for w in rings}
total = 0
spread_max = []
for w0 in range(0, P, G):
    tr = trace[w0: w0 + G].reshape(-1, S)  # [lanes, S] attempt index per save (-1: fill)
    lanes = tr.shape[0]
    n_it = int(tr.max()) + 1
    # rows written per iteration: each lane's save k at attempt tr[l, k]; the wave's oldest open row
    # at iteration i = min over lanes of their next unsaved k (lanes whose solve ended: S)
    written = [(int(tr[l, k]), l, k) for l in range(lanes) for k in range(S) if tr[l, k] >= 0]
    written.sort()
    total += len(written)
    # replay: iteration by iteration
    by_it = {}
    for it, l, k in written:
        by_it.setdefault(it, []).append((l, k))
    done_k = np.zeros(lanes, np.int64)  # next unsaved k per lane
    end_it = np.array([max(tr[l].max(), 0) for l in range(lanes)])
    smax = 0
    for it in sorted(by_it):
        # lanes that ended before this iteration no longer hold the ring back
        live = end_it >= it
        base = int(done_k[live].min()) if live.any() else S
        for l, k in by_it[it]:
            for w in rings:
                if k < base + w:
                    took[w] += 1
            smax = max(smax, k - base)
        for l, k in by_it[it]:
            done_k[l] = max(done_k[l], k + 1)
    spread_max.append(smax)
print(json.dumps({"individuals": P, "rollouts": R, "saves": S, "writes": total,
                  "ring_fraction": {str(w): took[w] / max(total, 1) for w in rings},
                  "spread_max_p50": float(np.median(spread_max)), "spread_max_p90": float(np.percentile(spread_max, 90)),
                  "attempts_mean": float(steps.mean()), "attempts_max": int(steps.max())}))
