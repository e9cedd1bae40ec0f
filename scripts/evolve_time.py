#!/usr/bin/env python3
"""Time GeneticProgramming.evolve (the native host library) on a configuration's population:
scripts/evolve_time.py --config c5 [--threads 8] -> median ms per generation (CPU only)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multitreegp_amd.genetic_programming import GeneticProgramming  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c5")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
ns = bench.apply_config_defaults(argparse.Namespace(pop=None, rollouts=None, ode_steps=200, config=a.config,
                                                    solver="rk4", obs_noise=0.0))
env, lib, ff, data, pop = bench.setup_workload(ns, 0)
P = pop.shape[0]
gp = GeneticProgramming(1, P, ff, lib.operator_list, lib.variable_list, lib.layer_sizes, max_nodes=pop.shape[2],
                        migration_percentage=0.0, elite_percentage=0.0, verbose=False)
fit = np.random.default_rng(0).random(P).astype(np.float32)
full = pop[None]
ts = []
for i in range(a.reps):
    t0 = time.perf_counter()
    gp.evolve(full, fit[None], 1000 + i)
    ts.append((time.perf_counter() - t0) * 1e3)
print(json.dumps({"config": a.config, "P": P, "shape": list(pop.shape), "threads": os.environ.get("MTGP_HOST_THREADS", "8"),
                  "ms_median": float(np.median(ts[1:])), "ms_all": [round(t, 2) for t in ts]}))
