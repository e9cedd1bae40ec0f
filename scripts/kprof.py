#!/usr/bin/env python3
"""Kernel-only driver for rocprofv3 (PMC passes and --kernel-trace --stats): the bench's own
workload (bench.setup_workload; --pop / --rollouts default to the configuration's sizes,
bench.CONFIG_DEFAULTS), N evaluations.  No worker processes are started (a pool forked under
rocprofv3 inherits its signal handlers)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multitreegp_amd import _native as nat  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--warmup", type=int, default=0,
                help="evaluations before the --iters ones (traced too; kstats_db.py --skip drops them)")
ap.add_argument("--pop", type=int, default=None, help="default: the config's (bench.CONFIG_DEFAULTS)")
ap.add_argument("--rollouts", type=int, default=None)
ap.add_argument("--no-traj", action="store_true")
ap.add_argument("--lib", default=nat.LIB_PATH)
ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
ap.add_argument("--solver", default="rk4", choices=["rk4", "dopri5"])
ap.add_argument("--obs-noise", type=float, default=0.0)
ap.add_argument("--ode-steps", type=int, default=200)
ap.add_argument("--state-size", type=int, default=2)
a = bench.apply_config_defaults(ap.parse_args())
env, lib, ff, data, pop = bench.setup_workload(argparse.Namespace(pop=a.pop, rollouts=a.rollouts, ode_steps=a.ode_steps,
                                                                      config=a.config, solver=a.solver,
                                                                      obs_noise=a.obs_noise, state_size=a.state_size), 0)
eng = DeviceEngine(ff, lib, 0.0, "cuda:0", native=nat.load(a.lib))
pd = torch.from_numpy(pop).cuda()
for i in range(a.warmup + a.iters):  # statuses checked once (the timed bench loop never synchronises either)
    eng.evaluate(pd, data, trajectories=not a.no_traj, step_counts=a.solver == "dopri5", check=i == 0)
torch.cuda.synchronize()
print("done")
