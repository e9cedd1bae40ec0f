"""Lane utilisation of the adaptive Dopri5 kernel (C3, bench workload): a wave iterates until its
slowest lane is done, so the useful fraction of wave iterations is mean attempts / mean over waves
of the wave's max attempts.  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402

args = bench.parse()
env, lib, ff, data, pop = bench.setup_workload(args, 0)
eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
pd = torch.from_numpy(pop).cuda()
res = eng.evaluate(pd, data, trajectories=not args.no_traj, step_counts=True)
torch.cuda.synchronize()
st = res["steps"].cpu().numpy()  # [P, R]
P, R = st.shape
order = eng.schedule(res["_flat"], R).cpu().numpy()
Rp = 1 << (R - 1).bit_length()
G = 64 // Rp
per_ind = st.max(axis=1)
waves = [per_ind[order[q:q + G]].max() for q in range(0, P, G)]
fin = res["fitness"].cpu().numpy()
out = {"P": P, "R": R, "mean_attempts": float(st.mean()), "median": float(np.median(st)),
       "p99": float(np.percentile(st, 99)), "max": int(st.max()), "frac_at_max_steps": float((st >= ff.max_steps).mean()),
       "mean_wave_max": float(np.mean(waves)), "lane_utilisation": float(st.mean() / np.mean(waves)),
       "frac_individuals_max_fitness": float((fin >= ff.max_fitness).mean())}
print(json.dumps(out), flush=True)
