#!/usr/bin/env python3
"""How often the C3 JIT calls report lanes that need the interpreter (slow sin/cos reduction):
diagnostic library built with MTGP_AB_FBCOUNT=1 (scripts/build_ab.py fbcount=MTGP_AB_FBCOUNT=1)."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multitreegp_amd import _native as nat  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--obs-noise", type=float, default=0.0)
args = ap.parse_args()
ns = argparse.Namespace(pop=None, rollouts=None, ode_steps=200, config=args.config, solver="rk4", obs_noise=args.obs_noise)
ns = bench.apply_config_defaults(ns)
env, lib, ff, data, pop = bench.setup_workload(ns, 0)
path = os.path.join(ROOT, "multitreegp_amd", "lib", "abrun", "libmtgp_hip_fbcount.so")
native = nat.load(path)
eng = DeviceEngine(ff, lib, 0.0, "cuda:0", native=native)
f = native.mtgp_ab_fb_count
cnt = (ctypes.c_ulonglong * 4)()
pd = torch.from_numpy(pop).cuda()
eng.evaluate(pd, data, trajectories=True)
torch.cuda.synchronize()
f(cnt)
eng.evaluate(pd, data, trajectories=True)
torch.cuda.synchronize()
f(cnt)
print(json.dumps({"chain_calls_with_fallback": cnt[0], "chain_calls": cnt[1], "single_calls_with_fallback": cnt[2],
                  "single_calls": cnt[3], "waves": (ns.pop * ns.rollouts + 63) // 64}))
