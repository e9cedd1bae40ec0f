#!/usr/bin/env python3
"""Diagnostic (never the product): per-wave residency of the C3 kernel from the MTGP_AB_WAVETIME
build -- each k_ctl_dynamic wave's start / end clock (s_memrealtime, 100 MHz, device-wide) and HW_ID / XCC_ID.

    MTGP_LIB=multitreegp_amd/lib/dbg/libmtgp_hip_wt.so python scripts/wave_times.py

Prints one JSON line: the kernel span (first start to last end, clock ticks), wave durations
(mean / p50 / p90 / max, relative to the mean), the residency = sum of wave durations / (waves
per SIMD x SIMDs x span), and per-SIMD busy spans -- how much of the kernel is tail (SIMDs whose
waves have all finished while others still run)."""
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
ap.add_argument("--config", default="c3", choices=["c3"])
ap.add_argument("--no-schedule", action="store_true")
ap.add_argument("--save", default="", help="write the raw per-wave data (.npz)")
a = ap.parse_args()
assert nat.LIB_PATH.endswith("libmtgp_hip_wt.so"), "run with MTGP_LIB=<the MTGP_AB_WAVETIME build>"
args = bench.apply_config_defaults(argparse.Namespace(pop=None, rollouts=None, ode_steps=200, config=a.config,
                                                      solver="rk4", obs_noise=0.0))
env, lib, ff, data, pop = bench.setup_workload(args, 0)
lib_native = nat.load()
eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
pd = torch.from_numpy(pop).cuda()
for i in range(3):
    eng.evaluate(pd, data, trajectories=True, check=i == 0, schedule=not a.no_schedule)
torch.cuda.synchronize()
n = 1 << 15
t = (ctypes.c_ulonglong * (2 * n))()
hw = (ctypes.c_uint * (2 * n))()
fn = lib_native.mtgp_ab_wave_times
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
got = fn(ctypes.addressof(t), ctypes.addressof(hw), n)
T = np.frombuffer(t, np.uint64).reshape(-1, 2)[:got].astype(np.int64)
H = np.frombuffer(hw, np.uint32).reshape(-1, 2)[:got]
live = T[:, 1] > T[:, 0]
T, H = T[live], H[live]
start, end = T[:, 0], T[:, 1]
span = int(end.max() - start.min())
dur = (end - start).astype(np.float64)
hwid = H[:, 0]
simd = (hwid >> 4) & 3
cu = (hwid >> 8) & 15
sh = (hwid >> 12) & 1
se = (hwid >> 13) & 7
xcc = H[:, 1] & 0xF
key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
simds = np.unique(key)
busy = []
for k in simds:
    m = key == k
    busy.append(int(end[m].max() - start[m].min()))
busy = np.array(busy, np.float64)
per_simd = np.array([np.sum(key == k) for k in simds])
out = {"waves": int(live.sum()), "simds": int(len(simds)), "waves_per_simd": [int(per_simd.min()), int(per_simd.max())],
       "span_ticks": span, "wave_ticks_mean": float(dur.mean()), "wave_rel_p50": float(np.median(dur) / dur.mean()),
       "wave_rel_p90": float(np.percentile(dur, 90) / dur.mean()), "wave_rel_max": float(dur.max() / dur.mean()),
       "wave_rel_min": float(dur.min() / dur.mean()),
       "residency": float(dur.sum() / (per_simd.max() * len(simds) * span)),
       "simd_busy_rel_mean": float(busy.mean() / span), "simd_busy_rel_p10": float(np.percentile(busy, 10) / span),
       "start_spread_rel": float((start.max() - start.min()) / span), "schedule": not a.no_schedule}
print(json.dumps(out))
if a.save:  # raw per-wave data + the schedule's inputs, for offline analysis
    res = eng.evaluate(pd, data, trajectories=True, check=False, schedule=not a.no_schedule)
    torch.cuda.synchronize()
    fl = res["_flat"]
    got2 = fn(ctypes.addressof(t), ctypes.addressof(hw), n)
    T2 = np.frombuffer(t, np.uint64).reshape(-1, 2)[:got2].astype(np.int64)
    H2 = np.frombuffer(hw, np.uint32).reshape(-1, 2)[:got2]
    cost = eng.schedule_cost(fl).cpu().numpy()
    order = fl.order.cpu().numpy() if fl.order is not None else np.arange(pop.shape[0], dtype=np.int32)
    np.savez(a.save, t=T2, hw=H2, cost=cost, order=order, plen=fl.plen.cpu().numpy(),
             weights=np.array(eng.schedule_weights()))
