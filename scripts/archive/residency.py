#!/usr/bin/env python3
"""Wave residency study (diagnostic variant MTGP_AB_TIMING (removed in round 4)): per-wave start/end real-time
stamps and HW_ID of the C3 evaluation, to see whether all waves are co-resident."""
import argparse, ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multitreegp_amd import _native as nat  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--jit", type=int, default=1)
a = ap.parse_args()
path = os.path.join(ROOT, "multitreegp_amd", "lib", "variants", "libmtgp_hip_timing.so")
lib = nat.load(path)
lib.mtgp_debug_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
env, lib_, ff, data, pop = bench.setup_workload(argparse.Namespace(pop=8192, rollouts=32, ode_steps=200, config="c3"), 0)
eng = DeviceEngine(ff, lib_, 0.0, "cuda:0", native=lib, jit=bool(a.jit))
pd = torch.from_numpy(pop).cuda()
fl = eng.flatten(pd)
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.evaluate(pd, data, trajectories=True, flattened=fl, check=False)
    e1.record()
    torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
nw = 4096
buf = np.zeros(nw * 4, np.uint64)
lib.mtgp_debug_probe(buf.ctypes.data, buf.size)
fallbacks = buf.reshape(nw, 4)[:, 3].astype(np.int64)
b = buf.reshape(nw, 4)
st, en, hw = b[:, 0].astype(np.int64), b[:, 1].astype(np.int64), b[:, 2]
t0 = st.min()
st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0  # s_memrealtime: 100 MHz
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
life = en_us - st_us
print(json.dumps({"jit": a.jit, "kernel_ms": ms, "start_us_pct": np.percentile(st_us, [0, 50, 90, 99, 100]).round(1).tolist(),
                  "end_us_pct": np.percentile(en_us, [0, 50, 90, 100]).round(1).tolist(),
                  "life_us_pct": np.percentile(life, [0, 50, 100]).round(1).tolist(),
                  "late_starters": int((st_us > 0.25 * en_us.max()).sum()),
                  "fallback_waves": int((fallbacks > 0).sum()), "fallbacks_max": int(fallbacks.max()),
                  "life_of_fallback_waves_us": np.percentile(life[fallbacks > 0], [0, 50, 100]).round(1).tolist()
                  if (fallbacks > 0).any() else None,
                  "life_no_fallback_us_max": float(life[fallbacks == 0].max()),
                  "distinct_cu_se_simd": int(len(set(zip(cu.tolist(), se.tolist(), simd.tolist()))))}))
