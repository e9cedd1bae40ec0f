set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dispatch_cost.py --ks 0,4,16 > gpurun_out/dc_wave.log 2>&1 && \
timeout -k 10 300 python -u - > gpurun_out/ab_wave.log 2>&1 <<'PY'
import sys, os, argparse, json, numpy as np, torch
sys.path.insert(0, os.getcwd())
import bench
from multitreegp_amd.engine import DeviceEngine
env, lib, ff, data, pop = bench.setup_workload(argparse.Namespace(pop=8192, rollouts=32, ode_steps=200, config="c3"), 0)
pd = torch.from_numpy(pop).cuda()
engs = {"jit": DeviceEngine(ff, lib, 0.0, "cuda:0", jit=True), "interp": DeviceEngine(ff, lib, 0.0, "cuda:0", jit=False)}
fls = {k: e.flatten(pd) for k, e in engs.items()}
times = {k: [] for k in engs}
for r in range(6):
    for k, e in engs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = e.evaluate(pd, data, trajectories=True, flattened=fls[k], check=False)  # builds JIT once
        torch.cuda.synchronize()
        e0.record()
        e.evaluate(pd, data, trajectories=True, flattened=fls[k], check=False)
        e1.record(); torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1))
print(json.dumps({k: sorted(v) for k, v in times.items()}), "jit_ok", DeviceEngine.jit_ok(fls["jit"]))
PY
