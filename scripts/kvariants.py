#!/usr/bin/env python3
"""A/B timing of kernel variants (multitreegp_amd/lib/variants/*.so) on one workload,
interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24)."""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pop", type=int, default=8192)
    ap.add_argument("--rollouts", type=int, default=32)
    ap.add_argument("--ode-steps", type=int, default=200)
    ap.add_argument("--no-traj", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--solver", default="rk4", choices=["rk4", "dopri5"])
    ap.add_argument("--obs-noise", type=float, default=0.0)
    ap.add_argument("--reflatten", action="store_true", help="flatten inside every timed evaluation (A/B of the "
                                                              "flattener; default: flatten once)")
    ap.add_argument("--order", default="orig", help="orig | pair (long with short) | sorted (host reorder)")
    ap.add_argument("--no-schedule", action="store_true", help="disable the device schedule (mtgp_schedule)")
    a = ap.parse_args()
    if a.config != "c3" and a.pop == 8192 and a.rollouts == 32:  # the config's own sizes
        a.pop, a.rollouts = {"c2": (1024, 16), "c5": (4096, 8)}[a.config]
    bargs = argparse.Namespace(pop=a.pop, rollouts=a.rollouts, ode_steps=a.ode_steps, config=a.config, solver=a.solver,
                               obs_noise=a.obs_noise)
    env, lib, ff, data, pop = bench.setup_workload(bargs, 0)
    dev = torch.device("cuda", 0)
    engines, envs = {}, {}
    for v in a.variants.split(","):
        # "name@VAR=value[@VAR2=value]": the library `name` with environment overrides (engine switches
        # such as MTGP_JIT_CHAIN=0) applied around each of its evaluations
        name, *kv = v.split("@")
        envs[v] = dict(x.split("=", 1) for x in kv)
        # variants/ is gpurun-ignored (never pushed wholesale): libraries for an A/B run are copied to lib/ab/
        path = nat.LIB_PATH
        if name != "prod":  # scripts/build_ab.py output (lib/abrun), else an older variant build
            for sub in ("abrun", "ab", "variants"):
                path = os.path.join(ROOT, "multitreegp_amd", "lib", sub, f"libmtgp_hip_{name}.so")
                if os.path.exists(path):
                    break
        engines[v] = DeviceEngine(ff, lib, 0.0, dev, native=nat.load(path))
        engines[v].native.mtgp_set_timing(1)
    pop_dev = torch.from_numpy(pop).to(dev)
    first = next(iter(engines.values()))
    first.prepare_data(data)  # (SR learns n_var from the data)
    fl = first.flatten(pop_dev)
    if a.order != "orig":
        cost = fl.plen.sum(dim=1).cpu().numpy()
        o = np.argsort(cost, kind="stable")
        if a.order == "pair":
            h = len(o) // 2
            o = np.stack([o[::-1][:h], o[:h]], axis=1).reshape(-1)
        pop_dev = torch.from_numpy(pop[o]).to(dev)
        fl = first.flatten(pop_dev)
    first.check_status(fl)
    ref = None
    times = {v: [] for v in engines}
    ktimes = {v: [] for v in engines}
    for r in range(a.rounds + 1):
        for v, eng in engines.items():
            old = {k: os.environ.get(k) for k in envs[v]}
            os.environ.update(envs[v])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            res = eng.evaluate(pop_dev, data, trajectories=not a.no_traj, flattened=None if a.reflatten else fl,
                               check=False,
                               schedule=not a.no_schedule)
            e1.record()
            for k, x in old.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x
            kms = eng.native.mtgp_last_kernel_ms()
            torch.cuda.synchronize()
            f = res["fitness"].cpu().numpy()
            if ref is None:
                ref = f
            same = bool(np.array_equal(f.view(np.uint32), ref.view(np.uint32)))
            if r > 0:
                times[v].append(e0.elapsed_time(e1))
                ktimes[v].append(kms)
            if not same:
                print(f"WARNING variant {v} fitness differs from first variant", flush=True)
    units = a.pop * a.rollouts * a.ode_steps
    for v, t in times.items():
        print(json.dumps({"tag": a.tag, "variant": v, "pop": a.pop, "R": a.rollouts, "traj": not a.no_traj,
                          "median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                          "kernel_median_ms": float(np.median(ktimes[v])), "kernel_min_ms": float(np.min(ktimes[v])),
                          "Gsteps_per_s": units / (np.median(t) / 1e3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
