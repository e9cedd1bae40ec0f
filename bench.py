#!/usr/bin/env python3
"""Benchmark: population x rollout ODE-steps/s of the fused MI355X evaluator (BASELINE.json).

Workload (N=1 line): BASELINE config C3 -- DynamicPolicy Acrobot, pop 8192 per GPU, 3 trees
per individual (2 hidden-state + 1 readout), max_nodes 64 / max_init_depth 10 (reference
sampler distribution), 32 rollouts, fixed-step RK4 h=0.05 x 200 steps, 201 save points,
trajectories written (xs, us, activities -> 28 B per unit-step, BASELINE.md byte accounting).
A "step" = one evaluate_population pass: device flatten + fused RK4 kernel + all-gather of
fitness.  Multi-GPU: one process per GPU (torchrun), weak scaling (8192 individuals per rank),
the only collective is the fitness all-gather (RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pop", type=int, default=8192, help="individuals per GPU")
    ap.add_argument("--rollouts", type=int, default=32)
    ap.add_argument("--ode-steps", type=int, default=200)
    ap.add_argument("--no-traj", action="store_true", help="fitness-only mode (early exit allowed)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def setup_workload(args, rank):
    import multitreegp_amd as mt
    from multitreegp_amd.sampling import sample_population
    env = mt.Acrobot(0.0, 0.0)
    ops = [("+", None, 2, 0.5), ("-", None, 2, 0.1), ("*", None, 2, 0.5), ("sin", None, 1, 0.1),
           ("cos", None, 1, 0.1)]
    lib = mt.NodeLibrary(ops, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1])
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4(), max_steps=1000)
    data = mt.control_data(env, args.rollouts, 0.05, None, seed=1, n_steps=args.ode_steps)
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mtgp_pop_c3_{args.pop}_r{rank}.npy")
    if os.path.exists(cache):
        pop = np.load(cache)
    else:
        pop = sample_population(1000 + rank, lib, args.pop, 1, max_init_depth=10, max_nodes=64)[0]
        os.makedirs(os.path.dirname(cache), exist_ok=True)
        np.save(cache, pop)
    return env, lib, ff, data, pop


def cpu_baseline(args, lib, ff, data, pop):
    """Time the C oracle (OpenMP port of the reference path) on a bounded sample."""
    from oracle import oracle as orc
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import oracle_model, oracle_rollouts
    d = ff.prepare(data)
    model = oracle_model(ff, d)
    ro = oracle_rollouts(d)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n = 16
    while True:
        t0 = time.perf_counter()
        orc.evaluate(model, pop[:n], lib, ro, trajectories=True)
        dt = time.perf_counter() - t0
        if dt > args.cpu_seconds / 4 or n >= pop.shape[0]:
            break
        n = min(pop.shape[0], int(n * max(2.0, args.cpu_seconds / 4 / max(dt, 1e-3))))
    units = n * d["R"] * d["n_steps"]
    return {"value": units / dt, "unit": "ODE-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} individuals x {d['R']} rollouts x {d['n_steps']} RK4 steps of the C3 workload, "
                      f"trajectories on, oracle/mtgp_oracle.c row-order interpreter, {threads} OpenMP threads, "
                      f"{dt:.2f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from multitreegp_amd import _native as nat
    from multitreegp_amd import distributed as mdist
    from multitreegp_amd.engine import DeviceEngine

    env, lib, ff, data, pop = setup_workload(args, rank)
    P = pop.shape[0]
    eng = DeviceEngine(ff, lib, 0.0, dev)
    pop_dev = torch.from_numpy(pop).to(dev)
    traj = not args.no_traj
    nat.load().mtgp_set_timing(1)

    def step():
        res = eng.evaluate(pop_dev, data, trajectories=traj, check=False)
        fit = mdist.gather_fitness(res["fitness"], P * ws, P) if ws > 1 else res["fitness"]
        return res, fit

    res, _ = step()
    eng.check_status(res["_flat"])
    for _ in range(args.warmup):
        step()

    kernel_ms = []
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, fit = step()
        kernel_ms.append(nat.load().mtgp_last_kernel_ms())  # syncs on the kernel's end event
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps

    d = eng.prepare_data(data)
    R, S, n_steps = d["R"], d["n_save"], d["n_steps"]
    units_per_step = P * R * n_steps * ws
    value = units_per_step / (ms_per_step / 1e3)

    # roofline of the dominant kernel (the fused RK4 evaluator): algorithmic bytes per launch
    plen = res["_flat"].plen
    prog_bytes = int(plen.sum().item()) * 8 + plen.numel() * 4
    traj_bytes = (S * P * R * (4 + 1 + 2) * 4) if traj else 0
    io_bytes = R * (4 + 4) * 4 + S * 4 + P * 4 + P * 4
    alg_bytes = traj_bytes + prog_bytes + io_bytes
    kmean = float(np.mean(kernel_ms))
    achieved = alg_bytes / (kmean / 1e3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "population x rollout ODE-steps/sec (C3 DynamicPolicy Acrobot, fixed-step RK4)",
        "value": value,
        "unit": "ODE-steps/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: reference-distribution random trees (numpy PCG64), x0 ~ U(-0.1,0.1)^4",
        "config": {"workload": "C3 DynamicPolicy Acrobot: pop 8192/GPU x 32 rollouts, 3 trees, max_nodes 64, "
                               "depth<=10, RK4 h=0.05 x 200, S=201, trajectories on" if traj else
                               "C3 fitness-only", "pop_per_gpu": P, "rollouts": R, "ode_steps": n_steps,
                   "trajectories": traj, "parallelism": f"population-sharded dp{ws}"},
        "kernel_ms": kmean,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes},
    }
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, lib, ff, data, pop)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
