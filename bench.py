#!/usr/bin/env python3
"""Benchmark: population x rollout ODE-steps/s of the fused MI355X evaluator (BASELINE.json).

Workload (N=1 line): BASELINE config C3 -- DynamicPolicy Acrobot, pop 8192 per GPU, 3 trees
per individual (2 hidden-state + 1 readout), max_nodes 64 / max_init_depth 10 (reference
sampler distribution), 32 rollouts, fixed-step RK4 h=0.05 x 200 steps, 201 save points,
trajectories written (xs, us, activities -> 28 B per unit-step, BASELINE.md byte accounting).
A "step" = one evaluate_population pass: device flatten + schedule + fused RK4 kernel +
all-gather of fitness.  Multi-GPU: one process per GPU (torchrun), weak scaling (8192
individuals per rank), the only collective is the fitness all-gather (RCCL).

Other BASELINE configs (not the driver's line; for DESIGN.md): --config c2 (Acrobot static
policy, pop 1024, 1 tree, depth <= 4, 16 rollouts) and --config c5 (64-dim SR "neural ODE":
64 trees, max_nodes 128, depth <= 16, 8 rollouts, RK4 h = 0.01 x 200, pop 4096 per GPU =
32768 over 8 GPUs).
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--pop", type=int, default=None, help="individuals per GPU (default: the config's)")
    ap.add_argument("--rollouts", type=int, default=None)
    ap.add_argument("--ode-steps", type=int, default=200)
    ap.add_argument("--no-traj", action="store_true", help="fitness-only mode (early exit allowed)")
    ap.add_argument("--solver", default="rk4", choices=["rk4", "dopri5"],
                    help="dopri5: the notebooks' Dopri5 + PIDController(rtol=atol=1e-4, dtmin=0.001), max_steps 1000 "
                         "(DynamicPolicy.ipynb:105 / StaticPolicy.ipynb:102); c2/c3 only")
    ap.add_argument("--obs-noise", type=float, default=0.0,
                    help="Acrobot observation noise (the notebooks use 0.1): in-kernel threefry normals per stage")
    ap.add_argument("--ext-ops", action="store_true",
                    help="C2/C3 node library + exp, log, sqrt, tanh, abs (p 0.1 each, like sin / cos): the JIT's "
                         "extended-operator templates under the headline workload (A/B line, not the headline)")
    ap.add_argument("--state-size", type=int, default=2,
                    help="C3 hidden-state trees (the notebook's 2); 4 .. 16 run the runtime-state-size kernels "
                         "with LDS-data JIT code (A/B line, not the headline)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1: nccl (= RCCL, the product) or gloo -- a rehearsal of the "
                         "multi-rank flow (barriers, fitness all-gather, max-over-ranks timing) with several "
                         "ranks on one GPU, which RCCL refuses; never a measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 PMC passes (HBM traffic, VALU issue) of the dominant kernel")
    ap.add_argument("--e2e-steps", type=int, default=20,
                    help="timed GeneticProgramming.evaluate_population calls from host numpy (H2D + flatten + "
                         "kernel + all-gather + D2H; SURVEY §8(d) end-to-end); 0 skips")
    a = ap.parse_args()
    apply_config_defaults(a)
    return a


# (individuals per GPU, rollouts) of each BASELINE configuration
CONFIG_DEFAULTS = {"c2": (1024, 16), "c3": (8192, 32), "c5": (4096, 8)}


def apply_config_defaults(a):
    """--pop / --rollouts default to the configuration's own sizes (bench.py and scripts/kprof.py)"""
    pop, R = CONFIG_DEFAULTS[a.config]
    a.pop = a.pop or pop
    a.rollouts = a.rollouts or R
    return a


def _cached_population(name, make):
    """Sampled populations are cached under TMPDIR (the C5 population takes ~15 s to sample).
    The sampler is vectorised (sampling.sample_trees_batch), so no worker pool is ever forked:
    bench and scripts/kprof.py run under rocprofv3, whose signal handlers a forked pool inherits."""
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mtgp_pop_v2_{name}.npy")
    if os.path.exists(cache):
        return np.load(cache)
    pop = make()
    os.makedirs(os.path.dirname(cache), exist_ok=True)
    np.save(cache + ".tmp.npy", pop)
    os.replace(cache + ".tmp.npy", cache)
    return pop


def setup_workload(args, rank):
    import multitreegp_amd as mt
    from multitreegp_amd.sampling import sample_population
    if args.config == "c5":
        nv = 64
        env = mt.LinearSystem(nv)
        lib = mt.NodeLibrary([("+", None, 2, 0.5), ("-", None, 2, 0.1), ("*", None, 2, 0.5), ("/", None, 2, 0.1)],
                             [[f"x{i}" for i in range(nv)]], [nv])
        ff = mt.SREvaluator(solver=mt.RK4(), dt0=0.01)
        x0 = env.sample_init_states(args.rollouts, np.random.default_rng(1))
        ts = (np.arange(args.ode_steps + 1, dtype=np.float32) * np.float32(0.01)).astype(np.float32)
        data = (x0, ts, mt.ground_truth(env, x0, ts), np.zeros((args.rollouts, 2), np.uint32))
        pop = _cached_population(f"c5_{args.pop}_r{rank}",
                                 lambda: sample_population(2000 + rank, lib, args.pop, 1, max_init_depth=16,
                                                           max_nodes=128)[0])
        return env, lib, ff, data, pop
    env = mt.Acrobot(0.0, getattr(args, "obs_noise", 0.0))
    ops = [("+", None, 2, 0.5), ("-", None, 2, 0.1), ("*", None, 2, 0.5), ("sin", None, 1, 0.1),
           ("cos", None, 1, 0.1)]
    ext = getattr(args, "ext_ops", False)
    if ext:
        ops = ops + [(name, None, 1, 0.1) for name in ("exp", "log", "sqrt", "tanh", "abs")]
    tag = "_ext" if ext else ""
    if args.solver == "dopri5":
        solver = dict(solver=mt.Dopri5(), stepsize_controller=mt.PIDController(rtol=1e-4, atol=1e-4, dtmin=0.001))
    else:
        solver = dict(solver=mt.RK4())
    if args.config == "c2":
        lib = mt.NodeLibrary(ops, [["y1", "y2", "y3", "y4"]], [1])
        ff = mt.FeedforwardEvaluator(env, 0.05, max_steps=1000, **solver)
        data = mt.control_data(env, args.rollouts, 0.05, None, seed=1, n_steps=args.ode_steps)
        pop = _cached_population(f"c2{tag}_{args.pop}_r{rank}",
                                 lambda: sample_population(3000 + rank, lib, args.pop, 1, max_init_depth=4,
                                                           max_nodes=30)[0])
        return env, lib, ff, data, pop
    ss = getattr(args, "state_size", 2)
    acts = [f"a{i + 1}" for i in range(ss)]
    lib = mt.NodeLibrary(ops, [["y1", "y2", "y3", "y4"] + acts + ["u"], acts], [ss, 1])
    ff = mt.DynamicEvaluator(env, ss, 0.05, max_steps=1000, **solver)
    data = mt.control_data(env, args.rollouts, 0.05, None, seed=1, n_steps=args.ode_steps)
    tag += "" if ss == 2 else f"_ss{ss}"
    pop = _cached_population(f"c3{tag}_{args.pop}_r{rank}",
                             lambda: sample_population(1000 + rank, lib, args.pop, 1, max_init_depth=10,
                                                       max_nodes=64)[0])
    return env, lib, ff, data, pop


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_passes(args, kernel_substr):
    """Live rocprofv3 PMC of the dominant kernel on this same workload (rank 0, N = 1), one
    counter group per pass as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes:
      FETCH_SIZE (KiB, x2: gfx950 counts half of a wide coalesced read) | WRITE_SIZE (KiB) |
      SQ_INSTS_VALU, SQ_WAVES, GRBM_GUI_ACTIVE (sum over 8 XCDs -> / 8 = kernel cycles).
    Each pass is a child process (scripts/kprof.py, one evaluation) under a hard time limit;
    any failure leaves the field null.  -> dict or None"""
    import shutil
    import subprocess
    import tempfile
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from pmc_summary import collect
    cmd_tail = ["--", sys.executable, os.path.join(ROOT, "scripts", "kprof.py"), "--iters", "1", "--config",
                args.config, "--pop", str(args.pop), "--rollouts", str(args.rollouts), "--solver", args.solver,
                "--obs-noise", str(args.obs_noise), "--ode-steps", str(args.ode_steps),
                "--state-size", str(args.state_size)] + \
        (["--no-traj"] if args.no_traj else [])
    out = {}
    with tempfile.TemporaryDirectory(prefix="mtgp_pmc_") as d:
        for i, counters in enumerate((["FETCH_SIZE"], ["WRITE_SIZE"], ["SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE"])):
            sub = os.path.join(d, f"p{i}")
            cmd = ["timeout", "-s", "KILL", "90", rp, "--pmc", *counters, "-d", sub, "-o", "p",
                   "--output-format", "csv"] + cmd_tail
            try:
                r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=120)
            except Exception as e:  # the pass is reported (stderr), the field stays null
                print(f"bench: PMC pass {counters} failed: {e!r}", file=sys.stderr)
                return None
            if r.returncode != 0:
                tail = r.stdout.decode(errors="replace")[-1500:]
                print(f"bench: PMC pass {counters} exited {r.returncode}:\n{tail}", file=sys.stderr)
                return None
            got = collect(sub, kernel_substr)
            if not got.get("dispatches"):
                print(f"bench: PMC pass {counters}: no dispatch of {kernel_substr!r} in the profile", file=sys.stderr)
                return None
            out.update(got)
    need = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")
    return out if all(k in out for k in need) else None


def cpu_baseline(args, lib, ff, data, pop, steps=None):
    """Time the C oracle (OpenMP port of the reference path) on a bounded sample."""
    from oracle import oracle as orc
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import oracle_model, oracle_rollouts
    d = ff.prepare(data)
    model = oracle_model(ff, d)
    ro = oracle_rollouts(d)
    # threads: OpenMP's team size, OMP_NUM_THREADS when set -- the GPU pool sets it to the job's CPU
    # share (16 per GPU) and asks jobs not to exceed it -- else the process's CPU affinity;
    # os.cpu_count() is the whole host
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", affinity))
    threads = omp
    n = 16
    while True:
        t0 = time.perf_counter()
        orc.evaluate(model, pop[:n], lib, ro, trajectories=True)
        dt = time.perf_counter() - t0
        if dt > args.cpu_seconds / 4 or n >= pop.shape[0]:
            break
        n = min(pop.shape[0], int(n * max(2.0, args.cpu_seconds / 4 / max(dt, 1e-3))))
    if steps is not None:  # Dopri5: the oracle takes exactly the GPU's (bit-identical) steps
        units = int(steps[:n].sum())
        what = f"{units} Dopri5 step attempts"
    else:
        units = n * d["R"] * d["n_steps"]
        what = f"{d['n_steps']} RK4 steps"
    why = ("the CPU affinity of this process" if "OMP_NUM_THREADS" not in os.environ else
           f"OMP_NUM_THREADS={omp}, set by the GPU pool as this job's CPU share (process affinity {affinity} of "
           f"{os.cpu_count()} host CPUs)")
    return {"value": units / dt, "unit": "ODE-steps/s", "cores": threads, "kind": "port",
            "cores_affinity": affinity, "cores_host": os.cpu_count(), "cores_why": why,
            "cpu_model": cpu_model(),
            "sample": f"{n} individuals x {d['R']} rollouts x {what} of the "
                      f"{args.config.upper()} workload, "
                      f"trajectories on, oracle/mtgp_oracle.c row-order interpreter, {threads} OpenMP threads "
                      f"of {os.cpu_count()} on {cpu_model()}, {dt:.2f} s"}


def host_evolve_threads() -> str:
    """The thread count libmtgp_host.so's evolve uses (mtgp_evolve.cpp host_threads): MTGP_HOST_THREADS,
    else OMP_NUM_THREADS (the pool's CPU share), else the affinity size, at most 64."""
    for var in ("MTGP_HOST_THREADS", "OMP_NUM_THREADS"):
        if os.environ.get(var):
            n = max(1, int(os.environ[var]))
            return f"{n if var == 'MTGP_HOST_THREADS' else min(n, 64)} ({var})"
    return f"{min(len(os.sched_getaffinity(0)), 64)} (affinity)"


def reduce_scalar(x: float, op, dev) -> float:
    """all_reduce of one float64 over the ranks: a device tensor under RCCL, a host one under gloo"""
    import torch
    import torch.distributed as dist
    on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=op)
    return float(t.item())


def end_to_end(args, ff, lib, data, pop, ws, rank, dev):
    """SURVEY §8(d) end-to-end rate: GeneticProgramming.evaluate_population (gp.py:403-433) on a
    host numpy population of P*ws individuals, as the user's loop calls it -- H2D copy of this
    rank's block, device flatten + schedule + JIT + fused kernel, fitness all-gather, D2H, argmin
    and best-so-far bookkeeping.  Each rank's block is its own population (the array is the rank's
    population tiled ws times), so the work per rank equals the kernel-resident line's."""
    import torch
    import torch.distributed as dist
    from multitreegp_amd.genetic_programming import GeneticProgramming
    P = pop.shape[0]
    full = np.ascontiguousarray(np.concatenate([pop] * ws)[None]) if ws > 1 else pop[None]
    gp = GeneticProgramming(1, P * ws, ff, lib.operator_list, lib.variable_list, lib.layer_sizes,
                            max_nodes=pop.shape[2], migration_percentage=0.0, elite_percentage=0.0, device=dev,
                            verbose=False)
    for _ in range(3):
        gp.evaluate_population(full, data)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.e2e_steps):
        fit, _ = gp.evaluate_population(full, data)  # returns host numpy: synchronous per call
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        el = reduce_scalar(el, dist.ReduceOp.MAX, dev)
    # the host half of a generation: GeneticProgramming.evolve (gp.py:475-497) on the same
    # population (native host library, include/mtgp_host.h)
    ev = []
    for i in range(4):
        t1 = time.perf_counter()
        gp.evolve(full, fit, 1000 + i)
        ev.append((time.perf_counter() - t1) * 1e3)
    return el * 1e3 / args.e2e_steps, fit, float(np.median(ev[1:]))


def build_record() -> dict:
    """Which kernel library this line measured: the in-tree libmtgp_hip.so, its size / mtime / hash
    prefix, and whether __graft_entry__.build() would have recompiled it (a source newer than the
    library) -- i.e. whether the line ran the shipped prebuilt library or a fresh build of the
    sources."""
    import hashlib
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import __graft_entry__ as ge
    from multitreegp_amd import _native as nat
    path = nat.LIB_PATH
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    st = os.stat(path)
    newest = max(ge.HIP_SOURCES, key=os.path.getmtime)
    embedded = nat.build_info().get("sources_sha256")
    tree = ge.sources_hash()
    return {"lib": os.path.relpath(path, os.path.dirname(os.path.abspath(__file__))), "bytes": st.st_size,
            "mtime": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(st.st_mtime)), "sha256_16": h.hexdigest()[:16],
            "sources_sha256_embedded": embedded, "sources_sha256_tree": tree,
            "sources_hash_match": embedded == tree,
            "stale_vs_sources": bool(ge._stale(path, ge.HIP_SOURCES)),
            "newest_source": os.path.basename(newest),
            "newest_source_mtime": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(os.path.getmtime(newest))),
            "note": "sources_hash_match: the library's embedded SHA-256 of its sources + flags (mtgp_build_info) "
                    "equals the hash of this tree's HIP_SOURCES"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rccl = args.dist_backend == "nccl"
    # (a gloo rehearsal may run more ranks than the box has GPUs: they share the devices)
    dev = torch.device("cuda", local if rccl else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if ws > 1:
        if rccl:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from multitreegp_amd import _native as nat
    from multitreegp_amd import distributed as mdist
    from multitreegp_amd.engine import DeviceEngine

    env, lib, ff, data, pop = setup_workload(args, rank)
    P = pop.shape[0]
    eng = DeviceEngine(ff, lib, 0.0, dev)
    pop_dev = torch.from_numpy(pop).to(dev)
    traj = not args.no_traj
    adaptive = args.solver == "dopri5"
    nat.load().mtgp_set_timing(1)

    def step():
        res = eng.evaluate(pop_dev, data, trajectories=traj, check=False, step_counts=adaptive)
        fit = mdist.gather_fitness(res["fitness"], P * ws, P, check=False) if ws > 1 else res["fitness"]
        return res, fit

    res, _ = step()
    eng.check_status(res["_flat"])
    for _ in range(args.warmup):
        step()

    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):  # no host synchronisation inside: the queue stays full
        res, fit = step()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        elapsed = reduce_scalar(elapsed, dist.ReduceOp.MAX, dev)
    ms_per_step = elapsed * 1e3 / args.steps
    n_hist = min(args.steps, 1024)  # the evaluator launches' hipEvent durations (ring of 1024), read after the run
    hist = (ctypes.c_float * n_hist)()
    got = nat.load().mtgp_kernel_ms_history(hist, n_hist)
    if got != n_hist:
        raise RuntimeError(f"kernel timing history returned {got} of {n_hist} launches")
    kernel_ms = list(hist)

    d = eng.prepare_data(data)
    R, S, n_steps = d["R"], d["n_save"], d["n_steps"]
    steps_host = res["steps"].cpu().numpy() if adaptive else None
    if adaptive:  # step attempts of this rank; every rank evaluates its own shard of the same size
        units_per_step = float(int(steps_host.sum()))
        if ws > 1:
            units_per_step = reduce_scalar(units_per_step, dist.ReduceOp.SUM, dev)
    else:
        units_per_step = P * R * n_steps * ws
    value = units_per_step / (ms_per_step / 1e3)

    # roofline of the dominant kernel (the fused RK4 evaluator): algorithmic bytes per launch
    plen = res["_flat"].plen
    prog_bytes = int(plen.sum().item()) * 8 + plen.numel() * 4
    traj_bytes = sum(res[k].numel() * 4 for k in ("xs", "ys", "us", "acts") if k in res)  # S*P*R*(4+4+1+2)*4
    io_bytes = sum(int(np.asarray(d[k]).nbytes) for k in ("x0", "params", "targets", "ts", "ys_true", "obs_keys",
                                                           "obs_w")
                   if d.get(k) is not None) + P * 4 * 2  # rollout data + nodes in + fitness out
    alg_bytes = traj_bytes + prog_bytes + io_bytes
    # SURVEY.md section 8(d)'s accounting: the same without the observations ys (28.3 B per
    # unit-step at C3 instead of 44.2); evaluate_candidate returns ys too (dyn.py:99, 105), so the
    # line's frac keeps them and both are reported
    alg_bytes_s8d = alg_bytes - (res["ys"].numel() * 4 if "ys" in res else 0)
    kmean = float(np.mean(kernel_ms))
    achieved = alg_bytes_s8d / (kmean / 1e3) / 1e9  # SURVEY §8(d) bytes per launch / kernel time
    achieved_ys = alg_bytes / (kmean / 1e3) / 1e9
    traffic = valu = None
    pmc = None
    if rank == 0 and ws == 1 and not args.no_pmc:
        kname = {"c3": "k_ctl_dynamic", "c2": "k_ctl_static", "c5": "k_sr_wide"}[args.config]
        if adaptive:
            kname = "k_ctl_dopri5"
        pmc = pmc_passes(args, kname)
    if pmc is not None:
        # HBM bytes per launch (FETCH x2 gfx950 correction, KiB -> B) and the VALU issue fraction:
        # wave64 VALU = 2 cycles on a SIMD-32 -> at most 0.5 wave-instructions per SIMD-cycle
        traffic = pmc["FETCH_SIZE"] * 1024 * 2 + pmc["WRITE_SIZE"] * 1024
        kcycles = pmc["GRBM_GUI_ACTIVE"] / 8.0
        valu = pmc["SQ_INSTS_VALU"] / (1024 * 0.5 * kcycles) if kcycles > 0 else None
    dt0 = {"c3": 0.05, "c2": 0.05, "c5": 0.01}[args.config]
    solver_txt = ("Dopri5 PID rtol=atol=1e-4 dtmin=0.001 dt0=0.05, max_steps 1000" if adaptive else
                  f"RK4 + diffrax ConstantStepSize dt0={dt0} ({n_steps} accumulated f32 steps), SaveAt(ts) by dense output")
    workloads = {
        "c3": "C3 DynamicPolicy Acrobot: pop %d/GPU x %d rollouts, %d trees, max_nodes 64, depth<=10, %s, S=%d"
              % (P, R, args.state_size + 1, solver_txt, S) + ("" if args.state_size == 2 else
                                                                f", state_size {args.state_size} (runtime-state-size interpreter kernel)"),
        "c2": "C2 StaticPolicy Acrobot: pop %d/GPU x %d rollouts, 1 tree, max_nodes 30, depth<=4, %s, S=%d"
              % (P, R, solver_txt, S),
        "c5": "C5 64-dim SR (neural-ODE style): pop %d/GPU x %d rollouts, 64 trees, max_nodes 128, depth<=16, "
              "%s, S=%d, MSE vs a stable linear system" % (P, R, solver_txt, S),
    }
    data_desc = {
        "c3": "synthetic: reference-distribution random trees (numpy PCG64), x0 ~ U(-0.1,0.1)^4",
        "c2": "synthetic: reference-distribution random trees (numpy PCG64), x0 ~ U(-0.1,0.1)^4",
        "c5": "synthetic: reference-distribution random trees (numpy PCG64), x0 ~ N(0,1)^64, "
              "target = fine RK4 of a random stable 64x64 linear system",
    }

    out = {
        "metric": "population x rollout ODE-steps/sec (fixed-step RK4, diffrax ConstantStepSize)",
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
        "data": data_desc[args.config],
        "config": {"workload": workloads[args.config] + (", trajectories on" if traj else ", fitness only")
                   + (f", obs_noise {args.obs_noise} (threefry in-kernel)" if args.obs_noise else "")
                   + (", node library + exp log sqrt tanh abs (JIT subroutines)" if args.ext_ops else ""),
                   "pop_per_gpu": P, "rollouts": R, "ode_steps": n_steps, "trajectories": traj,
                   "state_size": args.state_size if args.config == "c3" else None,
                   "parallelism": f"population-sharded dp{ws}"},
        "kernel_ms": kmean,
        # The kernel is bound by VALU issue / dependent-instruction latency, not by HBM (DESIGN.md
        # "Roofline"): frac is the HBM fraction on SURVEY §8(d)'s bytes (alg_bytes_s8d / kernel_ms /
        # 8 TB/s, reproducible from profiles/ with the rocprof average), valu_frac the primary figure
        # (VALU wave-instructions issued / the SIMDs' issue capacity over the kernel's cycles)
        "roofline": {"bound": "valu-issue", "primary": "valu_frac", "valu_frac": valu,
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                     "traffic_over_alg_ys": None if traffic is None else traffic / alg_bytes,
                     "alg_bytes_s8d": alg_bytes_s8d,
                     "alg_bytes_ys_inclusive": alg_bytes,
                     "frac_ys_inclusive": achieved_ys / PEAK_HBM_GBS,
                     "pmc": None if pmc is None else {k: pmc[k] for k in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU",
                                                                           "SQ_WAVES", "GRBM_GUI_ACTIVE")
                                                      if k in pmc}},
    }
    out["build"] = build_record()
    if ws > 1 and not rccl:
        out["rehearsal"] = "gloo process group, ranks sharing GPUs: a check of the multi-rank flow, not a measurement"
    if adaptive:
        out["metric"] = ("population x rollout ODE-steps/sec (adaptive Dopri5 + PIDController; a step = one step "
                         "attempt, rejected ones included)")
        out["config"]["ode_steps"] = units_per_step / (P * R * ws)  # mean attempts per rollout
        out["config"]["solver"] = "dopri5"
    if args.e2e_steps > 0:
        e2e_ms, e2e_fit, evolve_ms = end_to_end(args, ff, lib, data, pop, ws, rank, dev)
        ok = bool(np.array_equal(e2e_fit.reshape(-1)[:P].view(np.uint32), res["fitness"].cpu().numpy().view(np.uint32)))
        units = (units_per_step if not adaptive else float("nan"))
        out["end_to_end"] = {
            "what": "GeneticProgramming.evaluate_population from host numpy: H2D + flatten + schedule + JIT + "
                    "kernel + fitness all-gather + D2H + best tracking (SURVEY §8(d))",
            "ms_per_step": e2e_ms, "value": units / (e2e_ms / 1e3) if not adaptive else None,
            "unit": "ODE-steps/s", "steps": args.e2e_steps, "trajectories": False,
            "fitness_equal_to_kernel_line": ok,
            "h2d_bytes_per_rank": int(pop.nbytes),
            "host_evolve_ms": evolve_ms,
            "host_evolve_what": f"GeneticProgramming.evolve of the {P * ws}-candidate population (native host "
                                f"library on {host_evolve_threads()} threads), median of 3"}
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:  # (the contract: rank 0 at N = 1 only)
        out["cpu_baseline"] = cpu_baseline(args, lib, ff, data, pop, steps_host)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
