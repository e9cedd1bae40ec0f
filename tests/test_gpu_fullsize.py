"""Parity at the BASELINE configurations' own sizes (VERDICT r1 "what's weak" 2).

The bench runs C2 / C3 / C5 at full size; these tests run the same workloads (bench.py's
setup_workload: same populations, data and solver) through the HIP path and compare a
deterministic sample of individuals bit for bit with the CPU oracle -- fitness, per-rollout
fitness and the full trajectories.  The sample covers the first and the last wave of the
evaluation schedule, both individuals of paired waves, random picks, and every individual
with an event-terminated (inf-filled) rollout, up to the sample size.  The oracle evaluates
each individual independently, so evaluating only the sample gives the same bits.
"""
import argparse
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from helpers import bits_equal, mismatch_report, oracle_model, oracle_rollouts  # noqa: E402

pytestmark = pytest.mark.gpu


def _workload(cfg):
    import bench
    pop, R = {"c2": (1024, 16), "c3": (8192, 32), "c5": (4096, 8)}[cfg]
    a = argparse.Namespace(config=cfg, pop=pop, rollouts=R, ode_steps=200, solver="rk4", obs_noise=0.0)
    return bench.setup_workload(a, 0)


def _sample(order, inf_ind, P, n, seed=0):
    """slot order -> individual sample: first/last waves, paired waves, event-terminated, random"""
    order = np.asarray(order)
    pick = list(order[:8]) + list(order[-8:])            # first and last waves (G = 2 or 4 per wave)
    mid = len(order) // 2 & ~7
    pick += list(order[mid:mid + 8])                      # whole middle waves: both schedule halves
    pick += list(inf_ind[: n // 4])                       # event-terminated rollouts
    rng = np.random.default_rng(seed)
    pick += list(rng.choice(P, size=n, replace=False))
    out = []
    for i in pick:
        if int(i) not in out:
            out.append(int(i))
    return np.array(out[:n])


def _run(cfg, n_sample):
    import torch
    from multitreegp_amd.engine import DeviceEngine
    from oracle import oracle as orc
    env, lib, ff, data, pop = _workload(cfg)
    P = pop.shape[0]
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    res = eng.evaluate(torch.from_numpy(pop).cuda(), data, trajectories=True, rollout_fitness=True)
    torch.cuda.synchronize()
    d = eng.prepare_data(data)
    R, S = d["R"], d["n_save"]
    fl = res["_flat"]
    order = fl.order.cpu().numpy() if fl.order is not None else np.arange(P)
    xs = res["xs"]
    inf_ind = torch.isinf(xs.reshape(S, xs.shape[1], P, R)).any(3).any(1).any(0).nonzero().flatten().cpu().numpy()
    idx = _sample(order, inf_ind, P, n_sample)
    it = torch.from_numpy(idx).cuda()
    got = {"fitness": res["fitness"][it].cpu().numpy(), "rollout_fitness": res["rollout_fitness"][it].cpu().numpy()}
    for k in ("xs", "ys", "us", "acts"):
        if k in res:
            t = res[k]
            got[k] = t.reshape(S, t.shape[1], P, R)[:, :, it, :].permute(2, 3, 0, 1).cpu().numpy()
    ref = orc.evaluate(oracle_model(ff, d), pop[idx], lib, oracle_rollouts(d), trajectories=True)
    for k, v in got.items():
        assert bits_equal(v, ref[k]), mismatch_report(v, ref[k], f"{cfg} {k}")
    return idx, inf_ind, eng, fl


def test_fullsize_c3_dynamic_rk4_sample():
    """C3: 8192 individuals x 32 rollouts, 3 trees (max_nodes 64, depth <= 10), RK4 x 200,
    201 save points, JIT path, schedule on; 96 individuals compared in full."""
    idx, inf_ind, eng, fl = _run("c3", 96)
    from multitreegp_amd.engine import DeviceEngine
    assert DeviceEngine.jit_ok(fl)  # the JIT code ran (its units cover all 8192 individuals)
    assert len(idx) == 96


def test_fullsize_c2_static_rk4_sample():
    """C2: 1024 individuals x 16 rollouts (4 individuals per wave), 1 tree depth <= 4."""
    idx, inf_ind, eng, fl = _run("c2", 128)
    assert len(idx) == 128


def test_fullsize_c5_wide_sr_sample():
    """C5: 4096 individuals x 8 rollouts, 64 trees (max_nodes 128, depth <= 16), n_var 64,
    RK4 h = 0.01 x 200 (the workgroup-per-lane-set wide-state kernel)."""
    idx, inf_ind, eng, fl = _run("c5", 24)
    assert len(idx) == 24
