"""Time one coefficient-optimisation epoch (CoefficientOptimiser.loss_and_grad: parameterised
flatten + mtgp_sr_grad / mtgp_ctl_grad + reduction) for the 50 candidates gp.py:418-422 optimises,
RK4 and Dopri5 + PID, on the SR (Van der Pol) and dynamic Acrobot shapes.  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from helpers import dynamic_setup, sr_setup  # noqa: E402
from multitreegp_amd import coefficients as co  # noqa: E402
from multitreegp_amd.engine import DeviceEngine  # noqa: E402


def run(name, lib, ff, data, pop, reps=5):
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    opt.loss_and_grad(pop, data)  # warm-up (data upload, first launch)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        loss, grads = opt.loss_and_grad(pop, data)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    n_coef = int(sum(len(g) for g in grads))
    print(json.dumps({"case": name, "candidates": int(pop.shape[0]), "coefficients": n_coef,
                      "ms_per_epoch_median": 1e3 * float(np.median(ts)), "ms_min": 1e3 * float(np.min(ts))}),
          flush=True)


def main():
    dp = (1e-4, 1e-4, 0.001, 1000)
    for solver in (None, dp):
        tag = "dopri5" if solver else "rk4"
        env, lib, ff, data, pop = sr_setup(P=50, R=16, n_save=101, save_every=4, h=0.01, depth=5, N=30, seed=3,
                                           solver=solver)
        run(f"sr_vanderpol_{tag}", lib, ff, data, pop)
        env, lib, ff, data, pop = dynamic_setup(P=50, R=32, n_steps=200, depth=6, N=40, seed=3, solver=solver)
        run(f"dynamic_acrobot_{tag}", lib, ff, data, pop)


if __name__ == "__main__":
    main()
