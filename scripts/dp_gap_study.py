"""DynamicPolicy.ipynb parity gap: the printed bests of generations 5 / 30 / 50 against the oracle's
ensemble under alternative readings of diffrax's Dopri5 + PIDController rules (oracle-only flags
OR_DP_ALT_*, oracle/mtgp_oracle.c; the product follows the spec include/mtgp_dopri5.h = variant "spec").

For every variant and pin: the ensemble (16 one-ulp x0 moves + 32 draws from the printed coefficients'
rounding boxes, tests/test_notebook_pin.py) at the notebook's max_steps 1000 -> min / mean fitness, the
printed value's position, and the mean Dopri5 attempts per rollout of the central candidate.

    python scripts/dp_gap_study.py [--variants spec,eo6,...] [--json out.json]

Test infrastructure (CPU oracle only): never part of the product."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as orc  # noqa: E402
from helpers import oracle_model, oracle_rollouts  # noqa: E402
import test_notebook_pin as nb  # noqa: E402

FLAGS = {"eo6": 1, "fsal_t1": 2, "dtmin_attempt": 4, "sum_literal": 8, "norm_x": 16, "maxsteps_acc": 32,
         "event_all": 64, "interp_t0": 128}
VARIANTS = {"spec": 0, **FLAGS, "eo6+fsal_t1": 3, "eo6+sum_literal": 9, "eo6+fsal_t1+sum_literal": 11,
            "eo6+all_small": 1 | 2 | 4 | 8 | 128}


def run(alt, name, max_steps, n_ulp=16, n_box=32):
    make, c, printed = nb.DYNAMIC_PINS[name]
    env, lib, ff, data, _ = nb.dynamic_notebook(max_steps)
    d = ff.prepare(data)
    model = dict(oracle_model(ff, d), dp_alt=alt)
    pop = nb._dyn_candidate(lib, make, c)[None]
    central = orc.evaluate(model, pop, lib, oracle_rollouts(d), steps=True)
    ulp = [orc.evaluate(model, pop, lib, oracle_rollouts(nb._perturbed(d, 100 + s)))["fitness"][0] for s in range(n_ulp)]
    box = orc.evaluate(model, nb._dyn_box(lib, make, c, n_box), lib, oracle_rollouts(d))["fitness"]
    ens = np.concatenate([np.float32(ulp), box]).astype(np.float64)
    st = central["steps"][0]
    return dict(printed=printed, min=float(ens.min()), mean=float(ens.mean()), sd=float(ens.std()),
                quantile=float((ens < printed).mean()), gap_min=float(ens.min() - printed),
                central=float(central["fitness"][0]), attempts_mean=float(st.mean()),
                cut=int((st >= max_steps).sum()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--pins", default="gen5,gen30,gen50")
    ap.add_argument("--max-steps", type=int, default=1000)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = {}
    for v in a.variants.split(","):
        res[v] = {}
        for pin in a.pins.split(","):
            t0 = time.time()
            r = run(VARIANTS[v], pin, a.max_steps)
            res[v][pin] = r
            print(f"{v:24s} {pin:6s} printed {r['printed']:8.2f}  ens min {r['min']:8.2f} mean {r['mean']:8.2f} "
                  f"sd {r['sd']:5.2f}  q {r['quantile']:.2f}  gap {r['gap_min']:+7.2f}  attempts {r['attempts_mean']:7.1f} "
                  f"cut {r['cut']:2d}/16  ({time.time() - t0:.0f}s)", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
