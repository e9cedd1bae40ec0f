"""DynamicPolicy.ipynb's printed bests at the notebook's own selection scale.

The notebook prints the best fitness of generations 5 / 30 / 50 (DynamicPolicy.ipynb:118, 123,
127): the minimum over 5 populations x 100 candidates (DynamicPolicy.ipynb:94-100) of a fitness
that is chaotic at the last bit (obs noise resampled in every stage, Dopri5 + PID(1e-4) with
max_steps 1000: DynamicPolicy.ipynb:105).  The printed tree is only known through its sympy form
(gp.py:310-328, 344), which hides
  * the coefficients' rounding boxes (every coefficient printed with 2 decimals, gp.py:319),
  * which 2-decimal factors sympy multiplied out: -0.285*y1 is c0*c1*y1 with c0*c1 = -0.285
    (-0.30*0.95, -0.15*1.90, -0.57*0.50, ...), cos(0.16*0.27) inside gen 30's readout may be any
    2-decimal pair with product +-0.0432, cos(0.42) may be cos(-0.42),
  * the tree shape behind a product or a sympy expansion ((c0*c1)*y1 vs c0*(c1*y1) vs
    (c0*y1)*c1; (u + y3)*cos(c) vs cos(c)*u + cos(c')*y3),
and our arithmetic differs from XLA's in the last bits.  The ensemble below draws from all of
these at once, plus one-ulp moves of every initial state, and evaluates it on the GPU through the
product path (bit-exact with the oracle: checked on a sample here, and on the pins themselves by
test_notebook_pin.test_gpu_dynamic_notebook_pins_bitexact).  The question it answers: is the
printed value a plausible minimum over the notebook's candidates, i.e. does it fall inside the
ensemble's lower tail rather than below all of it?

Report: set MTGP_REPORT_DIR to write dp_selection_<pin>.json (quantiles, the printed value's
quantile, the cut-count distribution, the attempt histogram).
"""
import itertools
import json
import os

import numpy as np
import pytest

import multitreegp_amd as mt
from helpers import CONTROL_OPS, bits_equal, oracle_model, oracle_rollouts, tree_from_expr
from test_notebook_pin import DYNAMIC_PINS, dynamic_notebook


def factor_pairs(target: int, limit: int = 999):
    """Every ordered pair of nonzero integers (a, b), |a|, |b| <= limit, with a * b == target --
    the 2-decimal coefficient pairs (a / 100, b / 100) whose product sympy prints as target / 1e4."""
    out = []
    for a in range(1, limit + 1):
        if target % a == 0:
            b = target // a
            if 1 <= abs(b) <= limit:
                out.append((a, b))
                out.append((-a, -b))
    return out


def _gen5_variant(rng, c, shape, fac, cos_sign, expand):
    """[-0.285*y1, 0.913088940312308*u + 0.913088940312308*y3], [-0.95*a1 - 4.15*a2]"""
    box = lambda v: float(v) + rng.uniform(-0.005, 0.005)
    c0, c1 = box(fac[0] / 100), box(fac[1] / 100)
    prod = [("*", ("*", c0, c1), "y1"), ("*", c0, ("*", c1, "y1")), ("*", ("*", c0, "y1"), c1)][shape]
    ca, cb = box(cos_sign * c[2]), box(cos_sign * c[2])
    second = ("+", ("*", ("cos", ca), "u"), ("*", ("cos", cb), "y3")) if expand else \
        ("*", ("+", "u", "y3"), ("cos", ca))
    return [prod, second, ("-", ("*", box(c[3]), "a1"), ("*", box(c[4]), "a2"))]


def _gen30_variant(rng, c, fac):
    box = lambda v: float(v) + rng.uniform(-0.005, 0.005)
    cc = [box(v) for v in c]
    cc[3], cc[4] = box(fac[0] / 100), box(fac[1] / 100)
    return DYNAMIC_PINS["gen30"][0](cc)


def _gen50_variant(rng, c):
    return DYNAMIC_PINS["gen50"][0]([float(v) + rng.uniform(-0.005, 0.005) for v in c])


def ensemble_population(name, lib, n, seed):
    """n candidates drawn over the pin's hidden choices (see the module docstring) -> ([n, 3, 30, 4],
    the choices per candidate)"""
    rng = np.random.default_rng(seed)
    _, c, _ = DYNAMIC_PINS[name]
    trees, meta = [], []
    if name == "gen5":
        facs = factor_pairs(-2850)
        for _ in range(n):
            fac = facs[rng.integers(len(facs))]
            shape, sign, expand = int(rng.integers(3)), (1, -1)[rng.integers(2)], bool(rng.integers(2))
            trees.append(_gen5_variant(rng, c, shape, fac, sign, expand))
            meta.append(dict(fac=fac, shape=shape, cos_sign=sign, expand=expand))
    elif name == "gen30":
        facs = factor_pairs(432) + factor_pairs(-432)
        for _ in range(n):
            fac = facs[rng.integers(len(facs))]
            trees.append(_gen30_variant(rng, c, fac))
            meta.append(dict(fac=fac))
    else:
        for _ in range(n):
            trees.append(_gen50_variant(rng, c))
            meta.append({})
    pop = np.stack([np.stack([tree_from_expr(e, lib, 30) for e in t]) for t in trees])
    return pop, meta


def ulp_moved(data, seed):
    """every initial state moved by one ulp in a random direction (seed < 0: unmoved)"""
    if seed < 0:
        return data
    x0 = np.asarray(data[0], np.float32)
    rng = np.random.default_rng(seed)
    moved = np.nextafter(x0, np.where(rng.random(x0.shape) < 0.5, -1, 1).astype(np.float32)).astype(np.float32)
    return (moved,) + tuple(data[1:])


def test_factor_pairs():
    f = factor_pairs(-2850)
    assert (-30, 95) in f and (30, -95) in f and (-15, 190) in f and (-57, 50) in f and (95, -30) in f
    assert all(a * b == -2850 for a, b in f) and len(f) == len(set(f))
    assert (16, 27) in factor_pairs(432) and (-16, -27) in factor_pairs(432)
    assert all(abs(a) <= 999 and abs(b) <= 999 for a, b in factor_pairs(432))


def test_ensemble_population_prints_like_the_notebook():
    """Every hidden-choice variant renders (reference printer restated in to_string) to the
    notebook's sympy form once the coefficients are the central 2-decimal values."""
    import sympy
    env, lib, ff, data, variables = dynamic_notebook()
    strategy = mt.GeneticProgramming(1, 2, ff, CONTROL_OPS, variables, [2, 1], num_populations=1,
                                     migration_percentage=0.5, verbose=False)
    printed = "[-0.285*y1, 0.913088940312308*u + 0.913088940312308*y3], [-0.95*a1 - 4.15*a2]"
    _, c, _ = DYNAMIC_PINS["gen5"]

    class Central:  # the box draw's rng: no offset
        @staticmethod
        def uniform(lo, hi):
            return 0.0

    for fac, shape, sign, expand in itertools.product([(-30, 95), (-15, 190), (57, -50)], range(3), (1, -1), (0, 1)):
        cand = np.stack([tree_from_expr(e, lib, 30) for e in _gen5_variant(Central, c, shape, fac, sign, expand)])
        ours = strategy.to_string(cand)
        split = lambda s: [e.strip() for e in s.replace("[", "").replace("]", "").split(", ")]
        for a, b in zip(split(ours), split(printed)):
            diff = sympy.simplify(sympy.parse_expr(a) - sympy.parse_expr(b))
            assert abs(float(diff.subs({s: 0.3 for s in diff.free_symbols}))) < 1e-9, (fac, shape, a, b)


N_ULP = 16          # one-ulp x0 moves per pin (+ the unmoved data)
N_PER_DATA = 128    # hidden-choice draws per x0 set -> 17 x 128 = 2,176 members per pin


def _selection_ensemble(name, max_steps=1000):
    import torch
    from multitreegp_amd.engine import DeviceEngine
    env, lib, ff, data, _ = dynamic_notebook(max_steps)
    eng = DeviceEngine(ff, lib, 0.0, "cuda:0")
    fits, steps, metas = [], [], []
    sample = None
    for s in range(-1, N_ULP):
        pop, meta = ensemble_population(name, lib, N_PER_DATA, seed=1000 * (s + 2))
        dat = ulp_moved(data, s)
        res = eng.evaluate(torch.from_numpy(pop).cuda(), dat, rollout_fitness=True, step_counts=True)
        fits.append(res["fitness"].cpu().numpy())
        steps.append(res["steps"].cpu().numpy().reshape(N_PER_DATA, -1))
        metas += meta
        if s == 0:
            sample = (pop[:8], dat, fits[-1][:8])
    # the statements below are about the oracle's spec too: a sample checked bit for bit
    from oracle import oracle as orc
    pop8, dat, got = sample
    d = ff.prepare(dat)
    ref = orc.evaluate(oracle_model(ff, d), pop8, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(got, ref)
    return np.concatenate(fits), np.concatenate(steps), metas


def _report(name, fit, steps, metas, max_steps):
    printed = DYNAMIC_PINS[name][2]
    f = fit.astype(np.float64)
    cut = (steps >= max_steps).sum(axis=1)
    qs = [0.001, 0.01, 0.05, 0.25, 0.5]
    rep = dict(pin=name, printed=printed, members=int(f.size), max_steps=max_steps,
               printed_quantile=float((f <= printed).mean()), below_printed=int((f <= printed).sum()),
               min=float(f.min()), mean=float(f.mean()), sd=float(f.std()),
               quantiles={str(q): float(np.quantile(f, q)) for q in qs},
               cut_count_hist={str(k): int((cut == k).sum()) for k in range(steps.shape[1] + 1)},
               cut_mean=float(cut.mean()),
               attempts_hist=dict(zip([f"{a}-{a + 99}" for a in range(0, max_steps, 100)] + [f">={max_steps}"],
                                      [int(v) for v in np.histogram(np.minimum(steps, max_steps),
                                                                    bins=list(range(0, max_steps + 1, 100)) + [max_steps + 1])[0]])))
    # the lowest-fitness members' hidden choices and cut counts
    lo = np.argsort(f)[:10]
    rep["lowest"] = [dict(fitness=float(f[i]), cut=int(cut[i]), **{k: (list(v) if isinstance(v, tuple) else v)
                                                                     for k, v in metas[i].items()}) for i in lo]
    # fitness vs cut count: a solve cut at max_steps scores 250 + cost_0 (test_notebook_pin)
    rep["mean_fitness_by_cut"] = {str(k): float(f[cut == k].mean()) for k in np.unique(cut)}
    out = os.environ.get("MTGP_REPORT_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"dp_selection_{name}.json"), "w") as fh:
            json.dump(rep, fh, indent=1)
    print(json.dumps({k: rep[k] for k in ("pin", "printed", "members", "printed_quantile", "min", "mean", "sd",
                                          "quantiles", "cut_mean")}))
    return rep


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(DYNAMIC_PINS))
def test_gpu_dynamic_notebook_selection_ensemble(name):
    fit, steps, metas = _selection_ensemble(name)
    rep = _report(name, fit, steps, metas, 1000)
    assert rep["members"] >= 2000 and np.all(np.isfinite(fit))
    printed, q = rep["printed"], rep["printed_quantile"]
    if name == "gen5":
        # The established discrepancy (DESIGN.md "Parity pins", round 6): gen 5's printed value lies
        # below every one of the 2,176 members -- it survives selection at the notebook's scale (a
        # minimum over 500 candidates would sit near the 0.2 % quantile).  Our members are cut at
        # max_steps in 6-15 of 16 rollouts; 171.8 needs about 2.  Pinned so a change is noticed.
        assert q == 0.0 and rep["min"] - printed > 15.0, (rep["min"], printed)
    else:
        # inside the lower tail, where a minimum over the notebook's 500 candidates belongs
        assert 0.0 < q <= {"gen30": 0.02, "gen50": 0.2}[name], (name, q)


# ------------------------------------------------------------------ StaticPolicy.ipynb
N_ULP_STATIC = 512  # one-ulp x0 moves: the printed static bests are exact trees (no hidden coefficients)


@pytest.mark.gpu
def test_gpu_static_notebook_ulp_ensemble():
    """StaticPolicy.ipynb's coefficient-free bests (136.4901, 133.3388; StaticPolicy.ipynb:117-124)
    against 512 one-ulp moves of the notebook's initial states, on the GPU (the 16-member oracle
    ensemble of test_notebook_pin, scaled up).  The trees are exact, so the printed value is one
    draw of the tree's own last-bit chaos distribution -- but the draw that won a population-wide
    selection, so it belongs at the extreme lower tail (a minimum over ~500 candidates sits near
    the 0.2 % quantile).  Asserted: printed at or below the 1 % quantile, and below the ensemble
    minimum by less than a tenth of the ensemble's standard deviation -- which holds for
    y4 + sin(sin(y4)) (136.49 vs min 136.69 of 512, median 160.3; profiles/r06/
    static_ulp_ensemble.json).  y4 + sin(y4 + sin(y4 + sin(y4))) prints 133.34, 4.3 units (0.84 sd)
    below all 512 members (min 137.61, median 148.2): the same direction as DynamicPolicy's gen 5
    under the same noisy Dopri5 + PID regime (DESIGN.md "Parity pins"), recorded and asserted as an
    established discrepancy so that a change is noticed."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    from test_notebook_pin import STATIC_BESTS, _static_pop, static_notebook
    env, lib, ff, data = static_notebook()
    pop = _static_pop(lib)
    eng = DeviceEngine(ff, lib, 1.0, "cuda:0")  # size_parsinomy 1 (StaticPolicy.ipynb)
    pt = torch.from_numpy(pop).cuda()
    fits = np.stack([eng.evaluate(pt, ulp_moved(data, 5000 + s))["fitness"].cpu().numpy()
                     for s in range(N_ULP_STATIC)])
    rep = {}
    for i, (name, (_, printed)) in enumerate(STATIC_BESTS.items()):
        f = fits[:, i].astype(np.float64)
        rep[name] = dict(printed=printed, members=int(f.size), printed_quantile=float((f <= printed).mean()),
                         min=float(f.min()), median=float(np.median(f)), mean=float(f.mean()), sd=float(f.std()))
        rep[name]["q01"] = float(np.quantile(f, 0.01))
        assert np.all(np.isfinite(f))
    out = os.environ.get("MTGP_REPORT_DIR")
    if out:
        with open(os.path.join(out, "static_ulp_ensemble.json"), "w") as fh:
            json.dump(rep, fh, indent=1)
    print(json.dumps(rep))
    r1, r2 = rep["y4 + sin(sin(y4))"], rep["y4 + sin(y4 + sin(y4 + sin(y4)))"]
    assert r1["printed"] <= r1["q01"] and r1["min"] - r1["printed"] < 0.1 * r1["sd"], r1
    assert r2["printed"] < r2["min"] and r2["min"] - r2["printed"] < 1.5 * r2["sd"], r2
