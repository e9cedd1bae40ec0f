"""Pins against the only outputs the reference itself holds: the fitness values its three
example notebooks printed.  jax/diffrax cannot run here, so these recorded
values are the reference-side anchor of the oracle and, through the bit-exact GPU tests, of
the HIP path.

SymbolicRegression.ipynb (Van der Pol, Dopri5 + PIDController(1e-6, 1e-6, dtmin=0.001),
dt0 0.01, max_steps 500, data from PRNGKey(0)): the SR fitness is a smooth function of the
candidate, so a printed best solution pins the evaluator once its printed (2-decimal,
gp.py:319) coefficients are widened back to their rounding intervals -- the recorded fitness
must lie inside the fitness range of that coefficient box.

StaticPolicy.ipynb (Acrobot, obs_noise 0.1, Dopri5 + PID(1e-4, 1e-4, dtmin=0.001), dt0 0.05,
max_steps 1000, data from PRNGKey(1), size_parsinomy 1): the coefficient-free best policies
`y4 + sin(sin(y4))` (136.4901, StaticPolicy.ipynb:117-119) and `y4 + sin(y4 + sin(y4 +
sin(y4)))` (133.3388, :120-124) are exact trees, but the controlled acrobot is chaotic at the
last bit: moving one initial state by one ulp moves the mean fitness by several units
(test_static_notebook_values_are_chaotic).  Reproducing the printed 4 decimals would need the
JAX/XLA arithmetic bit for bit (XLA's sin/cos/log1p/pow and diffrax's summation orders, none of
which can run here); the check is therefore statistical: each printed best must sit in the
lower tail of our perturbation ensemble (it is the minimum over a whole evolving population).
DESIGN.md "Parity pins" records the numbers.
"""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import prng
from oracle import oracle as orc

from helpers import CONTROL_OPS, SR_OPS, bits_equal, oracle_model, oracle_rollouts, tree_from_expr

# ---------------------------------------------------------------- SymbolicRegression.ipynb
SR_N = 30


def sr_notebook():
    """SymbolicRegression.ipynb cells 0-6: key = PRNGKey(0); init_key, data_key = split(key);
    get_data(data_key, VanDerPol, T=20, batch_size=16); the notebook's evaluator."""
    env = mt.VanDerPolOscillator(0, 0)
    _init_key, data_key = prng.split(prng.PRNGKey(0))
    data = mt.environments.jax_sr_data(data_key, env, 16, 20.0)
    lib = mt.NodeLibrary(SR_OPS, [["x0", "x1"]], [2])
    ff = mt.SREvaluator(solver=mt.Dopri5(), dt0=0.01, max_steps=500,
                        stepsize_controller=mt.PIDController(atol=1e-6, rtol=1e-6, dtmin=0.001))
    return env, lib, ff, data


def _vdp_like(c1, c2, a=1.0):
    """x0**2*x1*a - x0 + 2*x1*(c1 - c2*x0**2) (SymbolicRegression.ipynb:166-176 printed forms)"""
    sq = ("*", "x0", "x0")
    first = ("*", sq, "x1") if a == 1.0 else ("*", ("*", a, sq), "x1")
    return ("+", ("-", first, "x0"), ("*", ("*", 2.0, "x1"), ("-", c1, ("*", c2, sq))))


# (generation, printed fitness, [tree expr factories over the box], box of coefficient intervals)
def _sr_pins():
    c_lo = lambda v, f=1: (v - 0.005 * f, v + 0.005 * f)
    return [
        # gen 5: [x1, -0.81*x0] -> 2.1709
        ("gen5", 2.1709, lambda c: ["x1", ("*", c[0], "x0")], [c_lo(-0.81)]),
        # gen 15: [x1, -0.92512*x0] -> 1.4823; the coefficient is a product of printed
        # 2-decimal coefficients (0.92512 = 0.49 * 0.59 * 3.2 or another split), widened by 2 %
        ("gen15", 1.4823, lambda c: ["x1", ("*", c[0], "x0")], [(-0.92512 * 1.02, -0.92512 * 0.98)]),
        # gen 85: [x1, x0**2*x1 - x0 + 2*x1*(0.47 - 1.0148*x0**2)] -> 0.0210 (1.0148 = 0.59 * 1.72)
        ("gen85", 0.0210, lambda c: ["x1", _vdp_like(c[0], c[1])], [c_lo(0.47), (1.0148 * 0.988, 1.0148 * 1.012)]),
        # gen 100: [x1 - 0.0019, x0**2*x1 - x0 + 2*x1*(0.49 - 1.0148*x0**2)] -> 0.0095 (0.0019 = 0.19 * 0.01)
        ("gen100", 0.0095, lambda c: [("-", "x1", c[2]), _vdp_like(c[0], c[1])],
         [c_lo(0.49), (1.0148 * 0.988, 1.0148 * 1.012), (0.185 * 0.005, 0.195 * 0.015)]),
    ]


def _box_population(lib, make, box, n=5):
    grids = np.meshgrid(*[np.linspace(lo, hi, n) for lo, hi in box], indexing="ij")
    coeffs = np.stack([g.ravel() for g in grids], 1)
    pop = np.stack([np.stack([tree_from_expr(e, lib, SR_N) for e in make([float(v) for v in c])]) for c in coeffs])
    return pop


def _sr_oracle(ff, data, lib, pop):
    d = ff.prepare(data)
    return orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]


def test_sr_notebook_data():
    """x0 = normal(split(split(PRNGKey(0))[1])[0], (16, 2)), ts = arange(0, 20, 0.2)."""
    env, lib, ff, (x0, ts, xs, keys) = sr_notebook()
    assert x0.shape == (16, 2) and ts.shape == (100,) and xs.shape == (16, 100, 2) and keys.shape == (16, 2)
    k = prng.split(prng.split(prng.PRNGKey(0))[1])[0]
    assert bits_equal(x0, orc.random_normals(k, 32, 0).reshape(16, 2))  # host normal == the spec's
    assert np.all(xs[:, 0] == x0) and np.all(np.isfinite(xs))


def test_sr_notebook_ground_truth_reaches_t_end_like_the_notebook():
    """The notebook's ground truth: Dopri5 + PID(1e-7, 1e-7, dtmin=0.001), dt0 0.001, max_steps
    2000 in float32 (its finite recorded fitness implies the solve reached t = 19.8).  The
    oracle's restatement with the same settings also finishes and agrees with the float64
    ground truth used by the pins to far below the fitness resolution."""
    env, lib, _, (x0, ts, xs, keys) = sr_notebook()
    ff = mt.SREvaluator(solver=mt.Dopri5(), dt0=0.001, max_steps=2000,
                        stepsize_controller=mt.PIDController(atol=1e-7, rtol=1e-7, dtmin=0.001))
    # Van der Pol as trees: dx0 = x1, dx1 = (1 - x0*x0)*x1 - x0 (vd_pol_oscillator.py:22-23, mu = 1)
    vdp = np.stack([tree_from_expr("x1", lib, SR_N),
                    tree_from_expr(("-", ("*", ("-", 1.0, ("*", "x0", "x0")), "x1"), "x0"), lib, SR_N)])[None]
    d = ff.prepare((x0, ts, xs, keys))
    out = orc.evaluate(oracle_model(ff, d), vdp, lib, oracle_rollouts(d), trajectories=True)
    f32 = out["xs"][0]
    assert np.all(np.isfinite(f32))
    np.testing.assert_allclose(f32, xs, atol=2e-4, rtol=0)
    assert out["fitness"][0] < 1e-7


@pytest.mark.parametrize("pin", _sr_pins(), ids=lambda p: p[0])
def test_sr_notebook_fitness_bracket(pin):
    """The printed fitness lies inside the oracle's fitness range over the rounding box of the
    printed coefficients (for the one-coefficient pins the box is narrow: < 12 % of the value)."""
    name, printed, make, box = pin
    env, lib, ff, data = sr_notebook()
    fit = _sr_oracle(ff, data, lib, _box_population(lib, make, box))
    lo, hi = float(fit.min()), float(fit.max())
    assert lo <= printed + 5e-5 and hi >= printed - 5e-5, (name, printed, lo, hi)
    if name in ("gen5", "gen15"):  # one coefficient: a narrow bracket (the later boxes are wide:
        assert hi - lo < 0.12 * printed, (name, lo, hi)  # near the optimum MSE is steep in them)


def test_sr_notebook_gen5_coefficient():
    """gen 5 `[x1, -0.81*x0]` -> 2.1709: the coefficient that gives the printed fitness (bisection
    on the oracle) prints as -0.81 again, i.e. lies in [-0.815, -0.805)."""
    env, lib, ff, data = sr_notebook()

    def f(c):
        pop = np.stack([tree_from_expr("x1", lib, SR_N), tree_from_expr(("*", float(c), "x0"), lib, SR_N)])[None]
        return float(_sr_oracle(ff, data, lib, pop)[0])

    lo, hi = -0.815, -0.805
    flo, fhi = f(lo), f(hi)
    assert (flo - 2.1709) * (fhi - 2.1709) < 0
    for _ in range(30):
        mid = 0.5 * (lo + hi)
        fm = f(mid)
        if (fm - 2.1709) * (flo - 2.1709) > 0:
            lo, flo = mid, fm
        else:
            hi, fhi = mid, fm
    assert "{:.2f}".format(0.5 * (lo + hi)) == "-0.81"


# --------------------------------------------------------------------- StaticPolicy.ipynb
STATIC_BESTS = {  # StaticPolicy.ipynb:117-124 (printed fitness includes size_parsinomy = 1 x nodes)
    "y4 + sin(sin(y4))": (("+", "y4", ("sin", ("sin", "y4"))), 136.4901),
    "y4 + sin(y4 + sin(y4 + sin(y4)))": (("+", "y4", ("sin", ("+", "y4", ("sin", ("+", "y4", ("sin", "y4")))))),
                                         133.3388),
}


def static_notebook():
    """StaticPolicy.ipynb cells 0-4: key = PRNGKey(1); init_key, data_key = split(key);
    get_data(data_key, Acrobot(0.05, 0.1), 16, 0.2, 50, "Constant"); the notebook's evaluator."""
    env = mt.Acrobot(0.05, 0.1)
    _init_key, data_key = prng.split(prng.PRNGKey(1))
    data = mt.environments.jax_control_data(data_key, env, 16, 0.2, 50.0)
    lib = mt.NodeLibrary(CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1])
    ff = mt.FeedforwardEvaluator(env, 0.05, solver=mt.Dopri5(), max_steps=1000,
                                 stepsize_controller=mt.PIDController(atol=1e-4, rtol=1e-4, dtmin=0.001))
    return env, lib, ff, data


def _static_pop(lib):
    return np.stack([tree_from_expr(e, lib, 30)[None] for e, _ in STATIC_BESTS.values()])


def _perturbed(d, seed):
    rng = np.random.default_rng(seed)
    x0 = d["x0"]
    d2 = dict(d)
    d2["x0"] = np.nextafter(x0, np.where(rng.random(x0.shape) < 0.5, -1, 1).astype(np.float32)).astype(np.float32)
    return d2


def test_static_notebook_values_are_chaotic():
    """Why the control notebooks cannot pin 4 decimals: one-ulp moves of the initial states move
    each best policy's fitness by several units, far beyond the printed precision."""
    env, lib, ff, data = static_notebook()
    d = ff.prepare(data)
    pop = _static_pop(lib)
    model = oracle_model(ff, d, parsimony=1.0)
    ens = np.stack([orc.evaluate(model, pop, lib, oracle_rollouts(_perturbed(d, 100 + s)))["fitness"]
                    for s in range(16)])
    assert np.all(np.isfinite(ens)) and np.all(ens > 0)
    spread = ens.max(0) - ens.min(0)
    assert np.all(spread > 5.0), spread
    for j, (_, printed) in enumerate(STATIC_BESTS.values()):
        mean, sd = ens[:, j].mean(), ens[:, j].std()
        # the printed value is the best of an evolving population of such draws: lower tail
        assert mean - 4.5 * sd <= printed <= mean + 1.0 * sd, (printed, mean, sd)


def test_static_notebook_nodes_and_rollouts():
    """Parsimony term and data shape of the notebook evaluation: 5 and 10 non-empty nodes,
    16 rollouts on 250 save points, and no rollout of the two bests fails (finite fitness)."""
    env, lib, ff, data = static_notebook()
    d = ff.prepare(data)
    pop = _static_pop(lib)
    assert [int((t[..., 0] != 0).sum()) for t in pop] == [5, 10]
    assert d["R"] == 16 and d["n_save"] == 250 and d["ts"][-1] == np.float32(49.8)
    out = orc.evaluate(oracle_model(ff, d, parsimony=1.0), pop, lib, oracle_rollouts(d))
    assert np.all(np.isfinite(out["rollout_fitness"]))
    np.testing.assert_allclose(out["fitness"] - np.float32([5, 10]), out["rollout_fitness"].mean(1), rtol=1e-6)


# ------------------------------------------------------------------------------ GPU
def _gp(lib_ops, variables, layer_sizes, ff, n, parsimony=0.0):
    return mt.GeneticProgramming(1, n, ff, lib_ops, variables, layer_sizes, num_populations=1,
                                 size_parsinomy=parsimony, migration_percentage=0.5, elite_percentage=0.0,
                                 verbose=False)


@pytest.mark.gpu
def test_gpu_sr_notebook_pins_bitexact():
    """Every SR pin box through GeneticProgramming.evaluate_population on the GPU: bit-exact
    with the oracle, so the bracket holds for the HIP path too."""
    env, lib, ff, data = sr_notebook()
    for name, printed, make, box in _sr_pins():
        pop = _box_population(lib, make, box)
        if pop.shape[0] % 2:
            pop = np.concatenate([pop, pop[:1]])
        strategy = _gp(SR_OPS, [["x0", "x1"]], [2], ff, pop.shape[0])
        fit, _ = strategy.evaluate_population(pop[None], data)
        ref = _sr_oracle(ff, data, lib, pop)
        assert bits_equal(fit[0], ref), name
        assert fit.min() <= printed + 5e-5 <= fit.max() + 1e-4, name


@pytest.mark.gpu
def test_gpu_static_notebook_config_bitexact():
    """The StaticPolicy notebook's whole evaluation (16 rollouts, 250 save points, obs noise,
    Dopri5 + PID, parsimony 1) on the GPU for the two printed bests plus 62 reference-
    distribution trees: fitness bit-exact with the oracle."""
    from multitreegp_amd.sampling import sample_population
    env, lib, ff, data = static_notebook()
    pop = np.concatenate([_static_pop(lib), sample_population(5, lib, 62, 1, max_init_depth=4, max_nodes=30)[0]])
    strategy = _gp(CONTROL_OPS, [["y1", "y2", "y3", "y4"]], [1], ff, pop.shape[0], parsimony=1.0)
    fit, _ = strategy.evaluate_population(pop[None], data)
    d = ff.prepare(data)
    ref = orc.evaluate(oracle_model(ff, d, parsimony=1.0), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(fit[0], ref)
    assert strategy.best_fitnesses[0] == ref.min()


@pytest.mark.gpu
def test_gpu_dynamic_notebook_config_bitexact():
    """DynamicPolicy.ipynb's evaluation setup (state_size 2, obs noise 0.1, Dopri5 + PID(1e-4),
    max_steps 1000, 16 rollouts x 250 save points, PRNGKey(1) data) on 64 sampled candidates."""
    from multitreegp_amd.sampling import sample_population
    env = mt.Acrobot(0.05, 0.1)
    _init_key, data_key = prng.split(prng.PRNGKey(1))
    data = mt.environments.jax_control_data(data_key, env, 16, 0.2, 50.0)
    variables = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
    lib = mt.NodeLibrary(CONTROL_OPS, variables, [2, 1])
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.Dopri5(), max_steps=1000,
                             stepsize_controller=mt.PIDController(atol=1e-4, rtol=1e-4, dtmin=0.001))
    pop = sample_population(6, lib, 64, 1, max_init_depth=4, max_nodes=30)[0]
    strategy = _gp(CONTROL_OPS, variables, [2, 1], ff, 64)
    fit, _ = strategy.evaluate_population(pop[None], data)
    d = ff.prepare(data)
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(fit[0], ref)


# -------------------------------------------------------------------- DynamicPolicy.ipynb
def dynamic_notebook(max_steps=1000):
    """DynamicPolicy.ipynb cells 0-4: key = PRNGKey(1); init_key, data_key = split(key);
    get_data(data_key, Acrobot(0.05, 0.1), 16, 0.2, 50, "Constant"); state_size 2; the notebook's
    evaluator Dopri5 + PIDController(1e-4, 1e-4, dtmin=0.001), dt0 0.05, max_steps 1000
    (DynamicPolicy.ipynb:105); size_parsinomy 0 (the gp.py:72 default)."""
    env = mt.Acrobot(0.05, 0.1)
    _init_key, data_key = prng.split(prng.PRNGKey(1))
    data = mt.environments.jax_control_data(data_key, env, 16, 0.2, 50.0)
    variables = [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]]
    lib = mt.NodeLibrary(CONTROL_OPS, variables, [2, 1])
    ff = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.Dopri5(), max_steps=max_steps,
                             stepsize_controller=mt.PIDController(atol=1e-4, rtol=1e-4, dtmin=0.001))
    return env, lib, ff, data, variables


# The printed bests (DynamicPolicy.ipynb:118, 123, 127) as trees.  to_string prints every
# coefficient with 2 decimals and sympy then multiplies them out (gp.py:318-319, 344), so the long
# decimals are sympy's values of coefficient expressions: 0.913088940312308 = cos(0.42),
# 0.134250724017567 = 0.16*(cos(0.16*0.27) - 0.16), 0.128749603586318 = 0.16*(cos(0.27*cos(0.16))
# - 0.16) (found by exhaustive search over the 2-decimal coefficients the runs print), -0.285 =
# -0.30*0.95, 2*a1 = a1 + a1, 2*a2**2 = (a2 + a2)*a2.  The exact tree shapes are not recoverable
# from the sympy form; other shapes differ in the last bits only, which the ulp ensemble covers.
def _dyn_gen5(c):  # [-0.285*y1, 0.913088940312308*u + 0.913088940312308*y3], [-0.95*a1 - 4.15*a2]
    return [("*", ("*", c[0], c[1]), "y1"), ("*", ("+", "u", "y3"), ("cos", c[2])),
            ("-", ("*", c[3], "a1"), ("*", c[4], "a2"))]


def _dyn_gen30(c):  # [(-a1 - sin(y4)*sin(y1 + 1.24) + 1.24)*sin(y4), (u + y3)*cos(0.134250724017567*y3)],
    #                  [a1*a2 + 2*a1 - 3.15*a2 - cos(2.15*a2) - 2.46]
    return [("*", ("-", ("-", c[0], "a1"), ("*", ("sin", "y4"), ("sin", ("+", "y1", c[1])))), ("sin", "y4")),
            ("*", ("+", "u", "y3"), ("cos", ("*", ("*", c[2], ("-", ("cos", ("*", c[3], c[4])), c[5])), "y3"))),
            ("-", ("-", ("+", ("*", "a1", "a2"), ("+", "a1", "a1")), ("*", c[6], "a2")),
             ("+", ("cos", ("*", c[7], "a2")), c[8]))]


def _dyn_gen50(c):  # [(-a1 - sin(y1)*sin(sin(y1 + 1.24)) - sin(y4)*sin(-a1 + y1 + 1.24) + 1.24)*sin(y4),
    #                   (u + y3)*cos(0.128749603586318*y3)], [2*a1 + 2*a2**2 - a2 - cos(cos(2.15*a2)) - 1.73]
    return [("*", ("-", ("-", ("-", c[0], "a1"), ("*", ("sin", "y1"), ("sin", ("sin", ("+", "y1", c[1]))))),
                   ("*", ("sin", "y4"), ("sin", ("+", ("-", "y1", "a1"), c[2])))), ("sin", "y4")),
            ("*", ("+", "u", "y3"), ("cos", ("*", ("*", c[3], ("-", ("cos", ("*", c[4], ("cos", c[5]))), c[6])), "y3"))),
            ("-", ("-", ("+", ("+", "a1", "a1"), ("*", ("+", "a2", "a2"), "a2")), "a2"),
             ("+", ("cos", ("cos", ("*", c[7], "a2"))), c[8]))]


DYNAMIC_PINS = {  # generation: (tree factory, printed 2-decimal coefficients, printed best fitness)
    "gen5": (_dyn_gen5, [-0.30, 0.95, 0.42, -0.95, 4.15], 171.8213),
    "gen30": (_dyn_gen30, [1.24, 1.24, 0.16, 0.16, 0.27, 0.16, 3.15, 2.15, 2.46], 133.5592),
    "gen50": (_dyn_gen50, [1.24, 1.24, 1.24, 0.16, 0.27, 0.16, 0.16, 2.15, 1.73], 129.2088),
}


def _dyn_candidate(lib, make, c):
    return np.stack([tree_from_expr(e, lib, 30) for e in make([float(v) for v in c])])


def _dyn_box(lib, make, c, n, seed=7):
    """n candidates with every printed coefficient drawn uniformly from its rounding box +-0.005"""
    rng = np.random.default_rng(seed)
    return np.stack([_dyn_candidate(lib, make, [v + rng.uniform(-0.005, 0.005) for v in c]) for _ in range(n)])


def _dyn_ensemble(name, max_steps, n_ulp=16, n_box=32, dp_alt=0):
    """fitness of the pinned candidate over a one-ulp x0 ensemble (central coefficients) and over
    its coefficient rounding box (notebook data); dp_alt: an oracle-only alternative reading of a
    diffrax rule (OR_DP_ALT_*, scripts/dp_gap_study.py)"""
    make, c, _ = DYNAMIC_PINS[name]
    env, lib, ff, data, _ = dynamic_notebook(max_steps)
    d = ff.prepare(data)
    model = dict(oracle_model(ff, d), dp_alt=dp_alt)
    pop = _dyn_candidate(lib, make, c)[None]
    ulp = [orc.evaluate(model, pop, lib, oracle_rollouts(_perturbed(d, 100 + s)))["fitness"][0] for s in range(n_ulp)]
    box = orc.evaluate(model, _dyn_box(lib, make, c, n_box), lib, oracle_rollouts(d))["fitness"]
    return np.concatenate([np.float32(ulp), box])


def test_dynamic_notebook_trees_print_like_the_notebook():
    """The reconstructed trees render (through the reference's own printer, restated in
    GeneticProgramming.to_string) to the notebook's strings up to sympy's term order."""
    import sympy
    env, lib, ff, data, variables = dynamic_notebook()
    strategy = _gp(CONTROL_OPS, variables, [2, 1], ff, 2)
    printed = {"gen5": "[-0.285*y1, 0.913088940312308*u + 0.913088940312308*y3], [-0.95*a1 - 4.15*a2]",
               "gen30": "[(-a1 - sin(y4)*sin(y1 + 1.24) + 1.24)*sin(y4), (u + y3)*cos(0.134250724017567*y3)], "
                        "[a1*a2 + 2*a1 - 3.15*a2 - cos(2.15*a2) - 2.46]",
               "gen50": "[(-a1 - sin(y1)*sin(sin(y1 + 1.24)) - sin(y4)*sin(-a1 + y1 + 1.24) + 1.24)*sin(y4), "
                        "(u + y3)*cos(0.128749603586318*y3)], [2*a1 + 2*a2**2 - a2 - cos(cos(2.15*a2)) - 1.73]"}
    for name, (make, c, _) in DYNAMIC_PINS.items():
        ours = strategy.to_string(_dyn_candidate(lib, make, c))
        split = lambda s: [e.strip() for e in s.replace("[", "").replace("]", "").split(", ")]
        for a, b in zip(split(ours), split(printed[name])):
            diff = sympy.simplify(sympy.parse_expr(a) - sympy.parse_expr(b))
            assert abs(float(diff.subs({s: 0.3 for s in diff.free_symbols}))) < 1e-9, (name, a, b)


def test_dynamic_notebook_solves_sit_on_the_max_steps_edge():
    """Why DynamicPolicy's printed values cannot be matched closely: every rollout of the printed
    bests needs about max_steps = 1000 Dopri5 attempts (obs noise resampled in every stage keeps
    the PID controller near the noise floor), and a solve cut at max_steps scores 250 + cost_0
    (the +inf fill is masked out of acrobot.py:82's cost and never reaches the threshold) -- so
    the fitness hinges on how many of 16 attempt counts fall below 1000.  At max_steps 800 every
    rollout of the gen-5 best is cut; at 4000 none is, and the fitness drops by > 30."""
    make, c, _ = DYNAMIC_PINS["gen5"]
    out = {}
    for ms in (800, 1000, 4000):
        env, lib, ff, data, _ = dynamic_notebook(ms)
        d = ff.prepare(data)
        out[ms] = orc.evaluate(oracle_model(ff, d), _dyn_candidate(lib, make, c)[None], lib, oracle_rollouts(d))
    assert np.all(out[800]["rollout_fitness"] >= 250.0)
    assert np.all(np.isfinite(out[4000]["rollout_fitness"]))
    assert out[1000]["fitness"][0] - out[4000]["fitness"][0] > 30.0
    assert (out[4000]["rollout_fitness"] < 250.0).sum() == 16


@pytest.mark.parametrize("name", list(DYNAMIC_PINS))
def test_dynamic_notebook_printed_best_in_ensemble_tail(name):
    """Each printed best (gen 5 / 30 / 50) against the oracle's ensemble: one-ulp x0 moves (16) and
    the printed coefficients' rounding boxes (32 draws).  The ensemble is wide (the noisy solves
    are chaotic at the last bit: sd 3-10 units), and the printed value is the minimum over 500
    evolving candidates, so it must sit in the ensemble's lower tail.  With the attempt limit
    relaxed (max_steps 4000, no solve cut) it does for all three: min <= printed <= mean.  At the
    notebook's max_steps 1000 the statement needs the selection-scale ensemble of
    tests/test_notebook_selection.py (2,176 members per pin over the sympy form's hidden choices):
    gen 30 and gen 50 then lie in the lower tail (quantiles 0.3 % and 5.6 %), gen 5 stays below
    every member (DESIGN.md "Parity pins": an established discrepancy)."""
    printed = DYNAMIC_PINS[name][2]
    relaxed = _dyn_ensemble(name, 4000)
    assert np.all(np.isfinite(relaxed))
    assert relaxed.min() <= printed + 1.0 and printed <= relaxed.mean(), (name, relaxed.min(), relaxed.mean())
    assert relaxed.mean() - printed < 4.0 * relaxed.std() + 1.0, (name, relaxed.mean(), relaxed.std())
    notebook = _dyn_ensemble(name, 1000)
    assert printed <= notebook.max()
    # At the notebook's max_steps the 48-member ensemble is too small to place a minimum over 500
    # candidates; the selection-scale statement (>= 2,000 members per pin, the printed value's
    # quantile) is tests/test_notebook_selection.py::test_gpu_dynamic_notebook_selection_ensemble.


# oracle-only alternative readings (oracle/mtgp_oracle.c OR_DP_ALT_*)
DP_ALT = {"eo6": 1, "fsal_t1": 2, "dtmin_attempt": 4, "sum_literal": 8, "norm_x": 16, "maxsteps_acc": 32,
          "event_all": 64, "interp_t0": 128}


@pytest.mark.parametrize("name", ["gen5", "gen30"])
def test_dynamic_notebook_gap_readings(name):
    """The gap study (scripts/dp_gap_study.py) in test form, at max_steps 1000:
    under the spec and under the readings diffrax demonstrably follows (or that only move the last
    bits) the printed value stays below the whole ensemble; only the two readings that contradict
    diffrax's published loop -- the error norm without the hidden state, max_steps counting accepted
    steps only -- put it inside the ensemble's lower tail.  The cause of the gap is unresolved."""
    printed = DYNAMIC_PINS[name][2]
    for alt in ("eo6", "fsal_t1", "dtmin_attempt", "interp_t0"):
        ens = _dyn_ensemble(name, 1000, n_ulp=8, n_box=16, dp_alt=DP_ALT[alt])
        assert printed < ens.min(), (name, alt, ens.min())
    for alt in ("norm_x", "maxsteps_acc"):
        ens = _dyn_ensemble(name, 1000, n_ulp=16, n_box=32, dp_alt=DP_ALT[alt])
        assert ens.min() <= printed + 0.5 and printed <= ens.mean(), (name, alt, ens.min(), ens.mean())


@pytest.mark.gpu
def test_gpu_dynamic_notebook_pins_bitexact():
    """The pinned DynamicPolicy candidates (central + rounding-box draws) through
    GeneticProgramming.evaluate_population on the GPU at the notebook's max_steps and at 4000:
    bit-exact with the oracle, so the ensemble statements above hold for the HIP path."""
    for ms in (1000, 4000):
        env, lib, ff, data, variables = dynamic_notebook(ms)
        d = ff.prepare(data)
        pop = np.concatenate([np.stack([_dyn_candidate(lib, make, c) for make, c, _ in DYNAMIC_PINS.values()]),
                              *[_dyn_box(lib, make, c, 7) for make, c, _ in DYNAMIC_PINS.values()]])
        pop = pop[:pop.shape[0] // 2 * 2]
        strategy = _gp(CONTROL_OPS, variables, [2, 1], ff, pop.shape[0])
        fit, _ = strategy.evaluate_population(pop[None], data)
        ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
        assert bits_equal(fit[0], ref), ms
