"""Coefficient optimisation (gp.py:418-473).

CPU: the oracle's forward-mode gradient (oracle/mtgp_oracle.c oracle_sr_grad) is pinned to the
complex-step derivative of an independent float64 restatement (d f / d c = Im f(c + i e) / e,
exact to rounding for the analytic + - * / sin cos RK4 chain); its loss equals the evaluator's
fitness bit for bit; the host transform (coefficient rows -> parameter slots) keeps every tree's
value; the Adam restatement matches optax's update rule; the optimise loop keeps the reference's
best-epoch semantics.  GPU: mtgp_sr_grad is bit-exact with the oracle, and
GeneticProgramming.evaluate_population with coefficient_optimisation=True reproduces a CPU run of
the same loop (oracle gradients + the same Adam) bit for bit.
"""
import numpy as np
import pytest

import multitreegp_amd as mt
from multitreegp_amd import coefficients as co
import np_reference as npr
from oracle import oracle as orc

from helpers import SR_OPS, bits_equal, mismatch_report, oracle_model, oracle_rollouts, sr_setup, tree_from_expr


# ------------------------------------------------------- independent complex-step restatement
def _eval_tree_c(tree, lib, data, prow, eps):
    """gp.py:356-388 over complex values: the value-column entry of row `prow` carries i*eps."""
    N = tree.shape[0]
    val = tree[:, 3].astype(np.complex128)
    if prow >= 0:
        val[prow] += 1j * eps

    def idx(v):
        j = int(v) if np.isfinite(v) else 0
        j = j + N if j < 0 else j
        return min(max(j, 0), N - 1)

    for i in range(N):
        f, a, b, c = tree[i]
        x, y = val[idx(a)], val[idx(b)]
        if f == 1:
            v = complex(c) + (1j * eps if i == prow else 0)
        else:
            k = min(max(int(f) if np.isfinite(f) else 0, 0), lib.n_funcs - 1)
            if k < 2:
                v = 0.0
            elif k >= lib.var_start:
                v = data[min(k - lib.var_start, len(data) - 1)]
            else:
                v = {"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "/": lambda: x / y,
                     "sin": lambda: np.sin(x), "cos": lambda: np.cos(x)}[lib.node_to_string[k]]()
        val[i] = v
    return val[N - 1]


def _sr_loss_c(cand, lib, d, prow_t, prow_i, eps=1e-30, euler=False):
    """SR_evaluator.__call__ (sr.py:30-45) over complex numbers: RK4 / Euler, MSE, NaN -> max, mean, clip."""
    x0, ys = d["x0"].astype(np.float64), np.transpose(d["ys_true"], (2, 0, 1)).astype(np.float64)  # [R, S, nv]
    R, nv = x0.shape
    h, ts = float(np.float32(d["h"])), d["ts"]

    def rhs(t, s):
        return np.array([_eval_tree_c(cand[q], lib, s, prow_i if q == prow_t else -1, eps) for q in range(nv)])

    fits = []
    with np.errstate(all="ignore"):
        for r in range(R):  # diffrax ConstantStepSize + SaveAt(ts) (np_reference.cs_solve) over complex numbers
            saved = npr.cs_solve(rhs, x0[r].astype(np.complex128), ts, h, "euler" if euler else "rk4", np.complex128)
            f = np.sum((saved - ys[r]) ** 2) / ts.shape[0]
            fits.append(f if np.isfinite(f.real) else complex(1e5))
    m = np.mean(fits)
    return m if 0 < m.real < 1e5 else complex(np.clip(m.real, 0, 1e5))


def _setup(P=12, R=4, euler=False, seed=3, n_var=2):
    env, lib, ff, data, pop = sr_setup(P=P, R=R, n_save=9, save_every=2, h=0.05, depth=4, N=20, seed=seed,
                                       n_var=n_var)
    if euler:
        ff = mt.SREvaluator(solver=mt.Euler(), dt0=0.05)
    d = ff.prepare(data)
    d["h"] = ff.dt0
    return lib, ff, data, d, pop


@pytest.mark.parametrize("euler", [False, True])
def test_oracle_loss_is_the_fitness(euler):
    lib, ff, data, d, pop = _setup(euler=euler)
    loss, grad, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(loss, ref)
    assert sum(len(r) for r in rows) > 10


@pytest.mark.parametrize("euler", [False, True])
def test_oracle_gradient_matches_complex_step(euler):
    """float32 forward mode vs the float64 complex-step derivative of an independent restatement,
    on every coefficient of candidates whose loss is finite and unclipped."""
    lib, ff, data, d, pop = _setup(euler=euler)
    loss, grad, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    rel, checked, ill = [], 0, 0
    for p in range(pop.shape[0]):
        if not (0 < loss[p] < 1e4):
            continue
        base = _sr_loss_c(pop[p], lib, d, -1, -1, euler=euler)
        checked += 1
        if not abs(base.real - loss[p]) <= 1e-3 * abs(loss[p]) + 1e-5:
            ill += 1  # float32 and float64 solves diverge (e.g. division by a vanishing subexpression):
            continue  # the float64 derivative says nothing about the float32 loss there
        for k, (t, i) in enumerate(rows[p]):
            g64 = _sr_loss_c(pop[p], lib, d, int(t), int(i), euler=euler).imag / 1e-30
            rel.append(abs(grad[p, k] - g64) / (abs(g64) + 1e-6 * (1 + abs(loss[p]))))
    assert checked >= 4 and ill <= checked // 4, (checked, ill)
    rel = np.array(rel)
    # float32 vs float64: ~1e-7 for well-conditioned candidates; a candidate dividing by a
    # near-zero subexpression shares one ~1 % rounding factor over all its coefficients
    assert rel.size >= 8 and np.median(rel) < 1e-5 and np.mean(rel < 1e-4) >= 0.75 and rel.max() < 0.02, rel


def test_oracle_gradient_of_a_known_fit():
    """dx0 = x1, dx1 = c*x0 around the Van der Pol data: the gradient in c agrees in sign and
    size with a central difference of the oracle's own float32 loss."""
    env, lib, ff, data, _ = sr_setup(P=2, R=4, n_save=11, save_every=2, h=0.05, N=20)
    d = ff.prepare(data)

    def cand(c):
        return np.stack([tree_from_expr("x1", lib, 20), tree_from_expr(("*", c, "x0"), lib, 20)])[None]

    loss, grad, _ = orc.sr_grad(oracle_model(ff, d), cand(-0.8), lib, oracle_rollouts(d))
    e = 1e-2
    up = orc.evaluate(oracle_model(ff, d), cand(-0.8 + e), lib, oracle_rollouts(d))["fitness"][0]
    dn = orc.evaluate(oracle_model(ff, d), cand(-0.8 - e), lib, oracle_rollouts(d))["fitness"][0]
    fd = (up - dn) / (2 * e)
    assert abs(grad[0, 0] - fd) <= 0.02 * abs(fd) + 1e-4


def test_parameterise_keeps_tree_values():
    """The host transform (coefficient rows -> variable rows on slots n_var + k, opcode clamp,
    variable clamp) leaves every tree's value unchanged, garbage arrays included."""
    from multitreegp_amd.sampling import sample_population
    lib = mt.NodeLibrary(SR_OPS, [["x0", "x1"]], [2])
    rng = np.random.default_rng(0)
    pop = sample_population(4, lib, 20, 1, max_init_depth=5, max_nodes=20)[0]
    garbage = rng.normal(0, 4, size=(8, 2, 20, 4)).astype(np.float32)
    garbage[..., 0] = rng.integers(-2, lib.n_funcs + 6, size=garbage.shape[:3]).astype(np.float32)
    garbage[..., 0][rng.random(garbage.shape[:3]) < 0.2] = 1.0
    pop = np.concatenate([pop, garbage])
    rows = co.coefficient_rows(pop)
    n_data = 2
    tpop, theta, nparam, K, libs = co.parameterise(pop, rows, lib, n_data, 0, 64)
    fn = np.frombuffer(bytes(libs.fn), np.int8)[: libs.n_funcs]
    for b in range(pop.shape[0]):
        x = rng.normal(size=2).astype(np.float32)
        data = np.concatenate([x, theta[b]]).astype(np.float32)
        for t in range(2):
            v0 = orc.eval_tree(pop[b, t], lib.fn_codes, lib.n_funcs, lib.var_start, x)
            v1 = orc.eval_tree(tpop[b, t], fn, libs.n_funcs, libs.var_start, data)
            assert bits_equal(v0, v1), (b, t)
    assert K == max(len(r) for r in rows) and list(nparam) == [len(r) for r in rows]


def test_adam_matches_optax_rule():
    """optax.adam update rule, float64 textbook vs the float32 restatement over 20 steps."""
    rng = np.random.default_rng(1)
    opt = co.adam(0.001, 0.9, 0.999)
    x = rng.normal(size=7).astype(np.float32)
    st = opt.init(x)
    m = v = np.zeros(7)
    x64 = x.astype(np.float64)
    for t in range(1, 21):
        g = rng.normal(size=7).astype(np.float32)
        u, st = opt.update(g, st, x)
        x = x + u
        m = 0.9 * m + 0.1 * g
        v = 0.999 * v + 0.001 * g.astype(np.float64) ** 2
        x64 = x64 - 0.001 * (m / (1 - 0.9 ** t)) / (np.sqrt(v / (1 - 0.999 ** t)) + 1e-8)
    np.testing.assert_allclose(x, x64, rtol=1e-5, atol=1e-6)
    # the first step moves every coordinate by -lr * sign(g)
    st = opt.init(np.zeros(3, np.float32))
    u, _ = opt.update(np.array([2.0, -3.0, 0.0], np.float32), st)
    np.testing.assert_allclose(u, [-0.001, 0.001, 0.0], rtol=1e-5)


class _QuadraticOptimiser(co.CoefficientOptimiser):
    """the optimise loop with an injected loss: sum over coefficients of (c - 3)^2"""

    def __init__(self):
        pass

    def loss_and_grad(self, candidates, data, rows=None):
        rows = co.coefficient_rows(candidates) if rows is None else rows
        vals = [c[r[:, 0], r[:, 1], 3] for c, r in zip(candidates, rows)]
        loss = np.array([np.sum((v - 3.0) ** 2) for v in vals], np.float32)
        return loss, [(2 * (v - 3.0)).astype(np.float32) for v in vals]


def test_optimise_loop_semantics():
    """gp.py:454-473: epoch e evaluates the candidates BEFORE its update; the result is the
    first minimum over the epochs and the candidate it was computed on."""
    lib = mt.NodeLibrary(SR_OPS, [["x0", "x1"]], [2])
    c = np.stack([tree_from_expr(("+", 1.0, "x0"), lib, 10), tree_from_expr(("*", 2.5, "x1"), lib, 10)])
    cands = np.stack([c, c])
    cands[1, 0, 8, 3] = 3.0  # second candidate: first coefficient already optimal
    opt = _QuadraticOptimiser()
    fit, out = opt.optimise(cands, None, 5, co.adam(0.5, 0.9, 0.999))
    # candidate 0: moving towards 3 each epoch -> the best is the last evaluated epoch (4 updates)
    assert fit[0] < np.sum((np.array([1.0, 2.5]) - 3) ** 2)
    assert np.isclose(fit[0], np.sum((out[0][[0, 1], [8, 8], 3] - 3.0) ** 2))
    # the structure is untouched, only coefficient values move
    assert np.array_equal(out[:, :, :, :3], cands[:, :, :, :3])
    # epoch-0 loss is the unmodified candidate's loss when nothing improves
    fit2, out2 = opt.optimise(np.stack([cands[1]]), None, 1)
    assert np.array_equal(out2[0], cands[1])


def test_coefficient_optimisation_config_checks():
    lib_ops, vl = SR_OPS, [["x0", "x1"]]
    ff = mt.SREvaluator(solver=mt.RK4(), dt0=0.05)
    with pytest.raises(AssertionError):
        mt.GeneticProgramming(20, 20, ff, lib_ops, vl, [2], coefficient_optimisation=True, gradient_steps=0,
                              verbose=False)
    # SR with the adaptive solve: mtgp_sr_grad's Dopri5 kernel (step sizes held at their primal values)
    ffd = mt.SREvaluator(solver=mt.Dopri5(), dt0=0.05, stepsize_controller=mt.PIDController(1e-4, 1e-4))
    mt.GeneticProgramming(20, 20, ffd, lib_ops, vl, [2], coefficient_optimisation=True, verbose=False)
    # the control evaluators with a fixed-step solver are differentiated too (mtgp_ctl_grad)
    from helpers import CONTROL_OPS
    env = mt.Acrobot(0.0, 0.0)
    dyn = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.RK4())
    mt.GeneticProgramming(20, 20, dyn, CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]], [2, 1],
                          coefficient_optimisation=True, verbose=False)
    st = mt.FeedforwardEvaluator(mt.HarmonicOscillator(0.0, 0.0), 0.05, solver=mt.Euler())
    mt.GeneticProgramming(20, 20, st, CONTROL_OPS, [["y1", "y2", "tar1"]], [1], coefficient_optimisation=True,
                          verbose=False)
    # ... and with Dopri5 + PID (step sizes held at their primal values)
    dynd = mt.DynamicEvaluator(env, 2, 0.05, solver=mt.Dopri5(), stepsize_controller=mt.PIDController(1e-4, 1e-4))
    mt.GeneticProgramming(20, 20, dynd, CONTROL_OPS, [["y1", "y2", "y3", "y4", "a1", "a2", "u"], ["a1", "a2"]],
                          [2, 1], coefficient_optimisation=True, verbose=False)


class _GlobalNormOptimiser:
    """an optimiser whose update couples every element it is given (global-norm scaling)"""

    def init(self, params):
        return 0

    def update(self, g, state, params=None):
        g = np.asarray(g, np.float32)
        n = np.float32(np.sqrt(np.sum(g.astype(np.float64) ** 2)) + 1e-12)
        return (-np.float32(0.1) * g / n).astype(np.float32), state + 1


def test_optimiser_state_per_candidate():
    """gp.py vmaps optimiser.init / update over the candidates, so an optimiser with
    cross-element state never couples two candidates: optimising a batch equals optimising each
    candidate alone."""
    lib = mt.NodeLibrary(SR_OPS, [["x0", "x1"]], [2])
    c = np.stack([tree_from_expr(("+", 1.0, "x0"), lib, 10), tree_from_expr(("*", 2.5, "x1"), lib, 10)])
    cands = np.stack([c, c, c])
    cands[1, 0, 8, 3] = 7.0
    cands[2, 1, 8, 3] = -4.0
    opt = _QuadraticOptimiser()
    fit, out = opt.optimise(cands, None, 4, _GlobalNormOptimiser())
    for b in range(3):
        f1, o1 = opt.optimise(cands[b: b + 1], None, 4, _GlobalNormOptimiser())
        assert fit[b] == f1[0] and np.array_equal(out[b], o1[0])


# ------------------------------------------------------------------- SR with Dopri5 + PID
def _setup_dp(P=12, R=4, seed=3, n_var=2, tol=1e-6):
    env, lib, ff, data, pop = sr_setup(P=P, R=R, n_save=9, save_every=2, h=0.05, depth=4, N=20, seed=seed,
                                       n_var=n_var, solver=(tol, tol, 0.001, 500))
    return lib, ff, data, ff.prepare(data), pop


def test_oracle_dopri5_loss_is_the_fitness():
    lib, ff, data, d, pop = _setup_dp()
    loss, grad, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(loss, ref), mismatch_report(loss, ref, "loss")
    assert sum(len(r) for r in rows) > 10


def test_oracle_dopri5_gradient_matches_central_differences():
    """The Dopri5 sensitivities hold the step sizes at their primal values (oracle
    sr_rollout_dual_dp; diffrax's PIDController stops their gradient the same way); a central
    difference of the oracle's own float32 loss also moves the controller's step sizes, by terms
    of the order of the tolerance.  Well-conditioned candidates
    (finite, unclipped loss; forward and backward differences within 2 % of each other) agree to a
    few 1e-3."""
    lib, ff, data, d, pop = _setup_dp(P=24, seed=3)
    m, ro = oracle_model(ff, d), oracle_rollouts(d)
    loss, grad, rows = orc.sr_grad(m, pop, lib, ro)
    rel = []
    for p in range(pop.shape[0]):
        if not (0 < loss[p] < 1e4):
            continue
        for k, (t, i) in enumerate(rows[p][:4]):
            c = pop[p: p + 1].copy()
            e = np.float32(1e-3 * max(1.0, abs(float(c[0, t, i, 3]))))
            base = c[0, t, i, 3]
            c[0, t, i, 3] = base + e
            up = orc.evaluate(m, c, lib, ro)["fitness"][0]
            c[0, t, i, 3] = base - e
            dn = orc.evaluate(m, c, lib, ro)["fitness"][0]
            fwd, bwd = (up - loss[p]) / e, (loss[p] - dn) / e
            if not abs(fwd - bwd) <= 0.02 * (abs(fwd) + abs(bwd)) + 1e-4:
                continue  # the step sequence (or the float32 loss) is not smooth here
            fd = (up - dn) / (2 * e)
            rel.append(abs(grad[p, k] - fd) / (abs(fd) + 1e-3 * (1 + abs(loss[p]))))
    rel = np.array(rel)
    assert rel.size >= 20 and np.median(rel) < 5e-3 and np.mean(rel < 3e-2) >= 0.85, np.sort(rel)


def test_oracle_dopri5_gradient_unfiltered_central_difference_error():
    """the same comparison WITHOUT the forward / backward agreement filter, over every
    finite, unclipped candidate and coefficient, so the size of the dropped controller (dt) term is
    measured rather than filtered away.  The numbers are reported (-s) and bounded loosely: the
    float32 central difference itself is noisy where the accept / reject sequence changes inside
    +-e, so the bound is on the bulk, not on every coefficient."""
    lib, ff, data, d, pop = _setup_dp(P=24, seed=3)
    m, ro = oracle_model(ff, d), oracle_rollouts(d)
    loss, grad, rows = orc.sr_grad(m, pop, lib, ro)
    rel = []
    for p in range(pop.shape[0]):
        if not (0 < loss[p] < 1e4):
            continue
        for k, (t, i) in enumerate(rows[p][:4]):
            c = pop[p: p + 1].copy()
            e = np.float32(1e-3 * max(1.0, abs(float(c[0, t, i, 3]))))
            base = c[0, t, i, 3]
            c[0, t, i, 3] = base + e
            up = orc.evaluate(m, c, lib, ro)["fitness"][0]
            c[0, t, i, 3] = base - e
            dn = orc.evaluate(m, c, lib, ro)["fitness"][0]
            if not (0 < up < 1e4 and 0 < dn < 1e4 and np.isfinite(grad[p, k])):
                continue  # the perturbed solve diverged or hit the fitness clip: no derivative to compare
            fd = (up - dn) / (2 * e)
            rel.append(abs(grad[p, k] - fd) / (abs(fd) + 1e-3 * (1 + abs(loss[p]))))
    rel = np.sort(np.array(rel))
    q = {f"p{int(x * 100)}": float(np.quantile(rel, x)) for x in (0.5, 0.75, 0.9, 1.0)}
    print("unfiltered Dopri5 gradient vs central difference, relative error over", rel.size, "coefficients:", q)
    assert rel.size >= 30 and q["p50"] < 1e-2 and q["p75"] < 0.1, q


def test_oracle_dopri5_gradient_of_a_known_fit():
    """dx0 = x1, dx1 = c*x0 on the Van der Pol data with Dopri5: sign and size of the gradient in
    c against a central difference of the oracle's loss."""
    env, lib, ff, data, _ = sr_setup(P=2, R=4, n_save=11, save_every=2, h=0.05, N=20, solver=(1e-6, 1e-6, 0.001, 500))
    d = ff.prepare(data)

    def cand(c):
        return np.stack([tree_from_expr("x1", lib, 20), tree_from_expr(("*", c, "x0"), lib, 20)])[None]

    loss, grad, _ = orc.sr_grad(oracle_model(ff, d), cand(-0.8), lib, oracle_rollouts(d))
    e = 1e-2
    up = orc.evaluate(oracle_model(ff, d), cand(-0.8 + e), lib, oracle_rollouts(d))["fitness"][0]
    dn = orc.evaluate(oracle_model(ff, d), cand(-0.8 - e), lib, oracle_rollouts(d))["fitness"][0]
    fd = (up - dn) / (2 * e)
    assert np.sign(grad[0, 0]) == np.sign(fd) and abs(grad[0, 0] - fd) < 0.05 * abs(fd), (grad[0, 0], fd)


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n_var,R", [(2, 8), (3, 5), (6, 4), (20, 3)])
def test_gpu_sr_grad_dopri5_bitexact(n_var, R):
    """mtgp_sr_grad with Dopri5 + PID (k_sr_grad_dp, 2 / 4 / 16 / 64-slot templates) vs the oracle:
    loss and every coefficient's gradient bit for bit, loss = the evaluator's fitness."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    lib, ff, data, d, pop = _setup_dp(P=24, R=R, seed=21 + n_var, n_var=n_var)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    loss, grads = opt.loss_and_grad(pop, data)
    rl, rg, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert sum(len(r) for r in rows) > 5
    assert bits_equal(loss, rl), mismatch_report(loss, rl, "loss")
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), (p, g, rg[p, : len(g)])
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit), mismatch_report(loss, fit, "fitness")

@pytest.mark.gpu
@pytest.mark.parametrize("euler", [False, True])
def test_gpu_sr_grad_bitexact(euler):
    """mtgp_sr_grad vs oracle_sr_grad: loss and every coefficient's gradient bit for bit."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    lib, ff, data, d, pop = _setup(P=40, R=8, euler=euler, seed=5)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    loss, grads = opt.loss_and_grad(pop, data)
    rl, rg, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert bits_equal(loss, rl)
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), p
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit)


@pytest.mark.gpu
@pytest.mark.parametrize("n_var,R", [(3, 5), (6, 8), (20, 3), (2, 5)])
def test_gpu_sr_grad_bitexact_wide(n_var, R):
    """The other k_sr_grad widths (n_var 3 -> 4 slots, 6 / 20 -> the 16 / 64-slot templates) and
    non-power-of-two rollout counts: loss and gradients bit for bit vs the oracle, loss = the
    evaluator's fitness."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    lib, ff, data, d, pop = _setup(P=24, R=R, seed=11 + n_var, n_var=n_var)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    loss, grads = opt.loss_and_grad(pop, data)
    rl, rg, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert sum(len(r) for r in rows) > 5
    assert bits_equal(loss, rl), mismatch_report(loss, rl, "loss")
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), p
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit), mismatch_report(loss, fit, "fitness")


@pytest.mark.gpu
def test_gpu_sr_grad_chunks():
    """More coefficients than one launch holds (cap forced to 3): the chunks give the same
    gradients as the oracle."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    lib, ff, data, d, pop = _setup(P=16, R=4, seed=7)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    opt.param_cap = lambda n_data: 3
    loss, grads = opt.loss_and_grad(pop, data)
    rl, rg, rows = orc.sr_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert max(len(r) for r in rows) > 3
    assert bits_equal(loss, rl)
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), p


@pytest.mark.gpu
@pytest.mark.parametrize("dopri5", [False, True])
def test_gpu_evaluate_population_optimises_coefficients(dopri5):
    """Generation 14 of a coefficient-optimising run (gp.py:418): the 50 best candidates get
    gradient_steps Adam steps; fitness, population and best tracking equal a CPU restatement of
    the same loop driven by the oracle's loss and gradients (RK4, and Dopri5 + PID)."""
    lib, ff, data, d, pop = _setup_dp(P=60, R=4, seed=9) if dopri5 else _setup(P=60, R=4, seed=9)
    strategy = mt.GeneticProgramming(20, 60, ff, SR_OPS, [["x0", "x1"]], [2], max_nodes=20, size_parsinomy=0.01,
                                     coefficient_optimisation=True, gradient_steps=4, verbose=False)
    strategy.current_generation = 14
    fit, newpop = strategy.evaluate_population(pop[None], data)
    model, ro = oracle_model(ff, d), oracle_rollouts(d)
    raw = orc.evaluate(model, pop, lib, ro)["fitness"]
    idx = np.argsort(raw, kind="stable")[:50]
    cands = pop[idx].copy()
    rows = co.coefficient_rows(cands)
    vals = np.concatenate([c[r[:, 0], r[:, 1], 3] for c, r in zip(cands, rows)]).astype(np.float32)
    offs = np.concatenate([[0], np.cumsum([len(r) for r in rows])])
    opt = co.adam()
    st = opt.init(vals)
    hist_c, hist_l = [], []
    for _ in range(4):
        loss, grad, _ = orc.sr_grad(model, cands, lib, ro)
        hist_c.append(cands.copy())
        hist_l.append(loss)
        g = np.concatenate([grad[b, : len(r)] for b, r in enumerate(rows)]).astype(np.float32)
        u, st = opt.update(g, st, vals)
        vals = (vals + u).astype(np.float32)
        for b, r in enumerate(rows):
            cands[b][r[:, 0], r[:, 1], 3] = vals[offs[b]: offs[b + 1]]
    Lh = np.stack(hist_l)
    best = np.argmin(Lh, axis=0)
    want_pop = pop.copy()
    want_pop[idx] = np.stack([hist_c[e][b] for b, e in enumerate(best)])
    want = raw.copy()
    want[idx] = Lh.min(axis=0)
    counts = (want_pop[..., 0] != 0).sum(axis=(1, 2)).astype(np.float32)
    want = (want + np.float32(0.01) * counts).astype(np.float32)
    assert bits_equal(newpop[0], want_pop)
    assert bits_equal(fit[0], want)
    assert strategy.best_fitnesses[14] == want.min()
    assert np.any(Lh.min(axis=0) < Lh[0])  # the optimisation improved some candidates


# ----------------------------------------------------- control evaluators (dyn.py / ff.py)
def _ctl_loss_c(cand, lib, ff, d, prow_t, prow_i, eps=1e-30):
    """Evaluator.__call__ of the dynamic / static control evaluators (dyn.py:37-118,
    ff.py:36-110) over complex float64 numbers, written from the reference text: f_obs (C = I,
    Acrobot wrap by floor-mod: real part wrapped, imaginary part kept), readout / state trees,
    drift (acrobot.py:51-72, harmonic_oscillator.py:58-69, reactor.py:60-69), clip on the real
    part, RK4 / Euler, the Event, the fitness functions (argmax on the real part), NaN -> max,
    mean, clip.  Noise-free."""
    dyn = ff.model_id == 1
    env = type(ff.env).__name__
    x0 = d["x0"].astype(np.float64)
    prm = d["params"].astype(np.float64)
    tg = d["targets"].astype(np.float64).reshape(x0.shape[0], -1)
    R, nv = x0.shape
    na = ff.state_size if dyn else 0
    no = ff.env.n_obs
    ts = d["ts"].astype(np.float32)
    h, S = float(np.float32(ff.dt0)), d["n_save"]
    solver = d.get("solver", 0)

    def tree(q, data):
        return _eval_tree_c(cand[q], lib, np.array(data, np.complex128), prow_i if q == prow_t else -1, eps)

    def clip(u, lo, hi):
        return complex(lo) if u.real < lo else (complex(hi) if u.real > hi else u)

    def obs(x):
        y = np.array(x[:no], np.complex128)
        if env == "Acrobot":
            for i in range(min(2, no)):
                y[i] = ((y[i].real + np.pi) % (2 * np.pi) - np.pi) + 1j * y[i].imag
        return y

    def drift(x, u, p, r):
        if env == "Acrobot":
            l1, l2, m1, m2 = p
            lc1, lc2, g = 0.5 * l1, 0.5 * l2, 9.81
            u = clip(u, -1, 1)
            t1, t2, td1, td2 = x
            d1 = m1 * lc1 ** 2 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * np.cos(t2)) + 2.0
            d2 = m2 * (lc2 ** 2 + l1 * lc2 * np.cos(t2)) + 1.0
            phi2 = m2 * lc2 * g * np.cos(t1 + t2 - np.pi / 2)
            phi1 = (-m2 * l1 * lc2 * td2 ** 2 * np.sin(t2) - 2 * m2 * l1 * lc2 * td1 * td2 * np.sin(t1)
                    + (m1 * lc1 + m2 * l1) * g * np.cos(t1 - np.pi / 2) + phi2)
            a2 = (u + d2 / d1 * phi1 - m2 * l1 * lc2 * td1 ** 2 * np.sin(t2) - phi2) / (m2 * lc2 ** 2 + 1.0 - d2 ** 2 / d1)
            a1 = -(d2 * a2 + phi1) / d1
            return np.array([td1, td2, a1, a2])
        if env == "HarmonicOscillator":
            w, z = p[:2]
            return np.array([x[1], -w * x[0] - z * x[1] + u])
        Vol, Cp, dHr, UA, q, Tf, Tcf, Volc = p
        Tc, T, c = x
        u = clip(u, 0, 300)
        kT = np.float64(np.float32(7.2e10)) * np.exp(float(np.float32(-72750.0 / 8.314)) / T)
        return np.array([u / Volc * (Tcf - Tc) + UA / Volc / Cp * (T - Tc),
                         q / Vol * (Tf - T) + (-dHr) / Cp * kT * c + UA / Vol / Cp * (Tc - T),
                         q / Vol * (1 - c) - kT * c])

    def rhs(s, r):
        x, a = s[:nv], s[nv:]
        y = obs(x)
        if dyn:
            u = tree(na, [0] * no + list(a) + [0] + list(tg[r]))
            da = [tree(i, list(y) + list(a) + [u] + list(tg[r])) for i in range(na)]
            return np.concatenate([drift(x, u, prm[r], r), np.array(da, np.complex128)])
        return drift(x, tree(0, list(y) + list(tg[r])), prm[r], r)

    def bad(s):
        b = not np.all(np.isfinite(s.real))
        if env == "Acrobot":
            b = b or abs(s[2].real) > 8 * np.pi or abs(s[3].real) > 18 * np.pi
        return b

    fits = []
    with np.errstate(all="ignore"):
        for r in range(R):
            s = np.concatenate([x0[r], np.zeros(na)]).astype(np.complex128)
            ev = {"prev_ok": not bad(s)}

            def event(y):  # Event(cond_fn_nan): the condition turns negative after a step
                ok = not bad(y)
                fire = ev["prev_ok"] and not ok
                ev["prev_ok"] = ok
                return fire
            # diffrax ConstantStepSize + SaveAt(ts) (np_reference.cs_solve) over complex numbers; +inf fill
            saved = list(npr.cs_solve(lambda t, y: rhs(y, r), s, ts, h, "euler" if solver == 2 else "rk4",
                                      np.complex128, event=event))
            us = []
            for sk in saved:
                y = obs(sk[:nv])
                us.append(tree(na, list(y) + list(sk[nv:]) + [0] + list(tg[r])) if dyn
                          else tree(0, list(y) + list(tg[r])))
            if env == "Acrobot":
                reach = [(-np.cos(sk[0].real) - np.cos(sk[0].real + sk[1].real)) > 1.5 for sk in saved]
                fs = int(np.argmax(reach))
                dts = np.float32(ts[1] - ts[0])
                cs = sum((0.0 if np.float32(ts[k] / dts) > fs else 0.01 * us[k] ** 2) for k in range(S))
                f = fs + (fs == 0) * S + cs
            elif env == "HarmonicOscillator":
                ud = prm[r][0] * tg[r][0]
                f = sum(0.5 * (sk[0] - tg[r][0]) ** 2 + 0.5 * (u - ud) ** 2 for sk, u in zip(saved, us))
            else:
                f = sum(0.01 * (sk[1] - tg[r][0]) ** 2 + 1e-4 * u ** 2 for sk, u in zip(saved, us))
            f = complex(f)
            fits.append(f if np.isfinite(f.real) else complex(1e4))
    m = np.mean(fits)
    return m if 0 < m.real < 1e4 else complex(np.clip(m.real, 0, 1e4))


def _ctl_setup(kind, env="acrobot", euler=False, P=10, R=3, n_steps=16, seed=5, obs_noise=0.0, dopri5=False):
    from helpers import dynamic_setup, static_setup
    solver = None
    setup = dynamic_setup if kind == "dynamic" else static_setup
    kw = dict(P=P, R=R, n_steps=n_steps, seed=seed, env=env, obs_noise=obs_noise)
    if dopri5:
        kw["solver"] = (1e-5, 1e-5, 0.002, 600)
    if kind == "dynamic":
        kw["depth"], kw["N"] = 4, 24
    e, lib, ff, data, pop = setup(**kw)
    if euler:
        ff = (mt.DynamicEvaluator(e, ff.state_size, ff.dt0, solver=mt.Euler()) if kind == "dynamic"
              else mt.FeedforwardEvaluator(e, ff.dt0, solver=mt.Euler()))
    del solver
    d = ff.prepare(data)
    return lib, ff, data, d, pop


CTL_CASES = [("dynamic", "acrobot", False, 0.0), ("dynamic", "acrobot", True, 0.0), ("static", "acrobot", False, 0.0),
             ("dynamic", "harmonic", False, 0.0), ("static", "reactor", False, 0.0),
             ("dynamic", "acrobot", False, 0.1), ("static", "reactor", True, 0.1)]


@pytest.mark.parametrize("kind,env,noise", [("dynamic", "acrobot", 0.0), ("static", "harmonic", 0.1),
                                             ("dynamic", "reactor", 0.0)])
def test_ctl_oracle_dopri5_loss_is_the_fitness(kind, env, noise):
    lib, ff, data, d, pop = _ctl_setup(kind, env, obs_noise=noise, n_steps=30, dopri5=True)
    loss, grad, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(loss, ref), mismatch_report(loss, ref, "loss")


def test_ctl_oracle_dopri5_gradient_matches_central_differences():
    """Control evaluators with Dopri5 (HarmonicOscillator, dynamic and static, with observation
    noise): the primal-step-size sensitivities vs central differences of the oracle's float32 loss
    on smooth, unclipped candidates (see the SR Dopri5 test)."""
    rel = []
    for kind in ("dynamic", "static"):
        lib, ff, data, d, pop = _ctl_setup(kind, "harmonic", P=24, obs_noise=0.1, n_steps=30, dopri5=True)
        m, ro = oracle_model(ff, d), oracle_rollouts(d)
        loss, grad, rows = orc.ctl_grad(m, pop, lib, ro)
        for p in range(pop.shape[0]):
            if not (0 < loss[p] < 1e3):
                continue
            for k, (t, i) in enumerate(rows[p][:4]):
                c = pop[p: p + 1].copy()
                e = np.float32(1e-3 * max(1.0, abs(float(c[0, t, i, 3]))))
                base = c[0, t, i, 3]
                c[0, t, i, 3] = base + e
                up = orc.evaluate(m, c, lib, ro)["fitness"][0]
                c[0, t, i, 3] = base - e
                dn = orc.evaluate(m, c, lib, ro)["fitness"][0]
                fwd, bwd = (up - loss[p]) / e, (loss[p] - dn) / e
                if not abs(fwd - bwd) <= 0.02 * (abs(fwd) + abs(bwd)) + 1e-4:
                    continue
                fd = (up - dn) / (2 * e)
                rel.append(abs(grad[p, k] - fd) / (abs(fd) + 1e-3 * (1 + abs(loss[p]))))
    rel = np.array(rel)
    assert rel.size >= 10 and np.median(rel) < 5e-3 and np.mean(rel < 3e-2) >= 0.85, np.sort(rel)


@pytest.mark.parametrize("kind,env,euler,noise", CTL_CASES)
def test_ctl_oracle_loss_is_the_fitness(kind, env, euler, noise):
    """oracle_ctl_grad's value half equals the evaluator's fitness bit for bit (every environment,
    RK4 / Euler, with observation noise)."""
    lib, ff, data, d, pop = _ctl_setup(kind, env, euler, obs_noise=noise)
    loss, grad, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    ref = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(loss, ref)
    assert sum(len(r) for r in rows) >= 5 and np.isfinite(grad).mean() > 0.5


@pytest.mark.parametrize("kind,env,euler", [("dynamic", "acrobot", False), ("dynamic", "acrobot", True),
                                            ("static", "acrobot", False), ("dynamic", "harmonic", False),
                                            ("static", "harmonic", True)])
def test_ctl_oracle_gradient_matches_complex_step(kind, env, euler):
    """float32 forward mode through the coupled control solve vs the float64 complex-step
    derivative of the independent restatement above, on every coefficient of candidates whose
    loss is finite and unclipped (the argmax step of acrobot.py:79 is piecewise constant, as in
    JAX)."""
    lib, ff, data, d, pop = _ctl_setup(kind, env, euler, P=8, R=2, n_steps=12)
    loss, grad, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    rel, checked, ill = [], 0, 0
    for p in range(pop.shape[0]):
        if not (0 < loss[p] < 1e4):
            continue
        base = _ctl_loss_c(pop[p], lib, ff, d, -1, -1)
        checked += 1
        if not abs(base.real - loss[p]) <= 1e-3 * abs(loss[p]) + 1e-4:
            ill += 1
            continue
        for k, (t, i) in enumerate(rows[p]):
            g64 = _ctl_loss_c(pop[p], lib, ff, d, int(t), int(i)).imag / 1e-30
            rel.append(abs(grad[p, k] - g64) / (abs(g64) + 1e-5 * (1 + abs(loss[p]))))
    rel = np.array(rel)
    assert checked >= 4 and ill <= checked // 4, (checked, ill)
    assert rel.size >= 6 and np.median(rel) < 1e-5 and np.mean(rel < 1e-4) >= 0.75 and rel.max() < 0.01, rel
    assert np.count_nonzero(grad) >= 4  # the coefficients do move the loss


# ------------------------------------------------------------ GPU: control evaluators
GPU_CTL_CASES = [("dynamic", "acrobot", False, 0.0, 4), ("dynamic", "acrobot", True, 0.0, 4),
                 ("static", "acrobot", False, 0.1, 4), ("dynamic", "harmonic", False, 0.0, 2),
                 ("static", "reactor", True, 0.1, 3), ("dynamic", "acrobot", False, 0.1, 2),
                 # Dopri5 + PID (k_ctl_grad's adaptive solve, step sizes held at their primal values)
                 ("dynamic", "acrobot", "dopri5", 0.0, 4), ("dynamic", "harmonic", "dopri5", 0.1, 2),
                 ("static", "reactor", "dopri5", 0.0, 3), ("static", "acrobot", "dopri5", 0.1, 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,env,euler,noise,n_obs", GPU_CTL_CASES)
def test_gpu_ctl_grad_bitexact(kind, env, euler, noise, n_obs):
    """mtgp_ctl_grad vs oracle_ctl_grad: loss and every coefficient's gradient bit for bit, every
    environment, RK4 / Euler, observation noise, n_obs < n_var; loss = the evaluator's fitness."""
    import torch
    from helpers import _ctl_solver, _mode, CONTROL_OPS
    from multitreegp_amd.engine import DeviceEngine
    from multitreegp_amd.sampling import sample_population
    cls = {"acrobot": mt.Acrobot, "harmonic": mt.HarmonicOscillator, "reactor": mt.StirredTankReactor}[env]
    e = cls(0.0, noise, n_obs=n_obs)
    ys = [f"y{i + 1}" for i in range(e.n_obs)]
    tg = [f"tar{i + 1}" for i in range(e.n_targets)]
    solver = (_ctl_solver((1e-5, 1e-5, 0.002, 600)) if euler == "dopri5"
              else dict(solver=mt.Euler()) if euler else _ctl_solver(None))
    if kind == "dynamic":
        lib = mt.NodeLibrary(CONTROL_OPS, [ys + ["a1", "a2", "u"] + tg, ["a1", "a2"] + tg], [2, 1])
        ff = mt.DynamicEvaluator(e, 2, 0.05, **solver)
    else:
        lib = mt.NodeLibrary(CONTROL_OPS, [ys + tg], [1])
        ff = mt.FeedforwardEvaluator(e, 0.05, **solver)
    data = mt.control_data(e, 6, 0.05, None, seed=4, n_steps=30, mode=_mode(env))
    pop = sample_population(8, lib, 30, 1, max_init_depth=5, max_nodes=24)[0]
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt = co.CoefficientOptimiser(eng)
    loss, grads = opt.loss_and_grad(pop, data)
    d = eng.prepare_data(data)
    rl, rg, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert bits_equal(loss, rl)
    for p, g in enumerate(grads):
        assert bits_equal(g, rg[p, : len(g)]), (p, g, rg[p, : len(g)])
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit)
    if (loss < ff.max_fitness).sum() >= 3:  # (random reactor policies mostly diverge: max_fitness, no gradient)
        assert sum(np.count_nonzero(g) for g in grads) > 5


@pytest.mark.gpu
def test_gpu_evaluate_population_optimises_control_coefficients():
    """gp.py:418-422 with the dynamic Acrobot evaluator: generation 14's 50 best candidates get
    gradient_steps Adam steps on their coefficients through mtgp_ctl_grad; fitness and population
    equal a CPU restatement of the loop driven by the oracle's loss and gradients."""
    from helpers import dynamic_setup
    e, lib, ff, data, pop = dynamic_setup(P=60, R=4, n_steps=30, depth=4, N=24, seed=12)
    strategy = mt.GeneticProgramming(20, 60, ff, lib.operator_list, lib.variable_list, lib.layer_sizes, max_nodes=24,
                                     size_parsinomy=0.01, coefficient_optimisation=True, gradient_steps=3,
                                     verbose=False)
    strategy.current_generation = 14
    fit, newpop = strategy.evaluate_population(pop[None], data)
    d = ff.prepare(data)
    model, ro = oracle_model(ff, d), oracle_rollouts(d)
    raw = orc.evaluate(model, pop, lib, ro)["fitness"]
    idx = np.argsort(raw, kind="stable")[:50]
    cands = pop[idx].copy()
    rows = co.coefficient_rows(cands)
    opt = co.adam()
    states = [opt.init(c[r[:, 0], r[:, 1], 3]) for c, r in zip(cands, rows)]
    hist_c, hist_l = [], []
    for _ in range(3):
        loss, grad, _ = orc.ctl_grad(model, cands, lib, ro)
        hist_c.append(cands.copy())
        hist_l.append(loss)
        for b, r in enumerate(rows):
            v = cands[b][r[:, 0], r[:, 1], 3]
            u, states[b] = opt.update(grad[b, : len(r)], states[b], v)
            cands[b][r[:, 0], r[:, 1], 3] = (v + u).astype(np.float32)
    L = np.stack(hist_l)
    best = np.argmin(L, axis=0)
    want_pop = pop.copy()
    want_pop[idx] = np.stack([hist_c[e_][b] for b, e_ in enumerate(best)])
    want_raw = raw.copy()
    want_raw[idx] = L.min(axis=0)
    counts = (want_pop[..., 0] != 0).sum(axis=(1, 2)).astype(np.float32)
    want = (want_raw + np.float32(0.01) * counts).astype(np.float32)
    assert bits_equal(fit.reshape(-1), want)
    assert np.array_equal(newpop.reshape(pop.shape), want_pop)
    assert (L.min(axis=0) < L[0]).any()  # the optimisation improved some candidate


def test_data_limits_raise_at_generation_0():
    """coefficient optimisation's data limit (at most 64 rollouts) raises at the first
    evaluate_population, not at generation 14 when the first optimisation runs (gp.py:418).
    Host-side check: no GPU needed, every rank raises together.  (Acrobot ts off the one-pass
    mask is differentiated since round 5: test_gpu_ctl_grad_offset_ts_bitexact.)"""
    from helpers import CONTROL_OPS, dynamic_setup
    e, lib, ff, data, pop = dynamic_setup(P=8, R=100, n_steps=10, depth=3, N=16, seed=2)
    gp = mt.GeneticProgramming(20, 8, ff, CONTROL_OPS, lib.variable_list, lib.layer_sizes, max_nodes=16,
                               migration_percentage=0.5, elite_percentage=0.0, coefficient_optimisation=True,
                               verbose=False)
    assert gp.current_generation == 0
    with pytest.raises(NotImplementedError, match="64 rollouts"):
        gp.evaluate_population(pop[None], data)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,env,solver,noise,ext", [
    ("dynamic", "acrobot", "rk4", 0.0, False), ("dynamic", "acrobot", "dopri5", 0.0, False),
    ("static", "reactor", "euler", 0.1, False), ("dynamic", "harmonic", "rk4", 0.1, True),
    ("static", "acrobot", "dopri5", 0.0, True)])
def test_gpu_ctl_grad_dual_jit_matches_interpreter(kind, env, solver, noise, ext):
    """mtgp_ctl_grad_jit (the programs as dual-number machine code, csrc/mtgp_jit_dual.h) vs the
    dual interpreter (mtgp_ctl_grad): loss and every gradient bit for bit, every program of the
    launch translated (info[0] == 0) and the code in the buffer (info[1] <= its size) -- i.e. the
    JIT path is the one that ran; the extended operators (/, exp, log, sqrt, tanh, abs) included."""
    import torch
    from helpers import _ctl_solver, _mode, CONTROL_OPS
    from multitreegp_amd.engine import DeviceEngine
    from multitreegp_amd.sampling import sample_population
    cls = {"acrobot": mt.Acrobot, "harmonic": mt.HarmonicOscillator, "reactor": mt.StirredTankReactor}[env]
    e = cls(0.0, noise)
    ys = [f"y{i + 1}" for i in range(e.n_obs)]
    tg = [f"tar{i + 1}" for i in range(e.n_targets)]
    ops = CONTROL_OPS + ([("/", None, 2, 0.1), ("exp", None, 1, 0.05), ("log", None, 1, 0.05),
                          ("sqrt", None, 1, 0.05), ("tanh", None, 1, 0.05), ("abs", None, 1, 0.05)] if ext else [])
    sv = {"rk4": _ctl_solver(None), "euler": dict(solver=mt.Euler()),
          "dopri5": _ctl_solver((1e-5, 1e-5, 0.002, 600))}[solver]
    if kind == "dynamic":
        lib = mt.NodeLibrary(ops, [ys + ["a1", "a2", "u"] + tg, ["a1", "a2"] + tg], [2, 1])
        ff = mt.DynamicEvaluator(e, 2, 0.05, **sv)
    else:
        lib = mt.NodeLibrary(ops, [ys + tg], [1])
        ff = mt.FeedforwardEvaluator(e, 0.05, **sv)
    data = mt.control_data(e, 6, 0.05, None, seed=9, n_steps=30, mode=_mode(env))
    pop = sample_population(13, lib, 30, 1, max_init_depth=5, max_nodes=24)[0]
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    opt_j = co.CoefficientOptimiser(eng, jit=True)
    lj, gj = opt_j.loss_and_grad(pop, data)
    info = opt_j.last_jit_info.cpu().numpy()
    assert info[0] == 0 and 0 < info[1] <= eng._grad_code[1], info
    li, gi = co.CoefficientOptimiser(eng, jit=False).loss_and_grad(pop, data)
    assert sum(len(g) for g in gj) > 5
    assert bits_equal(lj, li), mismatch_report(lj, li, "loss")
    for p, (a, b) in enumerate(zip(gj, gi)):
        assert bits_equal(a, b), (p, a, b)


OFFSET_CASES = [("dynamic", None, 1.0), ("dynamic", None, -0.35), ("static", None, 2.5), ("static", None, 0.07),
                ("dynamic", (1e-5, 1e-5, 0.002, 600), 1.5), ("dynamic", (1e-5, 1e-5, 0.002, 600), -0.4)]


def _offset_case(kind, solver, t0, P=10, R=8):
    from helpers import dynamic_setup, static_setup
    from test_gpu_acrobot_mask import _swing_data
    setup = dynamic_setup if kind == "dynamic" else static_setup
    kw = dict(P=P, R=R, n_steps=40, seed=13, solver=solver)
    if kind == "dynamic":
        kw["depth"], kw["N"] = 4, 24
    env, lib, ff, data, pop = setup(**kw)
    data = _swing_data(data, t0, seed=int(abs(t0) * 100) + 5)
    return lib, ff, data, pop


@pytest.mark.parametrize("kind,solver,t0", OFFSET_CASES[:3])
def test_ctl_oracle_loss_is_the_fitness_offset_ts(kind, solver, t0):
    """The oracle's dual Acrobot fitness on a grid off the one-pass form (the general mask,
    acrobot.py:82) equals its evaluator fitness bit for bit."""
    from multitreegp_amd.evaluators import acrobot_mask
    lib, ff, data, pop = _offset_case(kind, solver, t0)
    assert acrobot_mask(data[1]) is not None
    d = ff.prepare(data)
    rl, rg, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    fit = orc.evaluate(oracle_model(ff, d), pop, lib, oracle_rollouts(d))["fitness"]
    assert bits_equal(rl, fit), mismatch_report(rl, fit, "loss")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,solver,t0", OFFSET_CASES)
def test_gpu_ctl_grad_offset_ts_bitexact(kind, solver, t0):
    """Coefficient optimisation on Acrobot grids off the one-pass mask (MtgpRollouts.fit_kof: the
    kept cost prefix behind the first success for positive offsets, running into the +inf fill for
    negative ones): loss and every gradient bit for bit vs the oracle, loss = the evaluator's
    fitness; RK4 and Dopri5, dynamic and static; JIT and interpreter alike."""
    import torch
    from multitreegp_amd.engine import DeviceEngine
    lib, ff, data, pop = _offset_case(kind, solver, t0)
    eng = DeviceEngine(ff, lib, 0.0, torch.device("cuda", 0))
    d = eng.prepare_data(data)
    assert d.get("fit_kof") is not None
    rl, rg, rows = orc.ctl_grad(oracle_model(ff, d), pop, lib, oracle_rollouts(d))
    assert sum(len(r) for r in rows) > 5
    for jit in (True, False):
        loss, grads = co.CoefficientOptimiser(eng, jit=jit).loss_and_grad(pop, data)
        assert bits_equal(loss, rl), mismatch_report(loss, rl, "loss")
        for p, g in enumerate(grads):
            assert bits_equal(g, rg[p, : len(g)]), (jit, p, g, rg[p, : len(g)])
    fit = eng.evaluate(torch.from_numpy(pop).cuda(), data)["fitness"].cpu().numpy()
    assert bits_equal(loss, fit), mismatch_report(loss, fit, "fitness")
