"""Independent float64 numpy restatement of the reference hot path (test helper).

Written directly from the reference source text, sharing no code with oracle/mtgp_oracle.c or
the product: row-order tree interpretation (gp.py:356-388), Acrobot observation/drift
(control_environment_base.py:43-48, acrobot.py:29-72), the dynamic / feedforward / SR drifts
(dynamic_evaluate.py:107-118, feedforward_evaluate.py:104-110, SR_evaluator.py:85-88) and a
textbook RK4.  float64 + numpy's libm sin/cos, so agreement with the fp32 oracle is to a
tolerance, which pins the oracle's SEMANTICS (layouts, operand order, zero slots, wraps)."""
import numpy as np


def eval_tree(tree, lib, data):
    tree = np.asarray(tree, np.float64)
    N = tree.shape[0]
    val = tree[:, 3].copy()

    def idx(v):
        j = int(v) if np.isfinite(v) else 0
        if j < 0:
            j += N
        return min(max(j, 0), N - 1)

    with np.errstate(all="ignore"):
        for i in range(N):
            f, a, b, c = tree[i]
            x, y = val[idx(a)], val[idx(b)]
            if f == 1:
                v = c
            else:
                k = min(max(int(f), 0), lib.n_funcs - 1)
                name = lib.node_to_string.get(k)
                if k < 2:
                    v = 0.0
                elif k >= lib.var_start:
                    v = data[min(k - lib.var_start, len(data) - 1)]
                else:
                    v = {"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "/": lambda: x / y,
                         "sin": lambda: np.sin(x), "cos": lambda: np.cos(x), "exp": lambda: np.exp(x),
                         "log": lambda: np.log(x), "sqrt": lambda: np.sqrt(x), "tanh": lambda: np.tanh(x),
                         "abs": lambda: np.abs(x)}[name]()
            val[i] = v
    return val[N - 1]


def obs_noise(key, t, W, partitionable=False):
    """normal(fold_in(key, bitcast_i32(t)), (n,)) @ W (control_environment_base.py:43-48):
    threefry words from the host restatement, the normal map in float64 with scipy's erfinv
    (independent of the fp32 spec's Giles polynomial)."""
    from scipy.special import erfinv
    from multitreegp_amd import prng
    old = prng.threefry_partitionable()
    prng.set_threefry_partitionable(partitionable)
    try:
        k = prng.fold_in(key, int(np.array(t, np.float32).view(np.uint32)))
        bits = prng.random_bits(k, (W.shape[0],))
    finally:
        prng.set_threefry_partitionable(old)
    f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32).astype(np.float64) - 1.0
    lo = float(np.nextafter(np.float32(-1), np.float32(0)))
    u = np.maximum(lo, f * 2.0 + lo)
    return (np.sqrt(2.0) * erfinv(u)) @ np.asarray(W, np.float64)


def acro_f_obs(x, noise=None):
    y = np.array(x, np.float64)  # C = I
    if noise is not None:
        y = y + noise
    y[0] = np.remainder(y[0] + np.pi, 2 * np.pi) - np.pi
    y[1] = np.remainder(y[1] + np.pi, 2 * np.pi) - np.pi
    return y


def acro_drift(x, u, l1=1.0, l2=1.0, m1=1.0, m2=1.0):
    control = np.clip(u, -1, 1)
    t1, t2, td1, td2 = x
    lc1, lc2, moi1, moi2, g = 0.5 * l1, 0.5 * l2, 1.0, 1.0, 9.81
    d1 = m1 * lc1 ** 2 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * np.cos(t2)) + moi1 + moi2
    d2 = m2 * (lc2 ** 2 + l1 * lc2 * np.cos(t2)) + moi2
    phi2 = m2 * lc2 * g * np.cos(t1 + t2 - np.pi / 2)
    phi1 = -m2 * l1 * lc2 * td2 ** 2 * np.sin(t2) - 2 * m2 * l1 * lc2 * td1 * td2 * np.sin(t1) \
        + (m1 * lc1 + m2 * l1) * g * np.cos(t1 - np.pi / 2) + phi2
    a2 = (control + d2 / d1 * phi1 - m2 * l1 * lc2 * td1 ** 2 * np.sin(t2) - phi2) / (m2 * lc2 ** 2 + moi2 - d2 ** 2 / d1)
    a1 = -(d2 * a2 + phi1) / d1
    return np.array([td1, td2, a1, a2])


def dyn_rhs(cand, lib, s, state_size, params=(1, 1, 1, 1), noise=None):
    x, a = s[:4], s[4:]
    y = acro_f_obs(x, noise)
    u = eval_tree(cand[state_size], lib, np.concatenate([np.zeros(4), a, np.zeros(1)]))
    dx = acro_drift(x, u, *params)
    d = np.concatenate([y, a, [u]])
    da = [eval_tree(cand[i], lib, d) for i in range(state_size)]
    return np.concatenate([dx, da])


def ff_rhs(cand, lib, s, params=(1, 1, 1, 1), noise=None):
    return acro_drift(s, eval_tree(cand[0], lib, acro_f_obs(s, noise)), *params)


def sr_rhs(cand, lib, s):
    return np.array([eval_tree(cand[i], lib, s) for i in range(len(s))])


def rk4_t(rhs, s0, t0, h, n):
    """Textbook RK4 of a time-dependent rhs(t, s).  The stage TIMES are float32 like the
    kernel's (t = t0 + f32(i) * h; t + h/2, t + h/2, t + h): the observation noise is keyed on
    their bit patterns (cbase.py:45)."""
    s = np.array(s0, np.float64)
    out = [s.copy()]
    f = np.float32
    hf = f(h)
    with np.errstate(all="ignore"):
        for i in range(n):
            t = f(f(t0) + f(i) * hf)
            th, t1 = f(t + f(hf * f(0.5))), f(t + hf)
            k1 = rhs(t, s)
            k2 = rhs(th, s + 0.5 * h * k1)
            k3 = rhs(th, s + 0.5 * h * k2)
            k4 = rhs(t1, s + h * k3)
            s = s + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
            out.append(s.copy())
    return np.array(out)


def cs_grid(ts, dt0, max_steps=None):
    """diffrax.ConstantStepSize's step grid through diffeqsolve(t0=ts[0], t1=ts[-1], dt0), written
    from diffrax's published loop: float32 times, t += dt0 accumulated, the first end
    min(t0 + dt0, t1), later ends clipped to t1 when > t1 - 1e-6 (_clip_to_end).
    -> list of (t, tn) float32 pairs."""
    f = np.float32
    ts = np.asarray(ts, f)
    t, t1, dt0 = f(ts[0]), f(ts[-1]), f(dt0)
    tn = min(f(t + dt0), t1)
    out = []
    while t < t1 and (max_steps is None or len(out) < max_steps) and (not out or tn > t):
        out.append((t, tn))
        t = tn
        tn = f(t + dt0)
        if tn > f(t1 - f(1e-6)):
            tn = t1
    return out


def cs_solve(rhs, s0, ts, dt0, solver="rk4", dtype=np.float64, event=None):
    """diffeqsolve(solver, ConstantStepSize, SaveAt(ts)) restated from diffrax's text (the time grid
    of cs_grid, stage times t + c dt, increments (sum a f) dt, every ts[k] through the dense output:
    Euler linear, RK4 the cubic Hermite from the first and last stage increments).  dtype float64
    (semantics, to a tolerance) or float32 (literal rounding: every product / sum rounded in the
    order written).  rhs(t, s) -> ds.  event(s) -> True terminates after the step (its saves kept).
    -> saved [len(ts), n] (+inf after termination)."""
    d = dtype
    ts = np.asarray(ts, np.float32)
    S = ts.shape[0]
    y = np.array(s0, d)
    saved = np.full((S, y.shape[0]), np.inf, d)
    k = 0
    b0, b1 = d(1.0 / 6.0), d(1.0 / 3.0)
    with np.errstate(all="ignore"):
        for t, tn in cs_grid(ts, dt0):
            dtf = np.float32(tn - t)  # the step (float32 times: the stage times key the noise)
            dt = d(dtf)
            f0 = np.asarray(rhs(t, y), d)
            if solver == "euler":
                y1 = y + f0 * dt
            else:
                # zero tableau entries multiplied (diffrax's padded-row dot product, mtgp_cstep.h):
                # 0 f_j is a no-op for a finite f_j and NaN otherwise
                nz = lambda z, v: np.where(np.isnan(z), z, v)
                f1 = np.asarray(rhs(np.float32(t + np.float32(0.5) * dtf), y + (d(0.5) * f0) * dt), d)
                z = d(0) * f0
                f2 = np.asarray(rhs(np.float32(t + np.float32(0.5) * dtf), y + nz(z, d(0.5) * f1) * dt), d)
                z = z + d(0) * f1
                f3 = np.asarray(rhs(np.float32(t + dtf), y + nz(z, f2) * dt), d)
                y1 = y + (((b0 * f0 + b1 * f1) + b1 * f2) + b0 * f3) * dt
            while k < S and ts[k] <= tn:
                if t == tn:
                    th = d(0.0)
                elif d is np.float32:
                    th = np.float32(np.float32(ts[k] - t) / np.float32(tn - t))
                else:
                    th = (d(ts[k]) - d(t)) / (d(tn) - d(t))
                if solver == "euler":
                    saved[k] = y + th * (y1 - y)
                else:
                    k0, k1 = f0 * dt, f3 * dt
                    a = ((k0 + k1) + d(2) * y) - d(2) * y1
                    b = (((d(-2) * k0) - k1) - d(3) * y) + d(3) * y1
                    v = d(0) * th + a
                    v = v * th + b
                    v = v * th + k0
                    saved[k] = v * th + y
                k += 1
            y = y1
            if event is not None and event(y):
                break
    return saved


def rk4(rhs, s0, h, n):
    s = np.array(s0, np.float64)
    out = [s.copy()]
    with np.errstate(all="ignore"):
        for _ in range(n):
            k1 = rhs(s)
            k2 = rhs(s + 0.5 * h * k1)
            k3 = rhs(s + 0.5 * h * k2)
            k4 = rhs(s + h * k3)
            s = s + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
            out.append(s.copy())
    return np.array(out)


# ---- HarmonicOscillator / StirredTankReactor (harmonic_oscillator.py:8-80, reactor.py:7-81)
def ho_drift(x, u, omega, zeta):
    A = np.array([[0.0, 1.0], [-omega, -zeta]])
    b = np.array([[0.0], [1.0]])
    return A @ x + b @ np.atleast_1d(u)


def reactor_drift(x, u, Vol, Cp, dHr, UA, q, Tf, Tcf, Volc):
    Tc, T, c = x
    control = np.clip(u, 0, 300)
    k = 7.2e10 * np.exp(-72750 / 8.314 / T)
    dc = (q / Vol) * (1.0 - c) - k * c
    dT = (q / Vol) * (Tf - T) + (-dHr / Cp) * k * c + (UA / Vol / Cp) * (Tc - T)
    dTc = (control / Volc) * (Tcf - Tc) + (UA / Volc / Cp) * (T - Tc)
    return np.array([dTc, dT, dc])


def env_drift(name, x, u, params):
    return ho_drift(x, u, *params) if name == "harmonic" else reactor_drift(x, u, *params)


def env_fitness(name, xs, us, params, target):
    """fitness_function over the saved points (sum of quadratic costs), float64."""
    xs = np.asarray(xs, np.float64)
    us = np.asarray(us, np.float64).reshape(-1)
    if name == "harmonic":
        omega, zeta = params
        A = np.array([[0.0, 1.0], [-omega, -zeta]])
        b = np.array([[0.0], [1.0]])
        xd = np.array([target, 0.0])
        ud = (-np.linalg.pinv(b) @ A @ xd)[0]
        Q, R = np.array([[0.5, 0], [0, 0]]), 0.5
    else:
        xd = np.array([0.0, target, 0.0])
        ud = 0.0
        Q, R = np.diag([0.0, 0.01, 0.0]), 0.0001
    e = xs - xd
    return float(np.sum(np.einsum("si,ij,sj->s", e, Q, e) + (us - ud) * R * (us - ud)))


def dyn_rhs_env(name, cand, lib, s, state_size, params, target, n_var):
    x, a = s[:n_var], s[n_var:]
    y = np.array(x, np.float64)  # C = I, no noise, no wrap
    tg = np.atleast_1d(target).astype(np.float64)
    u = eval_tree(cand[state_size], lib, np.concatenate([np.zeros(n_var), a, np.zeros(1), tg]))
    dx = env_drift(name, x, u, params)
    d = np.concatenate([y, a, [u], tg])
    da = [eval_tree(cand[i], lib, d) for i in range(state_size)]
    return np.concatenate([dx, da])


def ff_rhs_env(name, cand, lib, s, params, target):
    u = eval_tree(cand[0], lib, np.concatenate([np.array(s, np.float64), np.atleast_1d(target)]))
    return env_drift(name, s, u, params)
