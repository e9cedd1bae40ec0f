#!/usr/bin/env python3
"""Fit of the sin polynomial of include/mtgp_f32math.h (spec v2): relative-error Lawson/IRLS fit of
sin r ~ r + r^3 (c3 + c5 s + c7 s^2 + c9 s^3), s = r^2, on |r| <= 1.002 pi/2, coefficients rounded to
f32 one at a time (the rest refitted after each rounding).  Prints the f32 bit patterns."""
import numpy as np
# relative-error minimax-ish fit of sin(r) ~ r + r^3 (c3 + c5 s + c7 s^2 + c9 s^3 + c11 s^4), s = r^2, |r| <= pi/2 + slack
R = np.pi / 2 * 1.002
r = np.cos(np.linspace(0, np.pi, 20001)) * R / 2 + R / 2   # cheb-ish nodes on (0, R]
r = r[r > 1e-4]
s = r * r
target = (np.sin(r) - r) / (r ** 3)      # q(s)
w = r ** 3 / np.sin(r)                    # relative-error weight
def fit(fixed):
    # fixed: dict power->value; fit remaining powers with IRLS-ish minimax (Lawson)
    pw = [0, 1, 2, 3]
    free = [p for p in pw if p not in fixed]
    t = target - sum(v * s ** p for p, v in fixed.items())
    A = np.stack([s ** p for p in free], 1)
    lw = np.ones_like(s)
    for it in range(200):
        W = w * np.sqrt(lw)
        c, *_ = np.linalg.lstsq(A * W[:, None], t * W, rcond=None)
        err = np.abs((A @ c - t) * w)
        lw = lw * err / err.mean()
        lw /= lw.sum()
    out = dict(fixed)
    out.update({p: v for p, v in zip(free, c)})
    e = (sum(out[p] * s ** p for p in pw) - target) * w
    return out, np.abs(e).max()
fixed = {}
for p in [0, 1, 2, 3]:
    c, e = fit(fixed)
    print(p, "max rel err", e, {k: float(v) for k, v in c.items()})
    fixed[p] = float(np.float32(c[p]))
c, e = fit({k: v for k, v in fixed.items() if k != 4}) if False else (fixed, None)
pw=[0,1,2,3]
e = (sum(fixed[p] * s ** p for p in pw) - target) * w
print("final f32 coeffs", [np.float32(fixed[p]).view(np.uint32) for p in pw], [repr(np.float32(fixed[p])) for p in pw], "max rel", np.abs(e).max())
