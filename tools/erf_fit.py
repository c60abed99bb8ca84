"""How cheap can conv0's exact-erf GELU get (conv0 forward <= 215 us)? Fits of erf on
[0, 4] as the kernels evaluate it: (a) rational x P(x^2) / Q(x^2) of degrees (n, m) -- the form of
csrc/common.h erf_fast2, (6, 4), one reciprocal per element -- and (b) division-free odd polynomials
x P(x^2) clamped to 1 past c. Printed: max |error| in exact and in f32 evaluation.
Outcome (r06): (5, 3) reaches 4.1e-6 for 2 packed fmas less per element pair (~6 % of
the kernel's VALU), every division-free form of <= 10 terms stays above 2e-5 (the x^2 monomial basis
cannot follow erf's saturation): no fit removes the reciprocal at f32-level accuracy.
CPU only: python tools/erf_fit.py"""
import numpy as np
from scipy.special import erf
from scipy.optimize import least_squares
x = np.linspace(1e-6, 4.0, 20000)
y = erf(x) / x   # even function g(x2)
X2 = x * x
def fit(n, m):
    # g ~ P(x2)/Q(x2), Q monic-free with Q(0)=1 normalisation: unknowns p0..pn, q1..qm
    # linearised LS then iterate weights (Loeb), then minimax-ish refine with least_squares on max
    w = np.ones_like(x)
    for it in range(30):
        A = np.concatenate([np.stack([X2**k for k in range(n+1)], 1), -np.stack([y * X2**k for k in range(1, m+1)], 1)], 1)
        A = A * w[:, None]
        coef, *_ = np.linalg.lstsq(A, y * w, rcond=None)
        p = coef[:n+1]; q = np.concatenate([[1.0], coef[n+1:]])
        Q = np.polyval(q[::-1], X2)
        err = (np.polyval(p[::-1], X2) / Q - y) * x   # error in erf
        w = 1.0 / np.abs(Q) * (np.abs(err) / np.abs(err).max() + 0.05) ** 0.5
    # refine minimax via least_squares with a smooth max proxy (L^p, p large)
    def res(c):
        p = c[:n+1]; q = np.concatenate([[1.0], c[n+1:]])
        e = (np.polyval(p[::-1], X2) / np.polyval(q[::-1], X2) - y) * x
        return e * 1e6
    c0 = np.concatenate([p, q[1:]])
    for pw in (4, 8, 16):
        r = least_squares(lambda c: np.abs(res(c)) ** (pw / 2) * np.sign(res(c)), c0, method="lm", max_nfev=4000)
        c0 = r.x
    p = c0[:n+1]; q = np.concatenate([[1.0], c0[n+1:]])
    # evaluate in float32 Horner
    xf = np.float32(x); x2f = np.float32(xf * xf)
    P = np.float32(p[n]);
    for k in range(n - 1, -1, -1): P = np.float32(np.float32(P * x2f) + np.float32(p[k]))
    Qf = np.float32(q[m])
    for k in range(m - 1, -1, -1): Qf = np.float32(np.float32(Qf * x2f) + np.float32(q[k]))
    ef = np.float32(xf * P) / Qf
    e64 = np.abs(np.polyval(p[::-1], X2) / np.polyval(q[::-1], X2) * x - erf(x)).max()
    e32 = np.abs(ef.astype(np.float64) - erf(x)).max()
    return p, q, e64, e32
for n, m in ((6, 4), (5, 3), (4, 3), (4, 2), (3, 3), (5, 2)):
    p, q, e64, e32 = fit(n, m)
    print(n, m, f"exact {e64:.2e} f32 {e32:.2e}", "ops", n + m)

# odd polynomial x*P(x^2) on [0,c], minimax via IRLS; f32 evaluation error estimated
def fit(n, c):
    x = np.cos(np.linspace(0, np.pi, 4000))*c/2 + c/2
    x = np.concatenate([x, np.linspace(0, c, 4000)])
    y = erf(x)
    A = np.stack([x * x**(2*k) for k in range(n)], 1)
    w = np.ones_like(x)
    for it in range(60):
        coef, *_ = np.linalg.lstsq(A * w[:, None], y * w, rcond=None)
        e = A @ coef - y
        w = w * (np.abs(e) / np.abs(e).max() + 1e-3) ** 0.5
    xs = np.linspace(0, 6, 200001)
    p = np.zeros_like(xs, dtype=np.float32)
    x32 = xs.astype(np.float32); xx = (x32*x32).astype(np.float32)
    cm = np.minimum(x32, np.float32(c)); cc = (cm*cm).astype(np.float32)
    acc = np.full_like(cc, np.float32(coef[-1]))
    for k in range(n-2, -1, -1):
        acc = (acc*cc + np.float32(coef[k])).astype(np.float32)
    r = np.minimum((cm*acc).astype(np.float32), np.float32(1.0))
    err = np.abs(r.astype(np.float64) - erf(xs)).max()
    return coef, err
print("division-free odd polynomials:")
for c in (3.2, 3.4, 3.6, 3.9):
    for n in (8, 9, 10, 11, 12):
        coef, err = fit(n, c)
        print(f"c={c} terms={n} maxerr={err:.2e}")
