"""Constant optimisation on the host for objectives the device cannot differentiate: a user
``loss_function`` (or a Python elementwise loss) evaluated through device ``eval_tree_array``
predictions.  The reference runs Optim.jl on ``f(t) = eval_loss(t, dataset, options;
regularization=false, idx)`` with only f supplied (src/ConstantOptimization.jl:43-81), so NLSolversBase
differentiates by finite differences; this module restates that procedure over a scalar host
objective:

  dispatch (:22-41)   no constants -> nothing; one constant -> Newton; else BFGS, both with
                      LineSearches' BackTracking (order 3, c1 = 1e-4, rho in [0.1, 0.5], alpha0 = 1)
  gradient            FiniteDiff central differences, step cbrt(eps) max(1, |c|)
  Newton's Hessian    FiniteDiff :hcentral second difference, step eps^(1/4) max(1, |c|), made
                      positive like PositiveFactorizations' cholesky!(Positive, [h]) (|h|, or 1 if h == 0)
  stopping            `iterations` iterations, |g|_inf <= g_tol, or an unchanged objective
  restarts (:53-68)   c0 .* (1 + randn/2), keep the best; accept iff it beats the baseline (:70-78)
Objective calls are counted like Optim's f_calls (the difference quotients are g_calls / h_calls).
Built-in distance losses never come here: srhip_optimize_constants runs those batched on the device
with exact dual-number gradients.
"""
from __future__ import annotations

import math

import numpy as np

_EPS = np.finfo(np.float64).eps


class _Counted:
    def __init__(self, f):
        self.f, self.calls = f, 0

    def __call__(self, c, count=True):
        if count:
            self.calls += 1
        v = float(self.f(np.asarray(c, dtype=np.float64)))
        return v if not math.isnan(v) else math.inf


def _fd_grad(f, x):
    g = np.zeros_like(x)
    for k in range(len(x)):
        h = np.cbrt(_EPS) * max(1.0, abs(x[k]))
        xp, xm = x.copy(), x.copy()
        xp[k] += h
        xm[k] -= h
        g[k] = (f(xp, count=False) - f(xm, count=False)) / (2 * h)
    return g


def _fd_hess_1d(f, x, fx):
    e = _EPS ** 0.25 * max(1.0, abs(x[0]))
    xp, xm = x.copy(), x.copy()
    xp[0] += e
    xm[0] -= e
    return (f(xp, count=False) - 2.0 * fx + f(xm, count=False)) / (e * e)


def backtracking(phi, phi0, dphi0, c1=1e-4, rho_hi=0.5, rho_lo=0.1, iterations=1000):
    """LineSearches.BackTracking (order 3) from alpha = 1: (alpha, phi(alpha)) or (None, None)."""
    a1 = a2 = 1.0
    phix0, phix1 = phi0, phi(a1)
    it_fin = 0
    while not math.isfinite(phix1) and it_fin < 52:  # iterfinitemax
        it_fin += 1
        a1 = a2
        a2 = a1 / 2
        phix1 = phi(a2)
    it = 0
    while phix1 > phi0 + c1 * a2 * dphi0:
        it += 1
        if it > iterations:
            return None, None
        if it == 1:
            with np.errstate(all="ignore"):
                a_tmp = -(dphi0 * a2 ** 2) / np.float64(2 * (phix1 - phi0 - dphi0 * a2))
        else:
            with np.errstate(all="ignore"):  # IEEE like Julia: a1 == a2 (alpha underflowed) gives Inf / NaN
                div = np.float64(1.0) / np.float64(a1 ** 2 * a2 ** 2 * (a2 - a1))
            e1, e0 = phix1 - phi0 - dphi0 * a2, phix0 - phi0 - dphi0 * a1
            a = (a1 ** 2 * e1 - a2 ** 2 * e0) * div
            b = (-a1 ** 3 * e1 + a2 ** 3 * e0) * div
            with np.errstate(all="ignore"):
                a_tmp = (np.float64(dphi0) / np.float64(2 * b) if abs(a) <= _EPS else
                         (-b + np.sqrt(max(b * b - 3 * a * dphi0, 0.0))) / np.float64(3 * a))
        a1 = a2
        a_tmp = a2 * rho_hi if np.isnan(a_tmp) else min(a_tmp, a2 * rho_hi)
        a2 = max(a_tmp, a2 * rho_lo)
        phix0, phix1 = phix1, phi(a2)
    return a2, phix1


def _step(f, x, fx, g, s):
    dphi0 = float(g @ s)
    return backtracking(lambda a: f(x + a * s), fx, dphi0)


def bfgs(f, x0, iterations=8, g_tol=1e-8):
    x = np.asarray(x0, dtype=np.float64).copy()
    fx = f(x)
    if not math.isfinite(fx):
        return x, fx
    g = _fd_grad(f, x)
    H = np.eye(len(x))
    for _ in range(iterations):
        if np.max(np.abs(g)) <= g_tol:
            break
        s = -H @ g
        if not float(g @ s) < 0:
            H = np.eye(len(x))
            s = -g
        a, fnew = _step(f, x, fx, g, s)
        if a is None:
            break
        xn = x + a * s
        gn = _fd_grad(f, xn)
        dx, dg = xn - x, gn - g
        dxdg = float(dx @ dg)
        if dxdg > 0:
            u = H @ dg
            H = H + (dxdg + float(dg @ u)) / dxdg ** 2 * np.outer(dx, dx) - (np.outer(u, dx) + np.outer(dx, u)) / dxdg
        fold = fx
        x, fx, g = xn, fnew, gn
        if fx == fold:
            break
    return x, fx


def newton(f, x0, iterations=8, g_tol=1e-8):
    x = np.asarray(x0, dtype=np.float64).copy()
    fx = f(x)
    if not math.isfinite(fx):
        return x, fx
    g = _fd_grad(f, x)
    h = _fd_hess_1d(f, x, fx)
    for _ in range(iterations):
        if np.max(np.abs(g)) <= g_tol:
            break
        hp = abs(h) if (math.isfinite(h) and h != 0.0) else 1.0
        a, fnew = _step(f, x, fx, g, -g / hp)
        if a is None:
            break
        fold = fx
        x, fx = x + a * (-g / hp), fnew
        g = _fd_grad(f, x)
        h = _fd_hess_1d(f, x, fx)
        if fx == fold:
            break
    return x, fx


def optimize(objective, x0, iterations=8, nrestarts=2, rng=None):
    """_optimize_constants over a host objective: (best constants, best value, improved, f_calls,
    baseline).  The baseline call itself is not counted (src/ConstantOptimization.jl:49-51)."""
    f = _Counted(objective)
    x0 = np.asarray(x0, dtype=np.float64)
    baseline = f(x0, count=False)
    if len(x0) == 0:
        return x0, baseline, False, 0, baseline
    algorithm = newton if len(x0) == 1 else bfgs
    best_x, best_f = algorithm(f, x0, iterations)
    rng = np.random.default_rng() if rng is None else rng
    for _ in range(nrestarts):
        xr, fr = algorithm(f, x0 * (1 + 0.5 * rng.standard_normal(len(x0))), iterations)
        if fr < best_f:
            best_x, best_f = xr, fr
    if best_f < baseline:
        return best_x, best_f, True, f.calls, baseline
    return x0, baseline, False, f.calls, baseline
