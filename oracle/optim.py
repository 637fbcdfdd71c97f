"""ORACLE — TEST INFRASTRUCTURE ONLY.  A restatement of the reference's constant optimiser for
outcome-level parity tests of srhip_optimize_constants:

  _optimize_constants (src/ConstantOptimization.jl:43-81): f(c) = eval_loss(tree(c);
  regularization=false); Optim.optimize(f, c0, BFGS(linesearch=BackTracking()),
  Optim.Options(iterations=8)) with Optim's default finite-difference gradient (f only is
  passed, :50; central differences, step cbrt(eps) * max(1, |c|)); nrestarts perturbed starts
  c0 .* (1 + randn/2) (:53-68); accept iff the best minimum beats the baseline (:70-78).
  BackTracking restated from LineSearches.jl (order 3, c1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1).
Optim.jl / LineSearches.jl are not in the container: restated from their published algorithms.
"""
from __future__ import annotations

import numpy as np

import oracle


def _loss_fn(tree_nodes, binops, unaops, X, y, w=None, loss_kind=0, p0=0.0):
    const_idx = [i for i, n in enumerate(tree_nodes) if n["degree"] == 0 and n["constant"]]
    order = _get_constants_order(tree_nodes)
    offs = np.array([0, len(tree_nodes)], dtype=np.int64)

    def f(c):
        nd = tree_nodes.copy()
        for k, i in enumerate(order):
            nd[i]["val"] = c[k]
        le, _, ok, _ = oracle.eval_loss_batch(nd, offs, binops, unaops, X, y, w, loss_kind, p0)
        return float(le[0]) if ok[0] else np.inf

    assert len(const_idx) == len(order)
    return f, order


def _get_constants_order(nodes):
    out = []

    def rec(i):
        n = nodes[i]
        if n["degree"] == 0:
            if n["constant"]:
                out.append(i)
            return
        rec(int(n["l"]))
        if n["degree"] == 2:
            rec(int(n["r"]))

    rec(0)
    return out


def _fd_grad(f, x, fx=None):
    g = np.zeros_like(x)
    for k in range(len(x)):
        h = np.cbrt(np.finfo(float).eps) * max(1.0, abs(x[k]))
        xp, xm = x.copy(), x.copy()
        xp[k] += h
        xm[k] -= h
        g[k] = (f(xp) - f(xm)) / (2 * h)
    return g


def _backtracking(phi, phi0, dphi0, c1=1e-4, rho_hi=0.5, rho_lo=0.1, iterations=1000):
    a1 = a2 = 1.0
    phix0, phix1 = phi0, phi(a1)
    it_fin = 0
    while not np.isfinite(phix1) and it_fin < 52:
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
            a_tmp = -(dphi0 * a2 ** 2) / (2 * (phix1 - phi0 - dphi0 * a2))
        else:
            div = 1.0 / (a1 ** 2 * a2 ** 2 * (a2 - a1))
            e1, e0 = phix1 - phi0 - dphi0 * a2, phix0 - phi0 - dphi0 * a1
            a = (a1 ** 2 * e1 - a2 ** 2 * e0) * div
            b = (-a1 ** 3 * e1 + a2 ** 3 * e0) * div
            if abs(a) <= np.finfo(float).eps:
                a_tmp = dphi0 / (2 * b)
            else:
                a_tmp = (-b + np.sqrt(max(b * b - 3 * a * dphi0, 0.0))) / (3 * a)
        a1 = a2
        a_tmp = a2 * rho_hi if np.isnan(a_tmp) else min(a_tmp, a2 * rho_hi)
        a2 = max(a_tmp, a2 * rho_lo)
        phix0, phix1 = phix1, phi(a2)
    return a2, phix1


def bfgs(f, x0, iterations=8, g_tol=1e-8):
    x = np.asarray(x0, dtype=np.float64).copy()
    fx = f(x)
    if not np.isfinite(fx):
        return x, fx
    g = _fd_grad(f, x)
    H = np.eye(len(x))
    for _ in range(iterations):
        if np.max(np.abs(g)) <= g_tol:
            break
        s = -H @ g
        dphi0 = float(g @ s)
        if not dphi0 < 0:
            H = np.eye(len(x))
            s = -g
            dphi0 = float(g @ s)
        a, fnew = _backtracking(lambda a: f(x + a * s), fx, dphi0)
        if a is None:
            break
        xn = x + a * s
        gn = _fd_grad(f, xn)
        dx, dg = xn - x, gn - g
        dxdg = float(dx @ dg)
        if dxdg > 0:
            u = H @ dg
            c1 = (dxdg + float(dg @ u)) / dxdg ** 2
            H = H + c1 * np.outer(dx, dx) - (np.outer(u, dx) + np.outer(dx, u)) / dxdg
        fold = fx
        x, fx, g = xn, fnew, gn
        if fx == fold:
            break
    return x, fx


def optimize_constants(tree_nodes, binops, unaops, X, y, w=None, iterations=8, nrestarts=2, rng=None):
    """(constants, loss, improved) for one tree (srhip_node table), reference procedure."""
    f, order = _loss_fn(tree_nodes, binops, unaops, X, y, w)
    x0 = np.array([tree_nodes[i]["val"] for i in order], dtype=np.float64)
    if len(x0) == 0:
        return x0, f(x0), False
    baseline = f(x0)
    best_x, best_f = bfgs(f, x0, iterations)
    rng = np.random.default_rng(0) if rng is None else rng
    for _ in range(nrestarts):
        xs = x0 * (1 + 0.5 * rng.standard_normal(len(x0)))
        xr, fr = bfgs(f, xs, iterations)
        if fr < best_f:
            best_x, best_f = xr, fr
    if best_f < baseline:
        return best_x, best_f, True
    return x0, baseline, False
