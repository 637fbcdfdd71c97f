"""ORACLE — TEST INFRASTRUCTURE ONLY.  A restatement of the reference's constant optimiser for
outcome-level parity tests of srhip_optimize_constants:

  dispatch_optimize_constants (src/ConstantOptimization.jl:22-41): no constants -> nothing;
  one constant -> Optim.Newton(linesearch=BackTracking()); else BFGS(linesearch=BackTracking()).
  _optimize_constants (:43-81): f(c) = eval_loss(tree(c); regularization=false);
  Optim.optimize(f, c0, algorithm, Optim.Options(iterations=8)) with only f passed (:50), so
  NLSolversBase differentiates by finite differences (FiniteDiff.jl): central gradient, step
  cbrt(eps) * max(1, |c|); Newton's Hessian by the second difference with step
  eps^(1/4) * max(1, |c|), factored by PositiveFactorizations' cholesky!(Positive, H) (a 1x1
  Hessian h becomes |h|, or 1 when h == 0); nrestarts perturbed starts c0 .* (1 + randn/2)
  (:53-68); accept iff the best minimum beats the baseline (:70-78).
  BackTracking restated from LineSearches.jl (order 3, c1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1).
Optim.jl 1.8-1.9 / LineSearches.jl 7 / NLSolversBase / FiniteDiff / PositiveFactorizations are not in
the container (Project.toml:45,49): restated from their published algorithms.
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
        le, _, ok, _ = oracle.eval_loss_batch(nd, offs, binops, unaops, X, y, w, loss_kind, p0, nthreads=1)
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


def _fd_grad(f, x, fx=None, scale=1.0):
    g = np.zeros_like(x)
    for k in range(len(x)):
        h = scale * np.cbrt(np.finfo(float).eps) * max(1.0, abs(x[k]))
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
            with np.errstate(all="ignore"):
                a_tmp = -(dphi0 * a2 ** 2) / np.float64(2 * (phix1 - phi0 - dphi0 * a2))
        else:
            with np.errstate(all="ignore"):  # IEEE like Julia: a1 == a2 (alpha underflowed) gives Inf / NaN
                div = np.float64(1.0) / np.float64(a1 ** 2 * a2 ** 2 * (a2 - a1))
            e1, e0 = phix1 - phi0 - dphi0 * a2, phix0 - phi0 - dphi0 * a1
            a = (a1 ** 2 * e1 - a2 ** 2 * e0) * div
            b = (-a1 ** 3 * e1 + a2 ** 3 * e0) * div
            with np.errstate(all="ignore"):
                if abs(a) <= np.finfo(float).eps:
                    a_tmp = np.float64(dphi0) / np.float64(2 * b)
                else:
                    a_tmp = (-b + np.sqrt(max(b * b - 3 * a * dphi0, 0.0))) / np.float64(3 * a)
        a1 = a2
        a_tmp = a2 * rho_hi if np.isnan(a_tmp) else min(a_tmp, a2 * rho_hi)
        a2 = max(a_tmp, a2 * rho_lo)
        phix0, phix1 = phix1, phi(a2)
    return a2, phix1


def bfgs(f, x0, iterations=8, g_tol=1e-8, fd_scale=1.0):
    x = np.asarray(x0, dtype=np.float64).copy()
    fx = f(x)
    if not np.isfinite(fx):
        return x, fx
    g = _fd_grad(f, x, scale=fd_scale)
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
        gn = _fd_grad(f, xn, scale=fd_scale)
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


def _fd_hess_1d(f, x, fx, scale=1.0):
    """FiniteDiff's :hcentral diagonal second difference (n = 1)."""
    e = scale * np.finfo(float).eps ** 0.25 * max(1.0, abs(x[0]))
    xp, xm = x.copy(), x.copy()
    xp[0] += e
    xm[0] -= e
    return (f(xp) - 2.0 * fx + f(xm)) / (e * e)


def newton(f, x0, iterations=8, g_tol=1e-8, fd_scale=1.0):
    """Optim.Newton(linesearch=BackTracking()) for one constant, finite-difference derivatives."""
    x = np.asarray(x0, dtype=np.float64).copy()
    assert len(x) == 1
    fx = f(x)
    if not np.isfinite(fx):
        return x, fx
    g = _fd_grad(f, x, scale=fd_scale)
    h = _fd_hess_1d(f, x, fx, scale=fd_scale)
    for _ in range(iterations):
        if np.max(np.abs(g)) <= g_tol:
            break
        hp = abs(h) if (np.isfinite(h) and h != 0.0) else 1.0  # cholesky!(Positive, [h])
        s = -g / hp
        dphi0 = float(g @ s)
        a, fnew = _backtracking(lambda a: f(x + a * s), fx, dphi0)
        if a is None:
            break
        xn = x + a * s
        fold = fx
        x, fx = xn, fnew
        g = _fd_grad(f, x, scale=fd_scale)
        h = _fd_hess_1d(f, x, fx, scale=fd_scale)
        if fx == fold:
            break
    return x, fx


def optimize_constants(tree_nodes, binops, unaops, X, y, w=None, iterations=8, nrestarts=2, rng=None, fd_scale=1.0):
    """(constants, loss, improved) for one tree (srhip_node table), reference procedure.
    fd_scale multiplies the finite-difference steps (1 = the reference's); tests use a second scale
    to see whether an outcome is resolved at all (see outcome_is_stable)."""
    f, order = _loss_fn(tree_nodes, binops, unaops, X, y, w)
    x0 = np.array([tree_nodes[i]["val"] for i in order], dtype=np.float64)
    if len(x0) == 0:
        return x0, f(x0), False
    algorithm = newton if len(x0) == 1 else bfgs  # src/ConstantOptimization.jl:27-31
    baseline = f(x0)
    best_x, best_f = algorithm(f, x0, iterations, fd_scale=fd_scale)
    rng = np.random.default_rng(0) if rng is None else rng
    for _ in range(nrestarts):
        xs = x0 * (1 + 0.5 * rng.standard_normal(len(x0)))
        xr, fr = algorithm(f, xs, iterations, fd_scale=fd_scale)
        if fr < best_f:
            best_x, best_f = xr, fr
    if best_f < baseline:
        return best_x, best_f, True
    return x0, baseline, False


def reference_outcome(tree_nodes, binops, unaops, X, y, w=None, iterations=8, rtol=1e-6):
    """(loss, stable): the reference procedure's single-start optimum, and whether that optimum is
    resolved -- i.e. reproduced (to rtol) when the finite-difference steps are 4x larger.  Where the
    reference's own outcome moves with its difference step (oscillatory objectives such as
    sin(exp(c + x)), whose gradients are not resolvable at the step size), any differentiation --
    the device's exact one included -- follows a different but equally valid trajectory, and the
    optimum is not a parity target."""
    _, l1, _ = optimize_constants(tree_nodes, binops, unaops, X, y, w, iterations, nrestarts=0)
    _, l4, _ = optimize_constants(tree_nodes, binops, unaops, X, y, w, iterations, nrestarts=0, fd_scale=4.0)
    stable = l1 == l4 or abs(l1 - l4) <= rtol * abs(l1) + 1e-12
    return l1, bool(stable)
