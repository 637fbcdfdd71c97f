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
        # LineSearches.jl's expressions with Julia's association: x^2 = x*x, x^3 = x*x*x (literal powers)
        if it == 1:
            with np.errstate(all="ignore"):
                a_tmp = -(np.float64(dphi0) * (a2 * a2)) / np.float64(2 * (phix1 - phi0 - dphi0 * a2))
        else:
            with np.errstate(all="ignore"):  # IEEE like Julia: a1 == a2 (alpha underflowed) gives Inf / NaN
                div = np.float64(1.0) / np.float64((a1 * a1) * (a2 * a2) * (a2 - a1))
                e1, e0 = phix1 - phi0 - dphi0 * a2, phix0 - phi0 - dphi0 * a1
                a = ((a1 * a1) * e1 - (a2 * a2) * e0) * div
                b = (-(a1 * a1 * a1) * e1 + (a2 * a2 * a2) * e0) * div
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


# ---- exact-gradient mode ------------------------------------------------------------------------
# libsrhip differentiates the objective exactly (forward-mode dual numbers) where the reference
# differentiates by finite differences.  This mode restates the same optimiser -- Optim's BFGS /
# Newton with LineSearches' BackTracking, in the arithmetic order of their source (Optim bfgs.jl
# update_h!: c1 = (dx'dg + dg'u) / (dx'dg)^2, c2 = 1 / dx'dg; direction s = -invH g; the 1x1 Newton
# Hessian as the central difference of the exact gradient with step cbrt(eps) max(1, |c|), made
# positive like cholesky!(Positive, H)) -- over the oracle's exact gradient (oracle.loss_grad), so
# the device optimiser's state machine is compared with no finite-difference noise on either side.

def _grad_fn(tree_nodes, binops, unaops, X, y, w, order):
    def g(c):
        nd = tree_nodes.copy()
        for k, i in enumerate(order):
            nd[i]["val"] = c[k]
        return oracle.loss_grad(nd, binops, unaops, X, y, w)
    return g


def _maxabs(v):
    m = 0.0
    for e in v:
        m = max(m, abs(float(e)))
    return m


def bfgs_exact(f, grad, x0, iterations=8, g_tol=1e-8):
    """(x, f(x), objective calls) -- Optim.BFGS(linesearch=BackTracking()) with the exact gradient."""
    x = np.asarray(x0, dtype=np.float64).copy()
    n = len(x)
    fx = f(x)
    calls = 1
    if not np.isfinite(fx):
        return x, fx, calls
    g = grad(x)
    H = [[1.0 if i == j else 0.0 for j in range(n)] for i in range(n)]
    if _maxabs(g) <= g_tol:
        return x, fx, calls
    for _ in range(iterations):
        s = [0.0] * n
        dphi0 = 0.0
        for i in range(n):
            acc = 0.0
            for j in range(n):
                acc += H[i][j] * g[j]
            s[i] = -acc
            dphi0 += g[i] * s[i]
        if not dphi0 < 0:
            H = [[1.0 if i == j else 0.0 for j in range(n)] for i in range(n)]
            dphi0 = 0.0
            for i in range(n):
                s[i] = -g[i]
                dphi0 -= g[i] * g[i]
        nc = [0]

        def phi(a):
            nc[0] += 1
            return f(np.array([x[i] + a * s[i] for i in range(n)]))

        a, fnew = _backtracking(phi, fx, dphi0)
        calls += nc[0]
        if a is None:
            break
        xn = np.array([x[i] + a * s[i] for i in range(n)])
        gn = grad(xn)
        dx = [a * s[i] for i in range(n)]
        dg = [gn[i] - g[i] for i in range(n)]
        dxdg = 0.0
        for i in range(n):
            dxdg += dx[i] * dg[i]
        if dxdg > 0.0:
            u = [0.0] * n
            dgu = 0.0
            for i in range(n):
                acc = 0.0
                for j in range(n):
                    acc += H[i][j] * dg[j]
                u[i] = acc
                dgu += dg[i] * acc
            c1 = (dxdg + dgu) / (dxdg * dxdg)
            c2 = 1.0 / dxdg
            for i in range(n):
                for j in range(n):
                    H[i][j] += c1 * dx[i] * dx[j] - c2 * (u[i] * dx[j] + dx[i] * u[j])
        fold = fx
        x, fx, g = xn, fnew, gn
        if fx == fold or _maxabs(g) <= g_tol:
            break
    return x, fx, calls


def newton_exact(f, grad, x0, iterations=8, g_tol=1e-8):
    """(x, f(x), objective calls) -- Optim.Newton(linesearch=BackTracking()) for one constant, exact
    gradient, Hessian = central difference of the exact gradient."""
    x = np.asarray(x0, dtype=np.float64).copy()
    fx = f(x)
    calls = 1
    if not np.isfinite(fx):
        return x, fx, calls
    g = grad(x)
    if _maxabs(g) <= g_tol:
        return x, fx, calls
    for it in range(iterations):
        e = 6.055454452393343e-06 * max(1.0, abs(float(x[0])))  # cbrt(eps(Float64))
        xp, xm = np.array([x[0] + e]), np.array([x[0] - e])
        fp, fm = f(xp), f(xm)
        h = (grad(xp)[0] - grad(xm)[0]) / (2.0 * e) if np.isfinite(fp) and np.isfinite(fm) else np.nan
        hp = abs(h) if (np.isfinite(h) and h != 0.0) else 1.0  # cholesky!(Positive, [h])
        s0 = -g[0] / hp
        dphi0 = g[0] * s0
        nc = [0]

        def phi(a):
            nc[0] += 1
            return f(np.array([x[0] + a * s0]))

        a, fnew = _backtracking(phi, fx, dphi0)
        calls += nc[0]
        if a is None:
            break
        xn = np.array([x[0] + a * s0])
        fold = fx
        x, fx = xn, fnew
        g = grad(x)
        if fx == fold or _maxabs(g) <= g_tol:
            break
    return x, fx, calls


def _devorder_fns(tree_nodes, binops, unaops, X, y, w, order):
    """(f, grad) with libsrhip's row-sum order (oracle.loss_grad_devorder) and the value oracle's
    did_succeed (f = Inf where the tree fails, as eval_loss returns L(Inf)).  Float32 data: the
    constants are rounded to Float32 at every call (the program holds Float32 immediates) while the
    optimiser's state stays Float64, as libsrhip's optimiser keeps it."""
    offs = np.array([0, len(tree_nodes)], dtype=np.int64)
    cache = {}
    f32 = np.asarray(X).dtype == np.float32

    def both(c):
        key = np.asarray(c, dtype=np.float64).tobytes()
        if key not in cache:
            nd = tree_nodes.copy()
            for k, i in enumerate(order):
                nd[i]["val"] = float(np.float32(c[k])) if f32 else c[k]
            _, _, ok, _ = oracle.eval_loss_batch(nd, offs, binops, unaops, X, y, w, 0, 0.0, nthreads=1)
            lv, g = oracle.loss_grad_devorder(nd, binops, unaops, X, y, w)
            cache.clear()
            cache[key] = (lv if ok[0] and np.isfinite(lv) else np.inf, g)
        return cache[key]

    return (lambda c: both(c)[0]), (lambda c: both(c)[1])


def optimize_constants_exact(tree_nodes, binops, unaops, X, y, w=None, iterations=8, starts=None,
                             device_order=False):
    """(constants, loss, improved, objective calls) for one tree -- the reference procedure
    (src/ConstantOptimization.jl:22-81: Newton for one constant, BFGS otherwise, best of the starts,
    accepted only if it beats the baseline) with the exact gradient.  ``starts``: the start points
    (default: the tree's own constants only).  ``device_order``: the objective and gradient summed
    in libsrhip's row order instead of exactly, so that a line search deciding at the rounding
    noise decides as the device does."""
    f, order = _loss_fn(tree_nodes, binops, unaops, X, y, w)
    grad = _grad_fn(tree_nodes, binops, unaops, X, y, w, order)
    if device_order:  # sums in libsrhip's row order: the same objective bits as the device's
        f, grad = _devorder_fns(tree_nodes, binops, unaops, X, y, w, order)
    x0 = np.array([tree_nodes[i]["val"] for i in order], dtype=np.float64)
    if np.asarray(X).dtype == np.float32:  # a Float32 tree's constants are Float32 values
        x0 = x0.astype(np.float32).astype(np.float64)
    if len(x0) == 0:
        return x0, f(x0), False, 0
    algorithm = newton_exact if len(x0) == 1 else bfgs_exact
    baseline = f(x0)
    best_x, best_f, calls = x0, np.inf, 0
    for s, xs in enumerate(starts if starts is not None else [x0]):
        xr, fr, c = algorithm(f, grad, np.asarray(xs, dtype=np.float64), iterations)
        calls += c
        # the first start is `result` unconditionally (:50); a restart replaces it only when its
        # minimum is strictly smaller (:65-67)
        if s == 0 or fr < best_f:
            best_x, best_f = xr, fr
    if best_f < baseline:
        return best_x, best_f, True, calls
    return x0, baseline, False, calls
