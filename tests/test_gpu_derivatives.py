"""Per-row derivatives on the device: eval_grad_tree_array (variable = true / false) and
eval_diff_tree_array (src/InterfaceDynamicExpressions.jl:90-95,118-124), on the shapes of the
reference's own derivative test (test/test_derivatives.jl:37-121: X = rand(3, 100) * 5, equations 1-5;
its custom operators are expressed with device operators: pow_abs2(x, y) = abs(x) ^ y,
custom_cos(x) = square(cos(x))).  The reference compares with Zygote at rtol 0.1; here the bar is
analytic derivatives and the oracle's central differences, at tight tolerances.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sr():
    import srhip

    return srhip


def _opts(sr):
    return sr.Options(binary_operators=("+", "*", "-", "/", "^"), unary_operators=("cos", "exp", "sin", "abs", "square"))


def pow_abs2(sr, x, y):
    return sr.Node("^", sr.Node("abs", x), y)


def custom_cos(sr, x):
    return sr.square(sr.cos(x))


def equations(sr):
    x1, x2, x3 = sr.Node("x1"), sr.Node("x2"), sr.Node("x3")
    eq1 = x1 + x2 + x3 + 3.2
    eq2 = pow_abs2(sr, x1, x2) + x3 + custom_cos(sr, 1.0 + x3) + 3.0 / x1
    eq3 = ((x2 + x2) * ((-0.5982493 / pow_abs2(sr, x1, x2)) / -0.54734415)) + (
        sr.sin(custom_cos(sr, sr.sin(sr.Node(val=1.2926733) - 1.6606787)
                          / sr.sin(((0.14577048 * x1) + ((0.111149654 + x1) - -0.8298334)) - -1.2071426))
               * (custom_cos(sr, x3 - 2.3201916) + ((x1 - (x1 * x2)) / x2)))
        / (0.14854191 - ((custom_cos(sr, x2) * -1.6047639) - 0.023943262)))
    return [eq1, eq2, eq3]


def _X(dtype):
    return (np.random.default_rng(0).random((3, 100)) * 5).astype(dtype)


def _analytic_grad(j, X):
    x1, x2, x3 = X.astype(np.float64)
    if j == 0:
        return np.ones((3, X.shape[1]))
    if j == 1:
        a = np.abs(x1)
        return np.stack([x2 * a ** (x2 - 1) * np.sign(x1) - 3.0 / x1 ** 2, a ** x2 * np.log(a),
                         1 - 2 * np.cos(1 + x3) * np.sin(1 + x3)])
    return None


def _fd_feature_grad(oracle, opts, nodes, X, f, h):
    Xp, Xm = X.copy(), X.copy()
    Xp[f] += h
    Xm[f] -= h
    yp, _ = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, Xp)
    ym, _ = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, Xm)
    return (yp - ym) / (2 * h)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_variable_gradients_reference_equations(ctx, oracle, dtype):
    """test_derivatives.jl:37-83: predictions, eval_grad_tree_array(variable=true) and
    eval_diff_tree_array for every feature, for equations 1-3."""
    sr = _sr()
    opts = _opts(sr)
    X = _X(dtype)
    rtol = 1e-10 if dtype == np.float64 else 2e-4
    for j, tree in enumerate(equations(sr)):
        out, grad, ok = sr.eval_grad_tree_array(tree, X, opts, variable=True)
        assert ok and grad.shape == (3, 100) and grad.dtype == dtype
        pred, pok = sr.eval_tree_array(tree, X, opts)
        assert pok and np.array_equal(out, pred)  # the evaluator's own predictions
        for f in range(3):
            o2, d2, ok2 = sr.eval_diff_tree_array(tree, X, opts, f + 1)
            assert ok2 and np.array_equal(o2, out) and np.array_equal(d2, grad[f])  # same kernel, same bits
        want = _analytic_grad(j, X)
        keep = np.ones(want.shape if want is not None else (3, X.shape[1]), dtype=bool)
        if want is None:  # equation 3: Richardson-extrapolated central differences of the oracle (F64),
            # on the rows where two step sizes agree (near eq3's poles the differences are unreliable)
            nodes, _ = sr.flatten([tree], opts, np.float64)
            X64 = X.astype(np.float64)
            d1 = np.stack([_fd_feature_grad(oracle, opts, nodes, X64, f, 1e-5) for f in range(3)])
            d2 = np.stack([_fd_feature_grad(oracle, opts, nodes, X64, f, 1e-5 / 4) for f in range(3)])
            want = (16 * d2 - d1) / 15
            keep = np.abs(d1 - d2) <= 1e-4 * np.maximum(1.0, np.abs(want))
            assert keep.mean() > 0.95
            tol = max(rtol, 1e-7) if dtype == np.float64 else 1e-3
        else:
            tol = rtol
        g64 = grad.astype(np.float64)
        np.testing.assert_allclose(g64[keep], want[keep], rtol=tol, atol=tol * np.abs(want[keep]).max())
        assert not np.allclose(grad * 0, want, rtol=0.1)  # the reference's own sanity check


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_constant_gradients_reference_equations(ctx, dtype):
    """test_derivatives.jl:85-121: d(3.2 x1)/dC = x1 (exactly), and equation 5's two constants."""
    sr = _sr()
    opts = _opts(sr)
    X = _X(dtype)
    x1, x2, x3 = sr.Node("x1"), sr.Node("x2"), sr.Node("x3")
    _, grad, ok = sr.eval_grad_tree_array(sr.Node(val=3.2) * x1, X, opts, variable=False)
    assert ok and grad.shape == (1, 100) and np.array_equal(grad[0], X[0])
    c1, c2 = 2.1, -3.2
    eq5 = pow_abs2(sr, x1, x2) + x3 + custom_cos(sr, sr.Node(val=c1) + x3) + sr.Node(val=c2) / x1
    _, grad, ok = sr.eval_grad_tree_array(eq5, X, opts, variable=False)
    Xd = X.astype(np.float64)
    c1t = np.float64(dtype(c1))
    want = np.stack([-2 * np.cos(c1t + Xd[2]) * np.sin(c1t + Xd[2]), 1.0 / Xd[0]])
    rtol = 1e-12 if dtype == np.float64 else 2e-5
    assert ok and grad.shape == (2, 100)
    np.testing.assert_allclose(grad.astype(np.float64), want, rtol=rtol, atol=rtol)


def test_constant_gradients_population_vs_oracle_differences(ctx, oracle):
    """variable=false on a random population (F64, 2000 rows, + - * / cos sin): every per-row
    d out / d c against central differences of the oracle's predictions, where those differences are
    self-consistent; gradients of several trees come from one launch."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "sin"))
    trees = sr.random_population(24, opts, 3, np.float64, seed=17, max_size=16)
    nodes, offs = sr.flatten(trees, opts, np.float64)
    X = np.random.default_rng(18).standard_normal((3, 2000))
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    pred, grads, ok = prog.eval_grad_predict(sr.DeviceDataset(ctx, X), variable=False)
    checked = 0
    for t in range(len(trees)):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        rok_pred, rok = oracle.eval_tree(tn, opts.binop_codes, opts.unaop_codes, X)
        assert bool(ok[t]) == (rok and np.all(np.isfinite(grads[t]))), t
        if not ok[t]:
            continue
        np.testing.assert_array_equal(pred[t], rok_pred)
        cidx = [i for i in range(len(tn)) if tn[i]["degree"] == 0 and tn[i]["constant"]]
        order = []

        def rec(i):
            n = tn[i]
            if n["degree"] == 0:
                if n["constant"]:
                    order.append(i)
                return
            rec(int(n["l"]))
            if n["degree"] == 2:
                rec(int(n["r"]))

        rec(0)
        assert sorted(order) == cidx and grads[t].shape == (len(order), 2000)
        for k, i in enumerate(order):
            def fd(h):
                a, b = tn.copy(), tn.copy()
                a[i]["val"] += h
                b[i]["val"] -= h
                return (oracle.eval_tree(a, opts.binop_codes, opts.unaop_codes, X)[0]
                        - oracle.eval_tree(b, opts.binop_codes, opts.unaop_codes, X)[0]) / (2 * h)

            h = 1e-5 * max(1.0, abs(tn[i]["val"]))
            d1, d2 = fd(h), fd(h / 4)
            ref = (16 * d2 - d1) / 15
            good = np.isfinite(ref) & (np.abs(d1 - d2) <= 1e-4 * np.maximum(1.0, np.abs(ref)))
            err = np.abs(grads[t][k] - ref)[good]
            assert np.all(err <= 1e-6 * np.maximum(1.0, np.abs(ref[good]))), (t, k, err.max())
            checked += int(good.sum())
    assert checked >= 20_000


def test_derivatives_with_idx_rows(ctx):
    """Derivatives over a row subset equal the full-dataset derivatives at those rows."""
    sr = _sr()
    opts = _opts(sr)
    X = _X(np.float64)
    tree = equations(sr)[1]
    nodes, offs = sr.flatten([tree], opts, np.float64)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X)
    _, full, _ = prog.eval_grad_predict(ds, variable=True)
    idx = np.array([5, 0, 99, 42, 42, 7])
    p, sub, ok = prog.eval_grad_predict(ds, variable=True, idx=idx)
    assert ok[0] and np.array_equal(sub[0], full[0][:, idx])
