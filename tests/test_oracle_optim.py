"""The oracle's restatement of the reference constant optimiser, pinned on the reference's own
known-answer test (test/test_optimizer_mutation.jl:8-42): starting from sin(x1*1.9 + 0.2) + x2*x2
on y = sin(2.1 x1 + 0.8) + x2^2, the optimiser recovers sin(c1 k + c2) ~ sin(2.1 k + 0.8) (atol 1e-3).
"""
import numpy as np


def _reference_case():
    import srhip

    opts = srhip.Options(binary_operators=("+", "-", "*"), unary_operators=("sin",))
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, 100))
    y = np.sin(X[0] * 2.1 + 0.8) + X[1] ** 2
    x1, x2 = srhip.Node("x1"), srhip.Node("x2")
    tree = srhip.sin(x1 * srhip.Node(val=1.9) + srhip.Node(val=0.2)) + x2 * x2
    nodes, offs = srhip.flatten([tree], opts, np.float64)
    return opts, X, y, nodes, offs


def test_oracle_optimizer_recovers_reference_constants():
    import optim

    opts, X, y, nodes, _ = _reference_case()
    c, loss, improved = optim.optimize_constants(nodes, opts.binop_codes, opts.unaop_codes, X, y,
                                                 rng=np.random.default_rng(1))
    assert improved
    for k in (0.0, 0.2, 0.5, 1.0):
        assert abs(np.sin(c[0] * k + c[1]) - np.sin(2.1 * k + 0.8)) < 1e-3
    assert loss < 1e-8


def test_oracle_newton_one_constant():
    """dispatch_optimize_constants uses Newton for one constant (src/ConstantOptimization.jl:27-31):
    on a quadratic objective (c * x1 vs y = 3.7 x1) one Newton step from any start lands on the
    minimum; on cos(c x1) vs cos(2.3 x1) from c = 2.0 the iteration converges to 2.3."""
    import optim
    import srhip

    rng = np.random.default_rng(3)
    X = rng.standard_normal((1, 200))
    opts = srhip.Options(binary_operators=("*",), unary_operators=("cos",))
    x1 = srhip.Node("x1")
    for tree, y, want in ((srhip.Node(val=-1.0) * x1, 3.7 * X[0], 3.7),
                          (srhip.cos(srhip.Node(val=2.0) * x1), np.cos(2.3 * X[0]), 2.3)):
        nodes, _ = srhip.flatten([tree], opts, np.float64)
        c, loss, improved = optim.optimize_constants(nodes, opts.binop_codes, opts.unaop_codes, X, y, nrestarts=0)
        assert improved and len(c) == 1
        assert abs(c[0] - want) < 1e-6, c
        assert loss < 1e-10
    # the direction is -g / |h|: on a concave stretch Newton still descends
    f = lambda c: np.cos(c[0])  # maximum at 0, concave on (-pi/2, pi/2)
    x, fx = optim.newton(f, np.array([0.3]))
    assert x[0] > 0.3 and fx < np.cos(0.3)
