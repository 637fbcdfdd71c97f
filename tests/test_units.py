"""dimensional_regularization's unit check (srhip.units), pinned on the reference's own expression
lists (test/test_units.jl:46-131 "Dimensional analysis", :395-426 "Dimensionless constants").  The
reference's custom_op(x, y) = x + y becomes "+"; its inv(x) cases are omitted (no device inv
operator).  Pure host logic: runs without a GPU."""
from fractions import Fraction

import numpy as np
import pytest


def _sr():
    import srhip

    return srhip


def test_uparse():
    from srhip.units import uparse

    m = uparse("m")
    assert m.value == 1.0 and m.dims[0] == 1 and sum(m.dims[1:]) == 0
    v = uparse("km/s")
    assert v.value == 1000.0 and v.dims[0] == 1 and v.dims[2] == -1
    a = uparse("m/s^2")
    assert a.dims[0] == 1 and a.dims[2] == -2
    assert uparse("m^3").dims[0] == 3 and uparse("hr").value == 3600.0 and uparse("hr").dims[2] == 1
    assert uparse("1").dimensionless() and uparse("").dimensionless()
    assert uparse("kg").value == 1.0 and uparse("kg").dims[1] == 1
    assert uparse("m^(1/2)").dims[0] == Fraction(1, 2)
    n = uparse("kg*m/s^2")
    assert n.dims == uparse("N").dims
    with pytest.raises(ValueError):
        uparse("furlong")


def test_dimensional_analysis_reference_expressions():
    sr = _sr()
    opts = sr.Options(binary_operators=("-", "*", "/", "+", "^"), unary_operators=("cos", "cbrt", "sqrt", "abs"))
    X = np.random.default_rng(0).standard_normal((3, 100))
    y = np.cos(X[2] * 2.1 - 0.2) + 0.5
    ds = sr.Dataset(X, y, X_units=["m", "1", "kg"], y_units="1")
    x1, x2, x3 = sr.Node("x1"), sr.Node("x2"), sr.Node("x3")
    C = lambda v: sr.Node(val=v)  # noqa: E731
    good = [
        C(3.2), 3.2 * x1 / x1, 1.0 * (3.2 * x1 - x2 * x1), 3.2 * x1 - x2, sr.cos(3.2 * x1),
        sr.cos(0.9 * x1 - 0.5 * x2), 1.0 * (x1 - 0.5 * (x3 * (sr.cos(0.9 * x1 - 0.5 * x2) - 1.2))),
        1.0 * (x1 + x1), 1.0 * (x1 + 2.1 * x3), 1.0 * ((x1 + 2.1 * x3) + x1), 1.0 * ((x1 + 2.1 * x3) + 0.9 * x1),
        x2, 1.0 * x1, 1.0 * x3, (1.0 * x1) ** C(3.2), 1.0 * (sr.Node("cbrt", x3 * x3 * x3) - x3),
        1.0 * (sr.Node("sqrt", x3 * x3) - x3), 1.0 * (sr.Node("sqrt", sr.Node("abs", x3) * sr.Node("abs", x3)) - x3),
    ]
    bad = [
        x1, x3, x1 - x3, 1.0 * sr.cos(x1), 1.0 * sr.cos(x1 - 0.5 * x2),
        1.0 * (x1 - (x3 * (sr.cos(0.9 * x1 - 0.5 * x2) - 1.2))), 1.0 * (x1 + x3), 1.0 * ((x1 + 2.1 * x3) + x3),
        1.0 * sr.cos(0.8606301 / x1) / sr.cos(sr.cos(x1) + 3.2263336), 1.0 * (x1 ** C(3.2)),
        1.0 * ((1.0 * x1) ** x1), 1.0 * (sr.Node("cbrt", x3 * x3) - x3), 1.0 * (sr.Node("sqrt", sr.Node("abs", x3)) - x3),
    ]
    from srhip.units import violates_dimensional_constraints as violates

    for e in good:
        assert not violates(e, ds, opts), sr.string_tree(e, opts)
    for e in bad:
        assert violates(e, ds, opts), sr.string_tree(e, opts)
    # the regularization term of _eval_loss (src/LossFunctions.jl:217-227)
    assert sr.dimensional_regularization(bad[0], ds, opts) == 1000
    assert sr.dimensional_regularization(good[0], ds, opts) == 0
    o2 = sr.Options(binary_operators=opts.binary_operators, unary_operators=opts.unary_operators,
                    dimensional_constraint_penalty=7.5)
    assert sr.dimensional_regularization(bad[0], ds, o2) == np.float64(7.5)
    assert sr.dimensional_regularization(bad[0], sr.Dataset(X, y), opts) == 0  # no units, no penalty


def test_dimensionless_constants_only():
    sr = _sr()
    X = np.random.default_rng(1).standard_normal((5, 64))
    y = np.random.default_rng(2).standard_normal(64)
    ds = sr.Dataset(X, y, X_units=["m^3", "km/s", "kg", "hr", "1"], y_units="kg")
    x1, x2, x3, x4, _ = [sr.Node(f"x{i}") for i in range(1, 6)]
    from srhip.units import violates_dimensional_constraints as violates

    strict = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "sin", "square", "cube"),
                        dimensionless_constants_only=True)
    valid = [1.5 * x1 / (sr.Node("cube", x2) * sr.Node("cube", x4)) * x3, x3, (sr.Node("square", x3) / x3) + x3]
    invalid = [sr.Node(val=1.5), 1.5 * x1, x3 - 1.0 * x1]
    for e in valid:
        assert not violates(e, ds, strict), sr.string_tree(e, strict)
    for e in invalid:
        assert violates(e, ds, strict), sr.string_tree(e, strict)
    loose = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "sin"))
    for e in invalid:
        assert not violates(e, ds, loose), sr.string_tree(e, loose)


def test_y_units_alone_make_features_dimensionless():
    sr = _sr()
    ds = sr.Dataset(np.ones((2, 4)), np.ones(4), y_units="m")
    assert ds.has_units() and all(u.dimensionless() for u in ds.X_units)
    from srhip.units import violates_dimensional_constraints as violates

    opts = sr.Options(binary_operators=("*",))
    assert violates(sr.Node("x1"), ds, opts)                      # dimensionless output, y in m
    assert not violates(sr.Node(val=2.0) * sr.Node("x1"), ds, opts)  # wildcard output
