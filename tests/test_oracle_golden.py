"""Pin the oracle: it must reproduce the reference's own known-answer tests (CPU, no GPU).

Each test restates one reference test file (see tests/golden/make_golden.py for the mapping)
and applies that file's own tolerance.
"""
import math

import numpy as np
import pytest

from conftest import load_cases


def test_evaluation_fusion_patterns(oracle):
    """test/test_evaluation.jl:5-74 — every DynamicExpressions fusion branch; |d|/N < 1e-6."""
    cases, ex = load_cases("evaluation.npz")
    assert len(cases) == 15
    for cs in cases:
        out, ok = oracle.eval_tree(cs["nodes"], ex["binops"], ex["unaops"], cs["X"])
        assert ok
        n = cs["X"].shape[1]
        assert np.all(np.abs(out.astype(np.float64) - cs["expected"]) / n < 1e-6)


def test_integer_evaluation(oracle):
    """test/test_integer_evaluation.jl:1-23 — Int32 tree, output stays Int32, exact, flag true."""
    cases, ex = load_cases("integer.npz")
    cs = cases[0]
    out, ok = oracle.eval_tree(cs["nodes"], ex["binops"], ex["unaops"], cs["X"])
    assert ok
    assert out.dtype == np.int32
    assert np.array_equal(out, cs["expected"])


def test_nan_detection(oracle):
    """test/test_nan_detection.jl:4-48 — six did_succeed == false cases (F32, F64) + controls."""
    cases, ex = load_cases("nan_detection.npz")
    assert len(cases) == 20
    for cs in cases:
        _, ok = oracle.eval_tree(cs["nodes"], ex["binops"], ex["unaops"], cs["X"])
        assert ok == bool(cs["expected_ok"])


def test_losses(oracle):
    """test/test_losses.jl:14-31 — _loss (mean) and _weighted_loss (sum(w l)/sum(w)); 1e-6."""
    cases, ex = load_cases("losses.npz")
    for cs in cases:
        le, lr, ok = oracle.eval_loss(ex["nodes"], ex["binops"], ex["unaops"], cs["X"], cs["y"], None,
                                      int(cs["kind"]), float(cs["p0"]))
        assert ok
        assert abs(le - float(cs["expected_mean"])) < 1e-6
        assert abs(lr - float(cs["expected_mean"])) < 1e-6
        le, lr, ok = oracle.eval_loss(ex["nodes"], ex["binops"], ex["unaops"], cs["X"], cs["y"], cs["w"],
                                      int(cs["kind"]), float(cs["p0"]))
        assert ok
        assert abs(le - float(cs["expected_weighted"])) < 1e-6
        assert abs(lr - float(cs["expected_weighted"])) < 1e-6


def test_tree_construction_losses(oracle):
    """test/test_tree_construction.jl:45-87 — exact trees: complete, eval ~ y, eval_loss ~ 0."""
    cases, _ = load_cases("tree_construction.npz")
    assert len(cases) == 18
    for cs in cases:
        X = cs["X"]
        out, ok = oracle.eval_tree(cs["nodes"], cs["binops"], cs["unaops"], X)
        assert ok
        n = X.shape[1]
        tol = float(cs["tol"])
        assert np.all(np.abs(out.astype(np.float64) - cs["y"].astype(np.float64)) / n < tol)
        le, _, ok = oracle.eval_loss(cs["nodes"], cs["binops"], cs["unaops"], X, cs["y"])
        assert ok and abs(le) < tol


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_operator_values(oracle, dtype):
    """test/test_operators.jl:26-71 — safe-op values, NaN cases, Bool strong-zero ops."""
    rows = np.load(__import__("conftest").GOLDEN + "/operators.npz", allow_pickle=False)["rows"]
    for r in rows:
        if r["arity"] == 1:
            got = float(oracle.scalar_un(int(r["op"]), r["a"], dtype))
        else:
            got = float(oracle.scalar_bin(int(r["op"]), r["a"], r["b"], dtype))
        exp = float(r["expected"])
        if math.isnan(exp):
            assert math.isnan(got), r
        else:
            assert abs(got - exp) < 1e-6, (r, got)


def test_relu_cond_strong_zero(oracle):
    """src/Operators.jl:82-96: Julia Bool * x is a strong zero — relu(NaN) == 0, cond(-1, NaN) == 0."""
    for dt in (np.float32, np.float64):
        assert oracle.scalar_un(36, float("nan"), dt) == 0.0
        assert oracle.scalar_bin(7, -1.0, float("nan"), dt) == 0.0
        assert math.copysign(1.0, float(oracle.scalar_un(36, -3.0, dt))) == -1.0  # relu(-3) == -0.0
