"""Generate the golden fixtures that pin the oracle (and, through it, the device path).

Julia is not installed in this container, so the reference itself cannot run: these fixtures
restate the reference's OWN known-answer tests — their trees, their operator sets, their input
shapes and their analytic ground truth — with NumPy-seeded inputs in place of Julia's
MersenneTwister streams:

  evaluation.npz         test/test_evaluation.jl:5-74        15 fusion-pattern cases, F32 3x100,
                                                              truth = the test's realfnc, tol |d|/N < 1e-6
  integer.npz            test/test_integer_evaluation.jl:1-23  x2*x3 + 2 - square(x1), Int32, exact
  nan_detection.npz      test/test_nan_detection.jl:4-48     six did_succeed == false cases x {F32, F64}
                                                              (+ benign-input controls, flag true)
  losses.npz             test/test_losses.jl:14-31           L1DistLoss and |x-y|^2.5 (LPDistLoss{2.5}),
                                                              mean and weighted, tol 1e-6
  tree_construction.npz  test/test_tree_construction.jl:8-100 f(x) = abs(3*unaop(x))^2 - (-1.2) for the
                                                              9 unary ops, eval_loss ~ 0, F32/F64
  operators.npz          test/test_operators.jl:26-71        scalar safe-op values / NaN cases

Trees are stored as srhip_node tables (include/srhip.h layout) built by the tiny independent
builder below (no product code is imported).  Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

NODE_DTYPE = np.dtype(
    [("degree", "u1"), ("constant", "u1"), ("op", "<u2"), ("feature", "<u2"), ("pad", "<u2"),
     ("l", "<i4"), ("r", "<i4"), ("val", "<f8")], align=True)

# device op codes (include/srhip.h)
C = dict(ADD=1, SUB=2, MUL=3, DIV=4, POW=5, GREATER=6, COND=7, LOGICAL_OR=8, LOGICAL_AND=9, MAX=10, MIN=11,
         NEG=32, SQUARE=33, CUBE=34, ABS=35, RELU=36, COS=37, SIN=38, TAN=39, EXP=40, LOG=41, LOG2=42,
         LOG10=43, LOG1P=44, SQRT=45, ACOSH=46, GAMMA=57)


# ---- a minimal tree builder: ("x", f) | ("c", v) | ("u", op, a) | ("b", op, a, b) -----------------
def x(f): return ("x", f)
def c(v): return ("c", v)
def u(op, a): return ("u", op, a)
def b(op, a, bb): return ("b", op, a, bb)


def to_table(tree, binops, unaops):
    rows = []

    def rec(t):
        i = len(rows)
        rows.append(None)
        if t[0] == "x":
            rows[i] = (0, 0, 0, t[1], 0, -1, -1, 0.0)
        elif t[0] == "c":
            rows[i] = (0, 1, 0, 0, 0, -1, -1, float(t[1]))
        elif t[0] == "u":
            li = rec(t[2])
            rows[i] = (1, 0, unaops.index(t[1]) + 1, 0, 0, li, -1, 0.0)
        else:
            li = rec(t[2])
            ri = rec(t[3])
            rows[i] = (2, 0, binops.index(t[1]) + 1, 0, 0, li, ri, 0.0)
        return i

    rec(tree)
    return np.array(rows, dtype=NODE_DTYPE)


def save(name, cases, **extra):
    out = {}
    for i, cs in enumerate(cases):
        for k, v in cs.items():
            out[f"c{i}_{k}"] = np.asarray(v)
    out["ncases"] = np.int64(len(cases))
    for k, v in extra.items():
        out[k] = np.asarray(v)
    np.savez(os.path.join(HERE, name), **out)


def codes(names):
    return np.array([C[n] for n in names], dtype=np.int32)


# ---- test/test_evaluation.jl ---------------------------------------------------------------------
def gen_evaluation():
    binops = ["MUL", "DIV", "ADD", "SUB"]  # options: binary_operators=(+, *, /, -) (order irrelevant)
    unaops = ["COS", "SIN"]
    f32 = np.float32
    cases_src = [
        # deg2_l0_r0_eval
        (b("MUL", x(1), x(2)), lambda x1, x2, x3: x1 * x2),
        (b("MUL", x(1), c(3.0)), lambda x1, x2, x3: x1 * f32(3.0)),
        (b("MUL", c(3.0), x(2)), lambda x1, x2, x3: f32(3.0) * x2),
        (b("MUL", c(3.0), c(6.0)), lambda x1, x2, x3: np.full_like(x1, f32(3.0) * f32(6.0))),
        # deg2_l0_eval
        (b("MUL", x(1), u("SIN", x(2))), lambda x1, x2, x3: x1 * np.sin(x2)),
        (b("MUL", c(3.0), u("SIN", x(2))), lambda x1, x2, x3: f32(3.0) * np.sin(x2)),
        # deg2_r0_eval
        (b("MUL", u("SIN", x(1)), x(2)), lambda x1, x2, x3: np.sin(x1) * x2),
        (b("MUL", u("SIN", x(1)), c(3.0)), lambda x1, x2, x3: np.sin(x1) * f32(3.0)),
        # deg1_l2_ll0_lr0_eval
        (u("COS", b("MUL", x(1), x(2))), lambda x1, x2, x3: np.cos(x1 * x2)),
        (u("COS", b("MUL", x(1), c(3.0))), lambda x1, x2, x3: np.cos(x1 * f32(3.0))),
        (u("COS", b("MUL", c(3.0), x(2))), lambda x1, x2, x3: np.cos(f32(3.0) * x2)),
        (u("COS", b("MUL", c(3.0), c(-0.5))), lambda x1, x2, x3: np.full_like(x1, np.cos(f32(3.0) * f32(-0.5)))),
        # deg1_l1_ll0_eval
        (u("COS", u("SIN", x(1))), lambda x1, x2, x3: np.cos(np.sin(x1))),
        (u("COS", u("SIN", c(3.0))), lambda x1, x2, x3: np.full_like(x1, np.cos(np.sin(f32(3.0))))),
        # everything else
        (b("MUL", b("ADD", u("SIN", b("MUL", u("COS", b("MUL", u("SIN", b("MUL", u("COS", x(1)), x(3))), c(3.0))),
                                         c(-0.5))), c(2.0)), c(5.0)),
         lambda x1, x2, x3: (np.sin(np.cos(np.sin(np.cos(x1) * x3) * f32(3.0)) * f32(-0.5)) + f32(2.0)) * f32(5.0)),
    ]
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3, 100)).astype(np.float32)
    X64 = X.astype(np.float64)
    cases = []
    for tree, fn in cases_src:
        truth = fn(X64[0], X64[1], X64[2])  # analytic truth in double from the same f32 inputs
        cases.append(dict(nodes=to_table(tree, binops, unaops), X=X, expected=np.asarray(truth, np.float64),
                          expected_ok=True, tol_per_elem=1e-6 * X.shape[1]))
    save("evaluation.npz", cases, binops=codes(binops), unaops=codes(unaops))


# ---- test/test_integer_evaluation.jl -------------------------------------------------------------
def gen_integer():
    binops = ["ADD", "MUL", "DIV", "SUB"]
    unaops = ["SQUARE"]
    tree = b("SUB", b("ADD", b("MUL", x(2), x(3)), c(2)), u("SQUARE", x(1)))
    rng = np.random.default_rng(0)
    X = rng.integers(-5, 6, size=(3, 100)).astype(np.int32)
    truth = X[1] * X[2] + np.int32(2) - X[0] * X[0]
    save("integer.npz", [dict(nodes=to_table(tree, binops, unaops), X=X, expected=truth.astype(np.int32),
                              expected_ok=True)], binops=codes(binops), unaops=codes(unaops))


# ---- test/test_nan_detection.jl ------------------------------------------------------------------
def gen_nan():
    binops = ["ADD", "MUL", "DIV", "SUB", "POW"]
    unaops = ["COS", "SIN", "EXP", "SQRT"]
    cases = []
    for dt in (np.float32, np.float64):
        src = [
            # (tree, X value, expected_ok)
            (u("EXP", u("EXP", u("EXP", u("EXP", b("ADD", x(1), c(1)))))), 100.0, False),
            (u("COS", b("DIV", x(1), c(0.0))), 100.0, False),
            (u("SQRT", b("SUB", x(1), c(1))), 0.0, False),
            (b("POW", b("SUB", x(1), c(1)), c(0.5)), 0.0, False),
            (u("COS", b("ADD", x(1), c(math.inf))), 0.0, False),
            (u("COS", b("ADD", x(1), c(math.nan))), 0.0, False),
            # controls (not in the reference): the same shapes on benign inputs succeed
            (u("EXP", u("EXP", b("ADD", x(1), c(1)))), 0.5, True),
            (u("COS", b("DIV", x(1), c(2.0))), 100.0, True),
            (u("SQRT", b("SUB", x(1), c(1))), 5.0, True),
            (b("POW", b("SUB", x(1), c(1)), c(0.5)), 5.0, True),
        ]
        for tree, xv, ok in src:
            X = np.full((1, 10), xv, dtype=dt)
            cases.append(dict(nodes=to_table(tree, binops, unaops), X=X, expected_ok=ok,
                              dtype=np.int64(0 if dt == np.float32 else 1)))
    save("nan_detection.npz", cases, binops=codes(binops), unaops=codes(unaops))


# ---- test/test_losses.jl -------------------------------------------------------------------------
def gen_losses():
    rng = np.random.default_rng(1)
    xv = rng.standard_normal(100).astype(np.float32)
    yv = rng.standard_normal(100).astype(np.float32)
    wv = np.abs(rng.standard_normal(100)).astype(np.float32)
    x64, y64, w64 = xv.astype(np.float64), yv.astype(np.float64), wv.astype(np.float64)
    cases = []
    # (kind, p0): L1DistLoss = 1; customloss(x, y) = abs(x - y)^2.5 == LPDistLoss{2.5} = kind 2
    for kind, p0, f in ((1, 0.0, lambda d: np.abs(d)), (2, 2.5, lambda d: np.abs(d) ** 2.5)):
        l = f(x64 - y64)
        cases.append(dict(kind=np.int64(kind), p0=np.float64(p0), X=xv.reshape(1, -1), y=yv, w=wv,
                          expected_mean=np.float64(l.sum() / len(l)),
                          expected_weighted=np.float64((w64 * l).sum() / w64.sum())))
    # the tree is the identity x1 (prediction == x)
    save("losses.npz", cases, nodes=to_table(x(1), ["ADD"], ["COS"]), binops=codes(["ADD"]), unaops=codes(["COS"]))


# ---- test/test_tree_construction.jl --------------------------------------------------------------
def gen_tree_construction():
    unas = [("COS", np.cos), ("EXP", np.exp), ("LOG", np.log), ("LOG2", np.log2), ("LOG10", np.log10),
            ("SQRT", np.sqrt), ("RELU", lambda v: np.where(v > 0, v, 0.0)),
            ("GAMMA", np.vectorize(math.gamma)), ("ACOSH", np.arccosh)]
    cases = []
    for name, fn in unas:
        binops = ["ADD", "MUL", "POW", "DIV", "SUB"]
        unaops = [name, "ABS"]
        # Node(5, (^)(Node(2, Node(;val=3.0) * Node(1, Node("x1"))), 2.0), Node(;val=-1.2))
        tree = b("SUB", b("POW", u("ABS", b("MUL", c(3.0), u(name, x(1)))), c(2.0)), c(-1.2))
        for dt in (np.float32, np.float64):
            rng = np.random.default_rng(0)
            if name in ("LOG", "LOG2", "LOG10", "ACOSH", "SQRT"):
                X = (rng.random((5, 100)) / 3).astype(dt)
            else:
                X = (rng.standard_normal((5, 100)) / 3).astype(dt)
            X = X + np.sign(X) * dt(0.1)
            if name == "ACOSH":
                X = X + dt(1.0)
            x1 = X[0].astype(np.float64)
            y = (np.abs(3.0 * fn(x1)) ** 2.0 - (-1.2)).astype(dt)
            tol = 3e-2 if name == "GAMMA" else 1e-6
            cases.append(dict(nodes=to_table(tree, binops, unaops), binops=codes(binops), unaops=codes(unaops),
                              X=X.astype(dt), y=y, tol=np.float64(tol)))
    save("tree_construction.npz", cases)


# ---- test/test_operators.jl: scalar semantics ----------------------------------------------------
def gen_operators():
    # (op code, arity, a, b, expected) with T in {F32, F64}; NaN expected encoded as nan
    nan = math.nan
    v, v2 = 0.5, 3.2
    rows = [
        (C["LOG"], 1, v, 0, math.log(v)), (C["LOG"], 1, -v, 0, nan),
        (C["LOG2"], 1, v, 0, math.log2(v)), (C["LOG2"], 1, -v, 0, nan),
        (C["LOG10"], 1, v, 0, math.log10(v)), (C["LOG10"], 1, -v, 0, nan),
        (C["LOG1P"], 1, v, 0, math.log1p(v)), (C["ACOSH"], 1, v2, 0, math.acosh(v2)),
        (C["ACOSH"], 1, -v2, 0, nan), (C["NEG"], 1, -v, 0, v), (C["SQRT"], 1, v, 0, math.sqrt(v)),
        (C["SQRT"], 1, -v, 0, nan), (C["MUL"], 2, v, v2, v * v2), (C["ADD"], 2, v, v2, v + v2),
        (C["SUB"], 2, v, v2, v - v2), (C["SQUARE"], 1, v, 0, v * v), (C["CUBE"], 1, v, 0, v * v * v),
        (C["POW"], 2, 0.0, -1.0, nan), (C["POW"], 2, -v, v2, nan), (C["POW"], 2, -v, -v2, nan),
        (C["POW"], 2, 0.0, -v2, nan), (C["POW"], 2, v, v2, v ** v2), (C["POW"], 2, v, -v2, v ** -v2),
        (C["POW"], 2, -1.0, 2.0, 1.0), (C["POW"], 2, -1.0, 2.1, nan),
        (C["LOG"], 1, 0.0, 0, nan), (C["LOG2"], 1, 0.0, 0, nan), (C["LOG10"], 1, 0.0, 0, nan),
        (C["LOG1P"], 1, -2.0, 0, nan),
        (C["GREATER"], 2, v, v2, 0.0), (C["GREATER"], 2, v2, v, 1.0), (C["RELU"], 1, -v, 0, 0.0),
        (C["RELU"], 1, v, 0, v), (C["LOGICAL_OR"], 2, v, v2, 1.0), (C["LOGICAL_OR"], 2, 0.0, v2, 1.0),
        (C["LOGICAL_AND"], 2, 0.0, v2, 0.0), (C["COND"], 2, v, v2, v2), (C["COND"], 2, -v, v2, 0.0),
    ]
    arr = np.array(rows, dtype=[("op", "<i4"), ("arity", "<i4"), ("a", "<f8"), ("b", "<f8"), ("expected", "<f8")])
    np.savez(os.path.join(HERE, "operators.npz"), rows=arr)


if __name__ == "__main__":
    gen_evaluation()
    gen_integer()
    gen_nan()
    gen_losses()
    gen_tree_construction()
    gen_operators()
    print("golden fixtures written to", HERE)
