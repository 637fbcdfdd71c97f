"""Device (libsrhip, through the C ABI) vs oracle vs golden fixtures.  Needs an MI355X.

Tolerances (north_star): losses within 1e-6 relative (Float32) / 1e-12 relative (Float64) of
the oracle's exact-sum loss; bit-exact for Int32; identical did_succeed masks.
"""
import math

import numpy as np
import pytest

from conftest import GOLDEN, load_cases

pytestmark = pytest.mark.gpu

F32_REL = 1e-6
F64_REL = 1e-12


def _sr():
    import srhip

    return srhip


def _program(ctx, nodes, offsets, binops, unaops, dtype):
    sr = _sr()
    opts = _codes_options(binops, unaops)
    return sr.Program(ctx, nodes, offsets, opts, dtype)


class _CodeOptions:
    """Minimal options carrying raw device op codes (golden fixtures store codes)."""

    def __init__(self, binops, unaops):
        import ctypes

        from srhip._lib import Operators

        self.binop_codes = np.ascontiguousarray(binops, dtype=np.int32)
        self.unaop_codes = np.ascontiguousarray(unaops, dtype=np.int32)
        ops = Operators()
        ops.nbin, ops.nuna = len(self.binop_codes), len(self.unaop_codes)
        ops.binops = self.binop_codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        ops.unaops = self.unaop_codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        self._ops = ops

    def c_operators(self):
        return self._ops


def _codes_options(b, u):
    return _CodeOptions(b, u)


def _one(nodes):
    return np.array([0, len(nodes)], dtype=np.int64)


def _ds(ctx, X, y=None, w=None):
    sr = _sr()
    return sr.DeviceDataset(ctx, X, y, w)


def assert_same_bits(pred, ref, what=""):
    """Predictions equal bit for bit; on failure every differing row with its distance in ULPs."""
    pred, ref = np.ascontiguousarray(pred), np.ascontiguousarray(ref)
    it = np.uint32 if pred.dtype.itemsize == 4 else np.uint64
    pb, rb = pred.view(it), ref.view(it)
    bad = np.nonzero(pb != rb)[0]
    if len(bad):
        ulps = [abs(int(pb[i]) - int(rb[i])) if (pred[i] >= 0) == (ref[i] >= 0) else -1 for i in bad[:16]]
        raise AssertionError(f"{what}: {len(bad)} rows differ; first (row, device, oracle, ulps): "
                             f"{[(int(i), pred[i], ref[i], u) for i, u in zip(bad[:16], ulps)]}")


def _rel(a, b):
    if a == b or (math.isnan(a) and math.isnan(b)):  # equal infinities / both NaN
        return 0.0
    return abs(a - b) / max(abs(b), 1e-300)


# ---- golden fixtures --------------------------------------------------------------------------
def test_golden_evaluation(ctx, oracle):
    cases, ex = load_cases("evaluation.npz")
    for cs in cases:
        prog = _program(ctx, cs["nodes"], _one(cs["nodes"]), ex["binops"], ex["unaops"], np.float32)
        pred, ok = prog.eval_predict(_ds(ctx, cs["X"]))
        assert ok[0]
        n = cs["X"].shape[1]
        assert np.all(np.abs(pred[0].astype(np.float64) - cs["expected"]) / n < 1e-6)
        ref, rok = oracle.eval_tree(cs["nodes"], ex["binops"], ex["unaops"], cs["X"])
        assert rok == bool(ok[0])
        assert_same_bits(pred[0], ref)


def test_golden_integer(ctx, oracle):
    cases, ex = load_cases("integer.npz")
    cs = cases[0]
    prog = _program(ctx, cs["nodes"], _one(cs["nodes"]), ex["binops"], ex["unaops"], np.int32)
    pred, ok = prog.eval_predict(_ds(ctx, cs["X"]))
    assert ok[0] and pred.dtype == np.int32
    assert np.array_equal(pred[0], cs["expected"])
    ref, _ = oracle.eval_tree(cs["nodes"], ex["binops"], ex["unaops"], cs["X"])
    assert np.array_equal(pred[0], ref)


def test_golden_nan_detection(ctx, oracle):
    cases, ex = load_cases("nan_detection.npz")
    for cs in cases:
        dt = np.float32 if int(cs["dtype"]) == 0 else np.float64
        prog = _program(ctx, cs["nodes"], _one(cs["nodes"]), ex["binops"], ex["unaops"], dt)
        _, ok = prog.eval_predict(_ds(ctx, cs["X"]))
        assert bool(ok[0]) == bool(cs["expected_ok"])
        y = np.zeros(cs["X"].shape[1], dtype=dt)
        loss, lok = prog.eval_loss(_ds(ctx, cs["X"], y), _sr().L2DistLoss())
        assert bool(lok[0]) == bool(cs["expected_ok"])
        assert math.isinf(loss[0]) == (not cs["expected_ok"])


def test_golden_losses(ctx, oracle):
    sr = _sr()
    cases, ex = load_cases("losses.npz")
    nodes = ex["nodes"]
    for cs in cases:
        kind, p0 = int(cs["kind"]), float(cs["p0"])
        loss = sr.L1DistLoss() if kind == 1 else sr.LPDistLoss(p0)
        prog = _program(ctx, nodes, _one(nodes), ex["binops"], ex["unaops"], np.float32)
        l, ok = prog.eval_loss(_ds(ctx, cs["X"], cs["y"]), loss)
        assert ok[0] and abs(l[0] - float(cs["expected_mean"])) < 1e-6
        l, ok = prog.eval_loss(_ds(ctx, cs["X"], cs["y"], cs["w"]), loss)
        assert ok[0] and abs(l[0] - float(cs["expected_weighted"])) < 1e-6


def test_golden_tree_construction(ctx, oracle):
    sr = _sr()
    cases, _ = load_cases("tree_construction.npz")
    for cs in cases:
        X, y = cs["X"], cs["y"]
        prog = _program(ctx, cs["nodes"], _one(cs["nodes"]), cs["binops"], cs["unaops"], X.dtype)
        pred, ok = prog.eval_predict(_ds(ctx, X))
        tol = float(cs["tol"])
        assert ok[0]
        assert np.all(np.abs(pred[0].astype(np.float64) - y.astype(np.float64)) / X.shape[1] < tol)
        l, lok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
        assert lok[0] and abs(l[0]) < tol


# ---- random populations ------------------------------------------------------------------------
OPS_C2 = dict(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))


def _population(sr, opts, ntrees, nfeat, dtype, seed, max_size=30):
    trees = sr.random_population(ntrees, opts, nfeat, dtype, seed, max_size)
    return trees, *sr.flatten(trees, opts, dtype)


def _data(nfeat, n, dtype, seed, weighted=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((nfeat, n)).astype(dtype)
    y = (2 * np.cos(X[min(3, nfeat - 1)].astype(np.float64)) + X[0].astype(np.float64) ** 2 - 2
         + 0.1 * rng.standard_normal(n)).astype(dtype)
    w = np.abs(rng.standard_normal(n)).astype(dtype) if weighted else None
    return X, y, w


@pytest.mark.parametrize("dtype,n,weighted", [
    (np.float32, 4099, False), (np.float32, 777, True), (np.float64, 3001, False), (np.float64, 1000, True),
])
def test_random_population_losses(ctx, oracle, dtype, n, weighted):
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    trees, nodes, offs = _population(sr, opts, 192, 5, dtype, seed=11)
    X, y, w = _data(5, n, dtype, seed=12, weighted=weighted)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    dl, dok = prog.eval_loss(_ds(ctx, X, y, w), sr.L2DistLoss())
    ol, orl, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, w, 0, 0.0)
    assert np.array_equal(dok, ook), np.nonzero(dok != ook)
    tol = F32_REL if dtype == np.float32 else F64_REL
    bad = [(t, dl[t], ol[t]) for t in np.nonzero(ook)[0] if _rel(dl[t], ol[t]) > tol]
    assert not bad, bad[:5]
    assert np.all(np.isinf(dl[~dok]))


@pytest.mark.parametrize("dtype,n", [(np.float32, 100), (np.float64, 100), (np.float32, 2000), (np.float64, 1000)])
def test_fused_single_block_reduction_equals_reduce_kernel(ctx, oracle, dtype, n, monkeypatch):
    """Single-row-block launches (small datasets, C1's 100 rows) finish each tree's reduction in the
    interpreter wave, in the reduce kernel's order: the same bits as the reduce kernel
    (SRHIP_NO_FUSED_REDUCE=1), the oracle's losses, and the coalescer's deferred one-copy upload."""
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    trees, nodes, offs = _population(sr, opts, 96, 2, dtype, seed=21, max_size=20)
    X, y, _ = _data(2, n, dtype, seed=22)
    ds = _ds(ctx, X, y, None)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    a, aok = prog.eval_loss(ds, sr.L2DistLoss())
    monkeypatch.setenv("SRHIP_NO_FUSED_REDUCE", "1")
    b, bok = prog.eval_loss(ds, sr.L2DistLoss())
    monkeypatch.delenv("SRHIP_NO_FUSED_REDUCE")
    assert np.array_equal(aok, bok) and np.array_equal(a.view(np.uint64), b.view(np.uint64))
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(aok, ook)
    tol = F32_REL if dtype == np.float32 else F64_REL
    assert not [t for t in np.nonzero(ook)[0] if _rel(a[t], ol[t]) > tol]
    # the coalescer (deferred upload: program and tree order in one copy) scores the same bits
    co = sr.Coalescer(ctx, ds, opts, sr.L2DistLoss(), max_wait_us=0)
    try:
        for t in range(0, 96, 7):
            loss, ok = co.score_loss(nodes[offs[t]:offs[t + 1]])
            assert bool(ok) == bool(aok[t]) and (not ok or np.float64(loss).view(np.uint64) == a[t:t + 1].view(np.uint64)[0])
    finally:
        co.close()


def test_random_population_predictions(ctx, oracle):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "sin", "exp"))
    trees, nodes, offs = _population(sr, opts, 64, 3, np.float32, seed=5)
    X, _, _ = _data(3, 1029, np.float32, seed=6)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    pred, ok = prog.eval_predict(_ds(ctx, X))
    for t in range(len(trees)):
        ref, rok = oracle.eval_tree(nodes[offs[t]:offs[t + 1]], opts.binop_codes, opts.unaop_codes, X)
        assert bool(ok[t]) == rok, t
        if rok:  # the same IEEE operations per row on both sides (-ffp-contract=off, one libm header)
            assert_same_bits(pred[t], ref, f"tree {t}")


def test_int32_population_bit_exact(ctx, oracle):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("square", "neg"))
    rng = np.random.default_rng(3)
    trees = sr.random_population(96, opts, 3, np.float64, seed=4)
    for tr in trees:  # integer constants
        for nd in tr:
            if nd.degree == 0 and nd.constant:
                nd.val = int(rng.integers(-7, 8))
    nodes, offs = sr.flatten(trees, opts, np.int32)
    X = rng.integers(-1000, 1000, size=(3, 2053)).astype(np.int32)
    y = rng.integers(-50, 50, size=2053).astype(np.int32)
    prog = sr.Program(ctx, nodes, offs, opts, np.int32)
    pred, ok = prog.eval_predict(_ds(ctx, X))
    assert ok.all()
    for t in range(len(trees)):
        ref, rok = oracle.eval_tree(nodes[offs[t]:offs[t + 1]], opts.binop_codes, opts.unaop_codes, X)
        assert rok and np.array_equal(pred[t], ref), t
    dl, dok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook) and np.array_equal(dl, ol)


@pytest.mark.parametrize("kind_name,args", [
    ("L1DistLoss", ()), ("LPDistLoss", (3.0,)), ("HuberLoss", (0.7,)), ("L1EpsilonInsLoss", (0.2,)),
    ("L2EpsilonInsLoss", (0.3,)), ("LogitDistLoss", ()), ("PeriodicLoss", (2.5,)), ("QuantileLoss", (0.3,)),
])
def test_loss_kinds(ctx, oracle, kind_name, args):
    sr = _sr()
    loss = getattr(sr, kind_name)(*args)
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 48, 4, np.float64, seed=21, max_size=12)
    X, y, _ = _data(4, 1500, np.float64, seed=22)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    dl, dok = prog.eval_loss(_ds(ctx, X, y), loss)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, loss.kind,
                                           loss.p0)
    assert np.array_equal(dok, ook)
    for t in np.nonzero(ook)[0]:
        assert _rel(dl[t], ol[t]) < 1e-10, (t, dl[t], ol[t])


def test_idx_batching(ctx, oracle):
    """eval_loss(...; idx) == loss over X[:, idx] (src/LossFunctions.jl:36-42,52-54)."""
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 40, 5, np.float32, seed=31)
    X, y, w = _data(5, 5000, np.float32, seed=32, weighted=True)
    idx = np.random.default_rng(33).integers(0, 5000, size=50)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    for ww in (None, w):
        dl, dok = prog.eval_loss(_ds(ctx, X, y, ww), sr.L2DistLoss(), idx=idx)
        ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X[:, idx].copy(),
                                               y[idx].copy(), None if ww is None else ww[idx].copy(), 0, 0.0)
        assert np.array_equal(dok, ook)
        for t in np.nonzero(ook)[0]:
            assert _rel(dl[t], ol[t]) < F32_REL


# ---- did_succeed edge semantics ------------------------------------------------------------------
def _eval1(ctx, sr, tree, X, opts, dtype=np.float32):
    nodes, offs = sr.flatten([tree], opts, dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    pred, ok = prog.eval_predict(_ds(ctx, X))
    return pred[0], bool(ok[0]), nodes


def test_overflowing_sum_of_finite_values_fails(ctx, oracle):
    """isfinite(sum(array)) is false for finite elements whose sum overflows (parity with the
    oracle's exact-sum rule; exercises the device's precise pass)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos",))
    x1 = sr.Node("x1")
    for c, expect in ((1e37, False), (1e35, True), (5e36, True)):
        X = np.ones((1, 100), dtype=np.float32)
        tree = sr.cos(x1) * sr.Node(val=c) + x1  # every element finite
        pred, ok, nodes = _eval1(ctx, sr, tree, X, opts)
        _, rok = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, X)
        assert ok == rok == expect, (c, ok, rok)


def test_constant_trees_and_leaves(ctx, oracle):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))
    X = np.random.default_rng(0).standard_normal((2, 37)).astype(np.float32)
    cases = [
        sr.Node(val=1.5),                                  # constant root
        sr.Node("x2"),                                     # feature root
        sr.cos(sr.Node(val=3.0)) * sr.Node("x1"),          # folded constant subtree
        sr.Node("x1") + sr.exp(sr.exp(sr.Node(val=100.0))),  # failing constant subtree
        sr.Node("x1") / sr.Node(val=0.0),                  # -> Inf elements
        sr.Node(val=3e38) * sr.Node(val=10.0),             # constant overflow
        sr.Node(val=1e37),                                 # fill(1e37, 37): sum overflows
        sr.Node("x1") * sr.Node(val=float("inf")),         # non-finite constant leaf
        sr.exp(sr.Node(val=float("-inf"))) + sr.Node("x1"),  # exp(-Inf) = 0 in the scalar path: ok
    ]
    for tree in cases:
        pred, ok, nodes = _eval1(ctx, sr, tree, X, opts)
        ref, rok = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, X)
        assert ok == rok, sr.string_tree(tree, opts)
        if ok:
            assert_same_bits(pred, ref, sr.string_tree(tree, opts))


def test_feature_column_checks(ctx, oracle):
    """A feature evaluated as a child array (under a non-fused unary node, or as the root) has its
    column checked; features consumed inline by fused kernels are not."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos", "exp"))
    X = np.ones((2, 50), dtype=np.float32)
    X[0, 7] = np.inf
    x1, x2 = sr.Node("x1"), sr.Node("x2")
    for tree in (x1, sr.cos(x1), sr.cos(sr.exp(x1)), sr.cos(x1) + x2, x2 * x1, sr.exp(sr.cos(x1)) + x2,
                 sr.cos(sr.Node(val=0.0) * x1), x2 + sr.cos(x2)):
        _, ok, nodes = _eval1(ctx, sr, tree, X, opts)
        _, rok = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, X)
        assert ok == rok, sr.string_tree(tree, opts)


@pytest.mark.parametrize("n", [1, 7, 63, 64, 65, 511, 512, 513, 4095, 4096, 4097, 9000])
def test_ragged_row_counts(ctx, oracle, n):
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 24, 3, np.float32, seed=n)
    X, y, _ = _data(3, n, np.float32, seed=n + 1)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    dl, dok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    for t in np.nonzero(ook)[0]:
        assert _rel(dl[t], ol[t]) < F32_REL


def test_deep_trees_use_large_stack(ctx, oracle):
    """Balanced trees need Strahler-number stack slots (K=8 kernel variant)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*", "-"), unary_operators=("cos",))

    def bal(d, k):
        if d == 0:
            return sr.Node(f"x{1 + k % 3}") if k % 2 else sr.Node(val=0.5 + 0.01 * k)
        return (bal(d - 1, 2 * k) if k % 3 else sr.cos(bal(d - 1, 2 * k))) + bal(d - 1, 2 * k + 1) * sr.Node(val=0.9)

    trees = [bal(d, 1) for d in (3, 5, 6, 7)]
    nodes, offs = sr.flatten(trees, opts, np.float32)
    X, y, _ = _data(3, 1000, np.float32, seed=9)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    assert prog.stats()["max_stack"] >= 5
    dl, dok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    for t in np.nonzero(ook)[0]:
        assert _rel(dl[t], ol[t]) < F32_REL


def test_all_operators_single_values(ctx, oracle):
    """Every device operator against the oracle on a grid of values (incl. domain edges)."""
    sr = _sr()
    from srhip.operators import BINARY, UNARY

    vals = np.array([-3.7, -1.0, -0.5, -0.0, 0.0, 0.3, 0.5, 1.0, 1.5, 2.0, 7.25, 40.0, -40.0, 1e-3], dtype=np.float64)
    for dtype in (np.float32, np.float64):
        una = sorted({v[0] for v in UNARY.values()})
        bina = sorted({v[0] for v in BINARY.values()})
        opts = sr.Options(binary_operators=bina, unary_operators=una)
        X = np.stack([np.repeat(vals, len(vals)), np.tile(vals, len(vals))]).astype(dtype)
        trees = [sr.Node(name, sr.Node("x1")) for name in una]
        trees += [sr.Node(name, sr.Node("x1"), sr.Node("x2")) for name in bina]
        nodes, offs = sr.flatten(trees, opts, dtype)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        pred, _ = prog.eval_predict(_ds(ctx, X))
        for t, tree in enumerate(trees):
            name = tree.op
            if tree.degree == 1:
                ref = np.array([oracle.scalar_un(opts.unaop_codes[opts.unary_index(name) - 1], v, dtype) for v in X[0]])
            else:
                ref = np.array([oracle.scalar_bin(opts.binop_codes[opts.binary_index(name) - 1], a, b, dtype)
                                for a, b in zip(X[0], X[1])])
            got = pred[t]
            same_nan = np.isnan(got) == np.isnan(ref)
            assert same_nan.all(), (name, dtype, X[:, ~same_nan], got[~same_nan], ref[~same_nan])
            fin = ~np.isnan(ref)
            rtol = 4e-6 if dtype == np.float32 else 1e-14
            if name in ("gamma", "^"):
                rtol = 2e-5 if dtype == np.float32 else 1e-13
            np.testing.assert_allclose(got[fin], ref[fin], rtol=rtol, atol=1e-30, err_msg=f"{name} {dtype}")


# ---- large sizes: size-independent properties ------------------------------------------------------
def test_c2_shape_subset_matches_oracle(ctx, oracle):
    """C2 shape (5 features x 1M rows, F32, ops + - * / cos exp, sizes U{1..30}) on 32 trees."""
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 32, 5, np.float32, seed=2)
    X, y, _ = _data(5, 1_000_000, np.float32, seed=0)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    dl, dok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    ol, orl, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    for t in np.nonzero(ook)[0]:
        assert _rel(dl[t], ol[t]) < F32_REL, (t, dl[t], ol[t], orl[t])


def test_row_permutation_invariance_and_determinism(ctx):
    """Loss is invariant (to rounding) under a row permutation; repeated calls are bit-identical.
    Float32 losses sum each lane's 4 consecutive rows in Float32 before widening (relative error
    <= 2^-23, srhip_eval_impl.h loss_tile), so a permutation moves the loss at that level -- inside
    the 1e-6 parity bar, and far inside the reference's own sequential Float32 sum."""
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 64, 5, np.float32, seed=41)
    X, y, _ = _data(5, 300_000, np.float32, seed=42)
    perm = np.random.default_rng(43).permutation(X.shape[1])
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    a, aok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    a2, _ = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    b, bok = prog.eval_loss(_ds(ctx, X[:, perm].copy(), y[perm].copy()), sr.L2DistLoss())
    assert np.array_equal(a, a2)
    assert np.array_equal(aok, bok)
    for t in np.nonzero(aok)[0]:
        assert _rel(a[t], b[t]) < 2.5e-7


def test_set_constants_matches_fresh_compile(ctx):
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    trees, nodes, offs = _population(sr, opts, 16, 3, np.float64, seed=51, max_size=15)
    X, y, _ = _data(3, 2000, np.float64, seed=52)
    ds = _ds(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    nconst = prog.num_constants()
    rng = np.random.default_rng(53)
    new = rng.standard_normal(int(nconst.sum()))
    prog.set_constants(new)
    a, aok = prog.eval_loss(ds, sr.L2DistLoss())
    k = 0
    for tr, nc in zip(trees, nconst):
        sr.set_constants(tr, new[k:k + nc])
        k += nc
    n2, o2 = sr.flatten(trees, opts, np.float64)
    b, bok = sr.Program(ctx, n2, o2, opts, np.float64).eval_loss(ds, sr.L2DistLoss())
    assert np.array_equal(aok, bok) and np.array_equal(a, b)


# ---- the reference-shaped Python API ---------------------------------------------------------------
def test_reference_api_eval_loss_and_score(ctx):
    """eval_loss == score_func(...)[2] (test/test_tree_construction.jl:86-87); parsimony and
    baseline effects (:90-99)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*", "^", "/", "-"), unary_operators=("cos", "abs"))
    X = (np.random.default_rng(0).standard_normal((5, 100)) / 3).astype(np.float32)
    X = X + np.sign(X) * np.float32(0.1)
    f = lambda v: np.abs(3.0 * np.cos(v)) ** 2.0 - (-1.2)
    y = f(X[0].astype(np.float64)).astype(np.float32)
    ds = sr.Dataset(X, y)
    x1 = sr.Node("x1")
    tree = sr.Node("-", sr.Node("^", sr.Node("abs", sr.Node(val=3.0) * sr.cos(x1)), sr.Node(val=2.0)), sr.Node(val=-1.2))
    out, ok = sr.eval_tree_array(tree, X, opts)
    assert ok and np.all(np.abs(out - y) / 100 < 1e-6)
    l = sr.eval_loss(tree, ds, opts)
    assert abs(l) < 1e-6 and l == sr.score_func(ds, tree, opts)[1]
    assert abs(sr.score_func(ds, tree, sr.Options(binary_operators=opts.binary_operators,
                                                 unary_operators=opts.unary_operators, parsimony=0.0))[0]) < 1e-6
    assert sr.score_func(ds, tree, sr.Options(binary_operators=opts.binary_operators,
                                             unary_operators=opts.unary_operators, parsimony=1.0))[0] > 1.0
    sr.update_baseline_loss(ds, opts)
    assert ds.use_baseline and ds.baseline_loss > 0


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_row_sharded_partials_match_single_device(ctx, oracle, dtype):
    """Two row shards on one device, combined as srhip.parallel combines ranks (sum / max), equal the
    unsharded evaluation; includes trees whose overflow check needs the precise pass."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    _, nodes, offs = _population(sr, opts, 96, 3, dtype, seed=77)
    # near-overflow trees: exp(exp(x1)) * c and x1 * 1e37 (finite values whose sums may overflow)
    x1 = sr.Node("x1")
    big = 3e37 if dtype == np.float32 else 1e306
    extra = [sr.exp(sr.exp(x1)) * sr.Node(val=1e30 if dtype == np.float32 else 1e300), x1 * sr.Node(val=big)]
    en, eo = sr.flatten(extra, opts, dtype)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    X, y, _ = _data(3, 5000, dtype, seed=3)
    X[0, :] = np.abs(X[0, :]) + 1.0
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    full_l, full_ok = prog.eval_loss(_ds(ctx, X, y), sr.L2DistLoss())
    parts = [prog.eval_loss_partials(_ds(ctx, X[:, a:b], y[a:b]), sr.L2DistLoss()) for a, b in ((0, 2100), (2100, 5000))]
    sums = parts[0][0] + parts[1][0]
    chk = np.maximum(parts[0][1], parts[1][1]) if prog.chk_reduce_op() == "max" else parts[0][1] + parts[1][1]
    loss, ok, status = prog.finalize(3, sums, chk)
    und = np.nonzero(status == 2)[0].astype(np.int32)
    if len(und):
        ops = sum(prog.eval_precise_partials(_ds(ctx, X[:, a:b], y[a:b]), und) for a, b in ((0, 2100), (2100, 5000)))
        uok = prog.precise_finalize(und, ops)
        ok[und] = uok
        loss[und] = np.where(uok, sums[2 * und] / sums[2 * und + 1], np.inf)
    assert np.array_equal(ok, full_ok)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(ok, ook)
    for t in np.nonzero(ok)[0]:
        assert _rel(loss[t], full_l[t]) < 1e-12


def test_loss_in_reference_type_L(ctx, oracle):
    """_eval_loss returns the dataset's loss type L (Float32 for Float32 data; _loss folds in T,
    src/LossFunctions.jl:13-33,45-75): srhip.eval_loss / score_func return L scalars, and the
    device's L-typed loss is the oracle's exact loss rounded to L -- equal, or one ULP of L apart
    where the exact losses (within 1e-6) straddle a rounding boundary of L."""
    sr = _sr()
    opts = sr.Options(**OPS_C2)
    trees, nodes, offs = _population(sr, opts, 160, 3, np.float32, seed=61)
    X, y, _ = _data(3, 20000, np.float32, seed=62)
    d = sr.Dataset(X, y)
    dl, dok = sr.eval_loss_batch(trees, d, opts)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    live = np.nonzero(ook)[0]
    dL, oL = dl[live].astype(np.float32), ol[live].astype(np.float32)
    ulps = np.abs(dL.view(np.int32).astype(np.int64) - oL.view(np.int32).astype(np.int64))
    assert np.all(ulps <= 1), live[ulps > 1]
    assert np.mean(ulps == 0) >= 0.85  # the device's Float32 4-row group sums: <= 2^-23 from exact
    for t in live[:20]:
        v = sr.eval_loss(trees[t], d, opts)
        assert isinstance(v, np.float32) and v == np.float32(dl[t])
        s, l2 = sr.score_func(d, trees[t], opts)
        assert isinstance(l2, np.float32) and isinstance(s, np.float32)


MARGIN_LOSSES = [("ZeroOneLoss", ()), ("PerceptronLoss", ()), ("LogitMarginLoss", ()), ("L1HingeLoss", ()),
                 ("L2HingeLoss", ()), ("SmoothedL1HingeLoss", (0.6,)), ("ModifiedHuberLoss", ()),
                 ("L2MarginLoss", ()), ("ExpLoss", ()), ("SigmoidLoss", ()), ("DWDMarginLoss", (1.5,))]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("kind_name,args", MARGIN_LOSSES)
def test_margin_loss_kinds(ctx, oracle, kind_name, args, dtype):
    """The LossFunctions margin losses the reference lists (src/Options.jl:220-229), of the agreement
    target * output, fused into the interpreter: device == oracle (same masks; losses within 1e-10
    for Float64, the Float32 parity bar for Float32).  Targets are +-1 (binary classification)."""
    sr = _sr()
    loss = getattr(sr, kind_name)(*args)
    opts = sr.Options(**OPS_C2)
    _, nodes, offs = _population(sr, opts, 48, 4, dtype, seed=41, max_size=12)
    X, _, _ = _data(4, 1500, dtype, seed=42)
    y = np.where(np.random.default_rng(43).standard_normal(1500) > 0, 1.0, -1.0).astype(dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    dl, dok = prog.eval_loss(_ds(ctx, X, y), loss)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, loss.kind,
                                           loss.p0)
    assert np.array_equal(dok, ook)
    tol = 1e-10 if dtype == np.float64 else F32_REL
    for t in np.nonzero(ook)[0]:
        assert _rel(dl[t], ol[t]) < tol, (t, dl[t], ol[t])
    assert ook.sum() >= 24
