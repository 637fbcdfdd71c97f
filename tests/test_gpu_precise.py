"""The precise pass on trees whose did_succeed turns on an exact column sum near the overflow
threshold.  Each tree is c * x1 over positive x1: every row is finite, the
check statistic puts the tree in the undecided band, and the sum lands just below (ok) or just above
(fails) the threshold of the type, alternating over the population.  The device-listed pass (up to
64 listed trees, the launch's workgroups per row block sized from the program's last count, each
taking every G-th listed tree) and, for trees past a smaller list (SRHIP_PRECISE_LIST), the same
device pass over a host-written list or the host-launched pass (SRHIP_PRECISE_OVERFLOW_HOST=1) must
all give the oracle's mask, evaluation after evaluation -- including four trees within the sums' own
precision of the threshold."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu


def _sr():
    import srhip

    return srhip


@pytest.mark.parametrize("overflow", ["none", "device", "host"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_precise_pass_near_threshold_matches_oracle(ctx, oracle, dtype, overflow, monkeypatch):
    """All 14 undecided trees on the device list (none: a fresh program's launch has 4 workgroups per
    row block, each taking every 4th listed tree), or a list of 4 (SRHIP_PRECISE_LIST) whose overflow
    takes the device-listed pass over a host-written list (device) or the host-launched pass
    (SRHIP_PRECISE_OVERFLOW_HOST=1): every form gives the oracle's mask."""
    if overflow != "none":
        monkeypatch.setenv("SRHIP_PRECISE_LIST", "4")
    if overflow == "host":
        monkeypatch.setenv("SRHIP_PRECISE_OVERFLOW_HOST", "1")
    sr = _sr()
    n = 1_000_000
    rng = np.random.default_rng(17)
    x = rng.uniform(0.25, 1.0, n).astype(dtype)
    X = np.stack([x, rng.standard_normal(n).astype(dtype)])
    y = np.zeros(n, dtype=dtype)
    thr = 2.0 ** 128 - 2.0 ** 103 if dtype == np.float32 else float(np.finfo(np.float64).max)
    s = float(np.sum(x.astype(np.longdouble)))
    opts = sr.Options(binary_operators=("*", "+"), unary_operators=("cos",))
    trees, expect = [], []
    for i in range(10):
        rel = (1 - 2e-5 * (i + 1)) if i % 2 == 0 else (1 + 2e-5 * (i + 1))
        c = dtype(thr / s * rel)
        trees.append(sr.Node(1, sr.Node(val=c), sr.Node(feature=1)))  # c * x1
        expect.append(i % 2 == 0)
    # four more within the sums' own precision of the threshold (Float64: 1 +- a few 1e-12; Float32: the
    # floats next to thr / s): whichever pass decides them -- listed (double-double sums) or host-launched
    # (long double) -- must agree with the oracle's exact sum
    c0 = thr / s
    for k in range(4):
        if dtype == np.float64:
            c = c0 * (1 + (-1) ** k * (k + 1) * 3e-12)
        else:
            c = float(np.nextafter(np.float32(c0), np.float32(np.inf if k % 2 else 0)))
            c = float(np.nextafter(np.float32(c), np.float32(np.inf if k % 2 else 0))) if k >= 2 else c
        trees.append(sr.Node(1, sr.Node(val=dtype(c)), sr.Node(feature=1)))
    # ordinary trees around them
    trees += [sr.Node(2, sr.Node(feature=2), sr.Node(val=1.5)) for _ in range(6)]
    nodes, offs = sr.flatten(trees, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    _, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    ook = np.asarray(ook, bool)
    assert list(ook[:10]) == expect, "the fixture's near-threshold sums"
    psums, pchk = prog.eval_loss_partials(ds, sr.L2DistLoss())
    status = prog.finalize(X.shape[0], psums, pchk)[2]
    assert (status[:14] == 2).all(), "every near-threshold tree needs the precise pass"
    for _ in range(3):  # first evaluation: list capacity 4 (host pass for the rest); then all listed
        _, ok = prog.eval_loss(ds, sr.L2DistLoss())
        assert np.array_equal(ok, ook), (np.nonzero(ok != ook)[0], ok[:10])
    prog.close()


def test_compact_decisions_match_tree_info(ctx, oracle, monkeypatch):
    """The per-call decisions read a compact per-tree record built at compile (TreeDecide); the
    TreeInfo path (SRHIP_DECIDE_SLOW=1) must give the same losses and masks bit for bit, and both the
    oracle's mask -- over random C2-shaped trees on data with a non-finite feature value (feature
    checks), huge constants (fill-constant checks) and overflowing operator outputs."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, trees, nodes, offs = workloads.c2(5, 384, 8192)
    X = np.array(X, copy=True)
    X[3, 100] = np.inf  # every tree reading x4 fails its column check
    extra = [sr.Node(1, sr.Node(val=np.float32(3e38)), sr.Node(feature=1)),  # c * x1: overflows
             sr.Node(3, sr.Node(feature=2), sr.Node(val=np.float32(2e38))),  # x2 - c
             sr.Node(2, sr.Node(feature=1), sr.Node(val=np.float32(1.0)))]
    en, eo = sr.flatten(extra, opts, np.float32)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    loss_fast, ok_fast = prog.eval_loss(ds, sr.L2DistLoss())
    monkeypatch.setenv("SRHIP_DECIDE_SLOW", "1")
    loss_slow, ok_slow = prog.eval_loss(ds, sr.L2DistLoss())
    prog.close()
    assert np.array_equal(ok_fast, ok_slow)
    assert np.array_equal(np.asarray(loss_fast).view(np.uint64), np.asarray(loss_slow).view(np.uint64))
    _, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(ok_fast, np.asarray(ook, bool))
    assert (~ok_fast).sum() >= 3 and ok_fast.sum() > 0


def test_unfolded_add_sub_decide_as_the_oracle(ctx, oracle):
    """Float32 + and -, and * by a constant, fold no check statistic (round 6): the statistic of each (tree, row block) is
    raised to the tree's bound on its +/- outputs (cM M + cF F + c0; TreeCompiler::skip_bounds), so a
    tree is decided ok only when those sums provably stay finite, and otherwise goes to the exact
    precise pass.  Trees whose +/- arrays overflow per row, overflow only in their column sum, cancel
    to zero after huge operands (undecided by the bound, ok by the precise pass), feed an overflowing
    sum into an unchecked cos, or read a feature with a NaN only through + -- through eval_loss,
    eval_predict and the row-shard partials -- all give the oracle's did_succeed and losses."""
    sr = _sr()
    n = 300_000
    rng = np.random.default_rng(23)
    X = rng.uniform(-1.0, 1.0, (3, n)).astype(np.float32)
    y = (X[0] - 0.5 * X[1]).astype(np.float32)
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("cos", "exp"))
    x1, x2, x3 = (sr.Node(feature=i) for i in (1, 2, 3))
    c = lambda v: sr.Node(val=v)  # noqa: E731
    add = lambda a, b: sr.Node(1, a, b)  # noqa: E731
    sub = lambda a, b: sr.Node(2, a, b)  # noqa: E731
    mul = lambda a, b: sr.Node(3, a, b)  # noqa: E731
    cos = lambda a: sr.Node(1, a)  # noqa: E731
    ex = lambda a: sr.Node(2, a)  # noqa: E731
    trees = [
        add(mul(x1, c(1.5e38)), mul(x2, c(1.5e38))),         # rows finite, the column sum overflows
        sub(mul(x1, c(1.0e35)), mul(x1, c(1.0e35))),         # huge operands, exactly zero: precise -> ok
        add(mul(x1, c(3.0e38)), mul(x2, c(3.0e38))),         # rows overflow to +-Inf
        mul(cos(add(mul(x1, c(3.0e38)), mul(x2, c(3.0e38)))), c(2.0)),  # cos of an overflowing sum
        sub(add(x1, c(0.5)), x2),                            # ordinary
        add(add(mul(x1, c(1.0e30)), x2), x3),                # large, finite, decided
        add(ex(mul(x1, c(80.5))), ex(mul(x2, c(80.5)))),     # exp columns just finite, their sum's near the limit
        add(x3, c(0.5)),                                     # a feature through + only
        sub(cos(x1), cos(add(x2, x3))),                      # cos of a sum, minus a cos
        mul(c(0.0), x3),                                     # * by a constant: 0 * NaN must still fail
        mul(add(x1, x2), c(2.0e38)),                         # * by a constant overflowing per row
        cos(mul(x3, c(0.0))),                                # an unchecked cos of 0 * x3
    ]
    trees = trees + sr.random_population(40, opts, 3, np.float32, seed=29, max_size=18)
    nodes, offs = sr.flatten(trees, opts, np.float32)
    for nan_row in (None, 12345):
        Xd = X.copy()
        if nan_row is not None:
            Xd[2, nan_row] = np.nan  # x3: the trees reading it through + must fail, exactly
        ds = sr.DeviceDataset(ctx, Xd, y)
        prog = sr.Program(ctx, nodes, offs, opts, np.float32)
        ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, Xd, y, None, 0, 0.0)
        ook = np.asarray(ook, bool)
        if nan_row is None:
            assert ook[1] and ook[4] and ook[5] and not ook[2] and not ook[3], ook[:9]
        else:
            assert not ook[5] and not ook[7] and not ook[8] and not ook[9] and not ook[11]
        for _ in range(2):
            loss, ok = prog.eval_loss(ds, sr.L2DistLoss())
            assert np.array_equal(ok, ook), (np.nonzero(ok != ook)[0], nan_row)
            for t in np.nonzero(ook)[0]:  # (a succeeding tree's loss may itself overflow: Inf on both)
                assert loss[t] == ol[t] or abs(loss[t] - ol[t]) <= 1e-6 * abs(ol[t]), (t, loss[t], ol[t])
        _, pok = prog.eval_predict(ds)
        assert np.array_equal(np.asarray(pok, bool), ook)
        psums, pchk = prog.eval_loss_partials(ds, sr.L2DistLoss())
        _, fok, st = prog.finalize(Xd.shape[0], psums, pchk)
        dec = st != 2  # (undecided trees take the precise pass; decided ones must already agree)
        assert np.array_equal(np.asarray(fok, bool)[dec], ook[dec]), np.nonzero(dec & (np.asarray(fok, bool) != ook))[0]
        prog.close()


@pytest.mark.parametrize("bad", [False, True])
def test_random_extreme_constants_decide_as_the_oracle(ctx, oracle, bad):
    """The static +/- / *c bounds against random trees whose constants span 1e-2 .. 3e38 in magnitude
    (C2's operators, 600 trees): overflows per row, in column sums, under unchecked cos, through
    products with tiny and huge constants -- with clean features and with an Inf and a NaN in two of
    them.  did_succeed equals the oracle's on every tree, in loss and prediction mode."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    trees = sr.random_population(600, opts, 3, np.float32, seed=31, max_size=20)
    nodes, offs = sr.flatten(trees, opts, np.float32)
    rng = np.random.default_rng(37)
    cmask = (nodes["degree"] == 0) & (nodes["constant"] != 0)
    mag = 10.0 ** rng.uniform(-2.0, 38.5, int(cmask.sum()))
    nodes["val"][cmask] = np.minimum(mag, 3.0e38) * rng.choice([-1.0, 1.0], int(cmask.sum()))
    n = 40_000
    X = rng.uniform(-3.0, 3.0, (3, n)).astype(np.float32)
    if bad:
        X[1, 777] = np.inf
        X[2, 999] = np.nan
    y = (X[0] * 0.5).astype(np.float32)
    y[~np.isfinite(y)] = 0.0
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    ook = np.asarray(ook, bool)
    assert 50 < ook.sum() < 590, ook.sum()
    loss, ok = prog.eval_loss(ds, sr.L2DistLoss())
    assert np.array_equal(ok, ook), np.nonzero(ok != ook)[0]
    for t in np.nonzero(ook)[0]:
        assert loss[t] == ol[t] or abs(loss[t] - ol[t]) <= 1e-6 * abs(ol[t]), (t, loss[t], ol[t])
    _, pok = prog.eval_predict(ds)
    assert np.array_equal(np.asarray(pok, bool), ook)
    prog.close()
