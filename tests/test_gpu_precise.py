"""The precise pass on trees whose did_succeed turns on an exact column sum near the overflow
threshold.  Each tree is c * x1 over positive x1: every row is finite, the
check statistic puts the tree in the undecided band, and the sum lands just below (ok) or just above
(fails) the threshold of the type, alternating over the population.  The device-listed pass (one
tree group per listed tree) and the host-launched pass for trees past the list's capacity (the
first evaluation of a program lists at most 4) must both give the oracle's mask, evaluation after
evaluation -- including four trees within the sums' own precision of the threshold.  Trees past the first
evaluation's list capacity go through the same device pass over a host-written list (or, with
SRHIP_PRECISE_OVERFLOW_HOST=1, the host-launched pass)."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu


def _sr():
    import srhip

    return srhip


@pytest.mark.parametrize("overflow", ["device", "host"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_precise_pass_near_threshold_matches_oracle(ctx, oracle, dtype, overflow, monkeypatch):
    """Trees past the device list's capacity take the device-listed pass over a host-written list
    (default) or the host-launched pass (SRHIP_PRECISE_OVERFLOW_HOST=1): both give the oracle's mask."""
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
