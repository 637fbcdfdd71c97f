"""The device's Float32 sin / cos re-evaluation branch (round 6, srhip_eval_impl.h jtrigf_*): the fast
Horner-form kernels flag rows near a Float32 rounding midpoint and a wave with a flagged row takes
Julia's own kernels.  tools/check_trigf.c proves the unflagged rows; this drives EVERY flagged input
(tests/golden/trig_tie_inputs.npy, written by that checker) through each per-wave tier on the GPU --
as an operator output and as a derived feature column, in prediction and loss mode -- and requires the
oracle's bits (srm_jtrigf)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PI = np.float32(np.pi)


def _column():
    """x: groups of 4096 rows (whole tiles in every launch geometry), each holding flagged inputs of one
    tier padded with values that keep the wave in that tier: A |x| < pi/4, B |x| <= 9pi/4, C up to
    2^28 pi/2, and a slow group (a huge value in every 1024-row tile: the Payne-Hanek path)."""
    ties = np.load(os.path.join(HERE, "golden", "trig_tie_inputs.npy")).view(np.float32)
    rng = np.random.default_rng(11)
    a = np.abs(ties)
    groups = [
        (ties[a < PI / 4], 0.7),
        (ties[(a >= PI / 4) & (a <= 7.068583)], 7.0),
        (ties[a > 7.068583], 4.0e8),
        (ties, 4.0e8),
    ]
    cols = []
    for gi, (vals, lim) in enumerate(groups):
        n = -(-max(len(vals), 1) // 4096) * 4096
        pad = rng.uniform(-lim, lim, n).astype(np.float32)
        pos = rng.permutation(n)[:len(vals)]
        pad[pos] = vals
        if gi == 3:
            pad[::1024] = np.float32(3.0e30)
        cols.append(pad)
    return np.concatenate(cols), sum(len(g[0]) for g in groups)


def test_flagged_trig_inputs_take_the_exact_branch(ctx, oracle):
    import srhip

    x, nties = _column()
    assert nties > 300  # the fixture: every flagged input of every tier, both kinds
    X = np.stack([x, np.float32(1.0) + 0 * x])
    opts = srhip.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "sin"))
    x1, x2 = srhip.Node("x1"), srhip.Node("x2")
    trees = [srhip.cos(x1 * x2), srhip.sin(x1 * x2), srhip.cos(x1), srhip.sin(x1),
             srhip.cos(x1) + srhip.sin(x1 * x2)]
    nodes, offs = srhip.flatten(trees, opts, np.float32)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    pred, ok = prog.eval_predict(srhip.DeviceDataset(ctx, X))
    for t in range(len(trees)):
        ref, rok = oracle.eval_tree(nodes[offs[t]:offs[t + 1]], opts.binop_codes, opts.unaop_codes, X)
        assert bool(ok[t]) == rok, t
        if rok:
            bad = np.nonzero(pred[t].view(np.uint32) != ref.view(np.uint32))[0]
            assert len(bad) == 0, (t, bad[:8], x[bad[:8]], pred[t][bad[:8]], ref[bad[:8]])
    # loss mode (the persistent launch and its derived columns) against the oracle's losses
    y = np.zeros_like(x)
    dl, dok = prog.eval_loss(srhip.DeviceDataset(ctx, X, y), srhip.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    for t in np.nonzero(ook)[0]:
        assert dl[t] == ol[t] or abs(dl[t] - ol[t]) <= 1e-6 * abs(ol[t]), (t, dl[t], ol[t])
