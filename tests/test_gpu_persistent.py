"""The persistent interpreter launch (the wide Float32 variant's loss launches --
a probe over the leading row blocks, then one workgroup per CU claiming row blocks and
interpreting the whole population over each) returns exactly the grid launch's results, in every
configuration of its knobs, and counts the work it does."""
import numpy as np
import pytest

import srhip
from srhip import workloads

pytestmark = pytest.mark.gpu

SETTINGS = [
    {},                                   # persistent, 4-block probe with (tree, tile) claims
    {"SRHIP_PROBE_TREE_CLAIMS": "1"},     # probe claims whole trees
    {"SRHIP_PROBE_BLOCKS": "0"},          # no probe
    {"SRHIP_TAIL_SLICES": "8"},           # the last round as population slices
    {"SRHIP_PRB_ROWS": "1024"},           # shorter row blocks
    {"SRHIP_NO_PERSISTENT": "1"},         # the grid launch
    {"SRHIP_NO_EARLY_EXIT": "1"},         # every row of every tree
]


@pytest.fixture(scope="module")
def c2_small():
    opts, X, y, trees, nodes, offs = workloads.c2(0, 384, 300_000)
    return opts, X, y, nodes, offs


def test_persistent_launch_equals_grid_launch_bitwise(c2_small, oracle, monkeypatch):
    opts, X, y, nodes, offs = c2_small
    ctx = srhip.Context(0)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    assert prog.stats()["max_stack"] <= 2  # the wide variant: the persistent path
    ds = srhip.DeviceDataset(ctx, X, y)
    res = []
    for env in SETTINGS:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        l, ok = prog.eval_loss(ds, srhip.L2DistLoss())
        res.append((env, l.copy(), ok.copy(), ctx.last_work()))
        for k in env:
            monkeypatch.delenv(k)
    l0, ok0 = res[0][1], res[0][2]
    for env, l, ok, _ in res[1:]:
        assert np.array_equal(ok, ok0), env
        assert np.array_equal(l.view(np.uint64), l0.view(np.uint64)), env
    # counted work: no more than nominal; every row when the early exit is off
    for env, _, _, w in res:
        assert 0 < w["node_rows"] <= w["nominal_node_rows"], (env, w)
        assert w["tree_rows"] <= len(offs) * X.shape[1]
    full = res[-1][3]
    assert full["node_rows"] == full["nominal_node_rows"]
    assert res[0][3]["node_rows"] < full["node_rows"]  # failed trees skipped
    # and the oracle
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(ok0, ook)
    live = np.nonzero(ook)[0]
    rel = np.abs(l0[live] - ol[live]) / np.maximum(np.abs(ol[live]), 1e-300)
    assert np.all((l0[live] == ol[live]) | (rel <= 1e-6)), live[rel > 1e-6]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_superinstructions_equal_plain_programs_bitwise(c2_small, monkeypatch, dtype):
    """The leaf-leaf operand forms and the fused push + leaf load (SRHIP_NO_SUPER=1 compiles without
    them): the same losses, masks and predictions bit for bit, in the persistent launch, the grid
    launch and the prediction mode; and the programs really are shorter."""
    opts, X, y, nodes, offs = c2_small
    ctx = srhip.Context(0)
    X, y = X.astype(dtype), y.astype(dtype)
    ds = srhip.DeviceDataset(ctx, X, y)
    out = {}
    for sup in ("0", "1"):
        monkeypatch.setenv("SRHIP_NO_SUPER", sup)
        monkeypatch.setenv("SRHIP_DUMP_CODE", f"/tmp/srhip_super_{sup}.bin")
        prog = srhip.Program(ctx, nodes, offs, opts, dtype)
        monkeypatch.delenv("SRHIP_DUMP_CODE")
        res = [prog.eval_loss(ds, srhip.L2DistLoss())]
        monkeypatch.setenv("SRHIP_NO_PERSISTENT", "1")
        res.append(prog.eval_loss(ds, srhip.L2DistLoss()))
        monkeypatch.delenv("SRHIP_NO_PERSISTENT")
        pred, pok = prog.eval_predict(ds, idx=np.arange(0, X.shape[1], 7))
        res.append((pred, pok))
        out[sup] = res
        prog.close()
    for (a, b) in zip(out["0"], out["1"]):
        assert np.array_equal(a[1], b[1])
        assert np.array_equal(np.asarray(a[0]).view(np.uint8), np.asarray(b[0]).view(np.uint8))
    n_sup = (np.fromfile("/tmp/srhip_super_0.bin", dtype=np.int32).reshape(-1, 2)[:, 0] >= 0).sum()
    n_plain = (np.fromfile("/tmp/srhip_super_1.bin", dtype=np.int32).reshape(-1, 2)[:, 0] >= 0).sum()
    assert n_sup < 0.9 * n_plain, (n_sup, n_plain)


def test_lost_row_block_is_reported_then_recovered(c2_small, monkeypatch):
    """A row-block counter left non-zero (seeded through SRHIP_DEBUG_BLOCK_CTR) makes the persistent launch
    skip blocks: the host's lost-block check must report it (not return partial losses), and the next
    evaluation must zero the counter and return the clean results bit for bit."""
    opts, X, y, nodes, offs = c2_small
    ctx = srhip.Context(0)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    ds = srhip.DeviceDataset(ctx, X, y)
    l0, ok0 = prog.eval_loss(ds, srhip.L2DistLoss())
    monkeypatch.setenv("SRHIP_DEBUG_BLOCK_CTR", "7")
    with pytest.raises(RuntimeError, match="row-block counter"):
        prog.eval_loss(ds, srhip.L2DistLoss())
    monkeypatch.delenv("SRHIP_DEBUG_BLOCK_CTR")
    l1, ok1 = prog.eval_loss(ds, srhip.L2DistLoss())
    assert np.array_equal(ok1, ok0)
    assert np.array_equal(l1.view(np.uint64), l0.view(np.uint64))
