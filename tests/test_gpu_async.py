"""srhip_eval_loss_submit / srhip_eval_loss_wait (include/srhip.h): evaluations queued on the context's
stream behind each other return exactly srhip_eval_loss's results -- losses bit for bit, the same
did_succeed -- whatever the number in flight and the order they are waited in, including programs
whose near-overflow trees go through the device's precise pass and row subsets (evaluated at submit).
The reference scores populations from concurrent tasks (src/SearchUtils.jl:121-122,
src/SingleIteration.jl:112); this is that seam without a parked thread per population."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_submitted_evaluations_equal_eval_loss_bitwise(ctx, oracle):
    import srhip
    from srhip import workloads

    pops = [workloads.c2(50 + i, 256, 200_000) for i in range(4)]
    opts, X, y = pops[0][0], pops[0][1], pops[0][2]
    ds = srhip.DeviceDataset(ctx, X, y)
    loss = srhip.L2DistLoss()
    # near-overflow trees (the precise pass) in the last population: x1 * c with the column sum near
    # Float32's overflow threshold
    x1 = srhip.Node("x1")
    big = [x1 * srhip.Node(val=float(v)) for v in (3.0e32, 1.0e33, 3.0e33, 1.7e33)]
    progs = []
    for i, (_, _, _, _, nodes, offs) in enumerate(pops):
        if i == 3:
            bn, bo = srhip.flatten(big, opts, np.float32)
            nodes = np.concatenate([nodes, bn])
            offs = np.concatenate([offs, bo[1:] + offs[-1]])
        progs.append((srhip.Program(ctx, nodes, offs, opts, np.float32), nodes, offs))
    want = [p.eval_loss(ds, loss) for p, _, _ in progs]
    # three in flight, waited out of order; then a fourth behind the rest
    t0, t1, t2 = (progs[i][0].eval_loss_submit(ds, loss) for i in range(3))
    got = {1: t1.wait()}
    t3 = progs[3][0].eval_loss_submit(ds, loss)
    got[0], got[3], got[2] = t0.wait(), t3.wait(), t2.wait()
    for i in range(4):
        assert np.array_equal(got[i][1], want[i][1]), i
        assert np.array_equal(got[i][0].view(np.uint64), want[i][0].view(np.uint64)), i
    # a fourth outstanding ticket on one context is refused (the first three still in flight)
    ts = [progs[i][0].eval_loss_submit(ds, loss) for i in range(3)]
    with pytest.raises(RuntimeError, match="in flight"):
        progs[3][0].eval_loss_submit(ds, loss)
    for t in ts:
        t.wait()
    # row subsets (evaluated at submit) and the oracle on the precise-pass population
    idx = np.random.default_rng(3).integers(0, X.shape[1], 5000)
    ti = progs[0][0].eval_loss_submit(ds, loss, idx=idx)
    li, oki = ti.wait()
    lw, okw = progs[0][0].eval_loss(ds, loss, idx=idx)
    assert np.array_equal(oki, okw) and np.array_equal(li.view(np.uint64), lw.view(np.uint64))
    _, nodes, offs = progs[3]
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(got[3][1], ook)
