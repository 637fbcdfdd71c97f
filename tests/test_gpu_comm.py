"""libsrhip's native multi-GPU exchanges (csrc/srhip_comm.cpp, RCCL) through the C ABI, at world
size 1 on one MI355X: the row-sharded evaluation equals the single-device evaluation bit for bit
(including trees whose overflow check needs the precise pass), the migration all-gather returns
this rank's k best trees as packed, and the raw all-reduce / all-gather are identities.  The
multi-rank protocol (what every rank sends and how it combines) is covered by the gloo world-2
tests of tests/test_distributed.py; RCCL cannot place two ranks on one device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sr():
    import srhip

    return srhip


@pytest.fixture(scope="module")
def comm(ctx):
    from srhip import parallel

    c = parallel.NativeComm(ctx, 1, 0, parallel.NativeComm.unique_id())
    yield c
    c.close()


def _population(sr, opts, n, nfeat, dtype, seed):
    trees = sr.random_population(n, opts, nfeat, dtype, seed=seed, max_size=30)
    nodes, offs = sr.flatten(trees, opts, dtype)
    return trees, nodes, offs


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_native_sharded_eval_world1_equals_eval_loss(ctx, comm, oracle, dtype):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    _, nodes, offs = _population(sr, opts, 200, 3, dtype, seed=5)
    x1 = sr.Node("x1")
    big = 3e37 if dtype == np.float32 else 1e306
    extra = [sr.exp(sr.exp(x1)) * sr.Node(val=1e30 if dtype == np.float32 else 1e300), x1 * sr.Node(val=big)]
    en, eo = sr.flatten(extra, opts, dtype)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    rng = np.random.default_rng(6)
    X = rng.standard_normal((3, 300_000)).astype(dtype)
    X[0, :] = np.abs(X[0, :]) + 1.0
    y = (np.cos(X[1]) * 2 + X[2] ** 2).astype(dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    full_l, full_ok = prog.eval_loss(ds, sr.L2DistLoss())
    sl, sok = comm.eval_loss_sharded(prog, ds, sr.L2DistLoss())
    assert np.array_equal(sok, full_ok)
    assert np.array_equal(sl, full_l)
    # the same through a row subset (batching idx)
    idx = rng.integers(0, X.shape[1], size=5000)
    il, iok = prog.eval_loss(ds, sr.L2DistLoss(), idx=idx)
    sl2, sok2 = comm.eval_loss_sharded(prog, ds, sr.L2DistLoss(), idx=idx)
    assert np.array_equal(sok2, iok) and np.array_equal(sl2, il)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(sok, ook)


def test_native_migrate_topk_world1(ctx, comm):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    _, nodes, offs = _population(sr, opts, 64, 3, np.float32, seed=9)
    rng = np.random.default_rng(10)
    losses = rng.random(64)
    losses[[3, 7]] = np.inf
    losses[11] = np.nan
    k, mx = 12, 30
    got = comm.migrate_topk(nodes, offs, losses, k, mx)
    assert len(got) == 1
    nd, of, ls = got[0]
    key = np.where(np.isfinite(losses), losses, np.inf)
    order = [int(t) for t in np.argsort(key, kind="stable") if offs[t + 1] - offs[t] <= mx][:k]
    assert len(of) == len(order) + 1 and np.array_equal(ls, losses[order])
    for i, t in enumerate(order):
        a, b = offs[t], offs[t + 1]
        assert np.array_equal(nd[of[i]:of[i + 1]].view(np.uint8), nodes[a:b].view(np.uint8))
    # the same selection as the torch-path packer (parallel._pack_topk), byte for byte
    from srhip import parallel

    payload, head = parallel._pack_topk(nodes, offs, losses, k, mx)
    ref = parallel._unpack_topk(payload[None, :], 1, head, k)[0]
    assert np.array_equal(ref[1], of) and np.array_equal(ref[2], ls)
    assert np.array_equal(ref[0].view(np.uint8), nd.view(np.uint8))
    # in flight while an evaluation runs on the context's stream
    X = rng.standard_normal((3, 100_000)).astype(np.float32)
    y = X[0].copy()
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    ds = sr.DeviceDataset(ctx, X, y)
    pend = comm.migrate_start(nodes, offs, losses, k, mx)
    prog.eval_loss(ds, sr.L2DistLoss())
    nd2, of2, ls2 = pend.wait()[0]
    assert np.array_equal(of2, of) and np.array_equal(ls2, ls)


def test_native_allreduce_allgather_world1(comm):
    a = np.array([1.5, -2.0, np.inf, 3.25])
    assert np.array_equal(comm.allreduce_f64(a, "sum"), a)
    assert np.array_equal(comm.allreduce_f64(a, "max"), a)
    blob = bytes(range(200))
    assert comm.allgather(blob) == [blob]


def test_bench_selfcheck_comparisons_world1(ctx, comm):
    """The bench's pre-timing check of the library's exchanges against torch.distributed's (bench.py
    _native_selfcheck) compares like with like: at world size 1 (a one-rank gloo group in this
    process) the native migration equals parallel.migrate_topk (parallel.same_migrants) and the
    native sharded evaluation equals parallel.eval_loss_sharded bit for bit."""
    import socket

    import torch.distributed as dist

    from srhip import parallel

    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    _, nodes, offs = _population(sr, opts, 64, 3, np.float32, seed=21)
    rng = np.random.default_rng(22)
    X = rng.standard_normal((3, 5000)).astype(np.float32)
    y = (X[0] * X[1] - 0.5).astype(np.float32)
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    loss = sr.L2DistLoss()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        l0, _ = prog.eval_loss(ds, loss)
        a = comm.migrate_topk(nodes, offs, l0, 12, 30)
        b = parallel.migrate_topk(nodes, offs, l0, 12, 30)
        assert parallel.same_migrants(a, b)
        b2 = [(b[0][0], b[0][1], np.asarray(b[0][2], np.float64) * 2.0)]
        assert not parallel.same_migrants(a, b2)
        la, oka = comm.eval_loss_sharded(prog, ds, loss)
        lb, okb = parallel.eval_loss_sharded(prog, 3, lambda: prog.eval_loss_partials(ds, loss),
                                             precise=lambda tr: prog.eval_precise_partials(ds, tr))
        assert np.asarray(la, np.float64).tobytes() == np.asarray(lb, np.float64).tobytes()
        assert np.array_equal(oka, okb)
    finally:
        prog.close()
        if own:
            dist.destroy_process_group()


def test_sharded_lost_row_block_is_reported_then_recovered(ctx, comm, monkeypatch):
    """The row-shard path's lost-block check: a seeded non-zero row-block counter is reported
    from the shard's own rows (a tree with a finite all-reduced statistic verifies the launch); the next
    sharded evaluation zeroes the counter and equals the clean one bit for bit."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, _, nodes, offs = workloads.c2(1, 128, 300_000)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    assert prog.stats()["max_stack"] <= 2  # the wide variant: the persistent path
    ds = sr.DeviceDataset(ctx, X, y)
    l0, ok0 = comm.eval_loss_sharded(prog, ds, sr.L2DistLoss())
    assert ok0.any()
    monkeypatch.setenv("SRHIP_DEBUG_BLOCK_CTR", "5")
    with pytest.raises(RuntimeError, match="row-block counter"):
        comm.eval_loss_sharded(prog, ds, sr.L2DistLoss())
    monkeypatch.delenv("SRHIP_DEBUG_BLOCK_CTR")
    l1, ok1 = comm.eval_loss_sharded(prog, ds, sr.L2DistLoss())
    assert np.array_equal(ok1, ok0) and np.array_equal(l1.view(np.uint64), l0.view(np.uint64))
