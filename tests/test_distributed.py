"""The multi-GPU protocols of srhip.parallel on CPU (gloo, world_size 2).

Row shards: each rank computes its shard's partials with the oracle (standing in for the device),
the ranks all-reduce, and libsrhip's host-side finalize (a host-only program: no device touched)
must reproduce the oracle's unsharded eval_loss (losses to 1e-12 relative, identical did_succeed).
Islands: migration's all-gather of node tables returns every rank's trees intact.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = dict(binary_operators=("+", "-", "*", "/"), unary_operators=("cos",))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem(dtype, n=1500, ntrees=48, seed=5):
    import srhip

    opts = srhip.Options(**OPS)
    trees = srhip.random_population(ntrees, opts, 3, dtype, seed=seed, max_size=25)
    nodes, offs = srhip.flatten(trees, opts, dtype)
    rng = np.random.default_rng(seed + 1)
    X = rng.standard_normal((3, n)).astype(dtype)
    y = (np.cos(X[0]) * 2 + X[1] ** 2).astype(dtype)
    w = rng.uniform(0.5, 2.0, n).astype(dtype)
    return opts, nodes, offs, X, y, w


def test_shard_rows_partition():
    from srhip.parallel import shard_rows

    for n in (0, 1, 7, 1000, 1001):
        for ws in (1, 2, 3, 8):
            blocks = [shard_rows(n, r, ws) for r in range(ws)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
            sizes = [hi - lo for lo, hi in blocks]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("weighted", [False, True])
def test_host_finalize_matches_oracle(oracle, dtype, weighted):
    """Single process: oracle partials of the whole dataset -> libsrhip finalize == oracle eval_loss."""
    import srhip

    opts, nodes, offs, X, y, w = _problem(dtype)
    w = w if weighted else None
    prog = srhip.Program(None, nodes, offs, opts, dtype)
    sums, chk = oracle.partials(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, w)
    loss, ok, status = prog.finalize(X.shape[0], sums, chk)
    assert not np.any(status == 2)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, w, 0, 0.0)
    assert np.array_equal(ok, ook)
    np.testing.assert_allclose(loss[ook], ol[ook], rtol=1e-12)
    assert np.all(np.isinf(loss[~ook]))


def _rank_main(rank, world, port, dtype_name, q):
    try:
        sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
        import torch.distributed as dist

        import oracle
        import srhip
        from srhip.parallel import allgather_trees, eval_loss_sharded, shard_rows

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        dtype = np.dtype(dtype_name).type
        opts, nodes, offs, X, y, w = _problem(dtype)
        lo, hi = shard_rows(X.shape[1], rank, world)
        prog = srhip.Program(None, nodes, offs, opts, dtype)
        part = lambda: oracle.partials(nodes, offs, opts.binop_codes, opts.unaop_codes,  # noqa: E731
                                       X[:, lo:hi], y[lo:hi], w[lo:hi])
        loss, ok = eval_loss_sharded(prog, X.shape[0], part)
        # migration exchange: rank r contributes its own trees
        mine = srhip.random_population(3 + rank, opts, 3, dtype, seed=100 + rank, max_size=12)
        mn, mo = srhip.flatten(mine, opts, dtype)
        got = allgather_trees(mn, mo)
        q.put((rank, loss, ok, [(g[0].tobytes(), g[1]) for g in got]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_row_sharded_and_migration_gloo_world2(oracle, dtype):
    import multiprocessing as mp

    import srhip

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, np.dtype(dtype).name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[2] is not None, r[1]
    opts, nodes, offs, X, y, w = _problem(dtype)
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, w, 0, 0.0)
    for _, loss, ok, _ in res:
        assert np.array_equal(ok, ook)
        np.testing.assert_allclose(loss[ook], ol[ook], rtol=1e-12)
    assert np.array_equal(res[0][1], res[1][1])  # identical decision on every rank
    for rank in range(2):
        mine = srhip.random_population(3 + rank, opts, 3, dtype, seed=100 + rank, max_size=12)
        mn, mo = srhip.flatten(mine, opts, dtype)
        for _, _, _, got in res:
            assert got[rank][0] == mn.tobytes()
            assert np.array_equal(got[rank][1], mo)


def _search_rank_main(rank, world, port, q):
    """One rank of the island search (C3 protocol) with the oracle scorer standing in for the GPU."""
    try:
        sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"),
                        os.path.join(ROOT, "tests")]
        import torch.distributed as dist

        import oracle
        import srhip
        from srhip import search as S
        from test_search import OracleScorer, _data

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        X, y = _data(100, seed=3)
        o = srhip.Options(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"),
                          populations=4, population_size=20, ncycles_per_iteration=30, maxsize=15, seed=9,
                          should_optimize_constants=False)
        d = srhip.Dataset(X, y)
        d.baseline_loss, d.use_baseline = np.float64(np.mean((y - y.mean()) ** 2)), True
        sc = OracleScorer(d, o, oracle)
        res = S.equation_search(d, None, o, niterations=3, scorer=sc)
        front = [(srhip.string_tree(m.tree, o), m.loss) for m in res.pareto_frontier()]
        q.put((rank, front, len(res.populations), res.num_evals, sc.calls))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(e), None, None, None))


def test_island_search_gloo_world2():
    """C3's protocol at world size 2: each rank evolves its half of the populations; after every
    iteration the ranks exchange best_sub_pops + hall-of-fame frontiers (all-gather) and migrate
    from the global set, so both ranks end with the same hall of fame, which beats the constant
    baseline."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_search_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[2] is not None, r[1]
    (_, f0, np0, ne0, c0), (_, f1, np1, ne1, c1) = res
    assert np0 == 2 and np1 == 2          # populations 0,2 on rank 0; 1,3 on rank 1
    assert ne0 == ne1 and ne0 >= c0 + c1 - 1  # global evaluation count on every rank
    assert [l for _, l in f0] == [l for _, l in f1]  # one global hall of fame
    import srhip  # noqa: F401
    from test_search import _data

    X, y = _data(100, seed=3)
    assert min(l for _, l in f0) < 0.5 * np.mean((y - y.mean()) ** 2)


def _migrate_rank_main(rank, world, port, q):
    """One rank of the bench's per-step exchanges: migrate_topk (fixed-size all-gather) and
    allreduce_partials (one buffer, SUM + MAX)."""
    try:
        sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
        import torch.distributed as dist

        import srhip
        from srhip.parallel import allreduce_partials, migrate_topk

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        opts = srhip.Options(**OPS)
        trees = srhip.random_population(20 + 5 * rank, opts, 3, np.float32, seed=200 + rank, max_size=25)
        nodes, offs = srhip.flatten(trees, opts, np.float32)
        losses = np.random.default_rng(300 + rank).uniform(0, 10, len(trees))
        losses[::4] = np.inf  # failed trees never migrate ahead of finite ones
        got = migrate_topk(nodes, offs, losses, k=6, max_nodes=20)
        sums = np.arange(7, dtype=np.float64) * (rank + 1)
        chk = np.array([1.0 + rank, np.nan if rank == 1 else 2.0, 3.0 - rank])
        rs, rc = allreduce_partials(sums, chk, "max")
        q.put((rank, [(g[0].tobytes(), g[1], g[2]) for g in got], rs, rc))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(e), None, None))


def test_migrate_topk_and_fused_allreduce_gloo_world2():
    """The multi-GPU bench's collectives at world size 2: every rank receives every rank's 6 best
    trees (finite losses first, trees over 20 nodes skipped) bit for bit with their losses, and the
    one-buffer partials all-reduce sums the sums and takes the max of the check statistics (a NaN
    sent as +Inf)."""
    import multiprocessing as mp

    import srhip

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_migrate_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[2] is not None, r[1]
    opts = srhip.Options(**OPS)
    for rank in range(2):
        trees = srhip.random_population(20 + 5 * rank, opts, 3, np.float32, seed=200 + rank, max_size=25)
        nodes, offs = srhip.flatten(trees, opts, np.float32)
        losses = np.random.default_rng(300 + rank).uniform(0, 10, len(trees))
        losses[::4] = np.inf
        order = np.argsort(losses, kind="stable")
        sel = [t for t in order if offs[t + 1] - offs[t] <= 20][:6]
        want = b"".join(nodes[offs[t]:offs[t + 1]].tobytes() for t in sel)
        for _, got, _, _ in res:
            nd, of, ls = got[rank]
            assert nd == want
            assert np.array_equal(ls, losses[sel])
            assert np.array_equal(np.diff(of), [offs[t + 1] - offs[t] for t in sel])
    for _, _, rs, rc in res:
        assert np.array_equal(rs, np.arange(7, dtype=np.float64) * 3)
        assert np.array_equal(rc, [2.0, np.inf, 3.0])


def _overflow_rank_main(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))
        import torch.distributed as dist

        import srhip
        from srhip.parallel import IterationExchange

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        opts = srhip.Options(**OPS)
        # capacity for 4 members of <= 8 nodes; rank 1 sends 10 members of up to 25 nodes (a custom
        # complexity mapping lets trees outgrow maxsize + 1 nodes), rank 0 stays within it
        ex = IterationExchange(4, 4 * 8, 3, comm=None, group=None, world=world)
        n = 2 if rank == 0 else 10
        trees = srhip.random_population(n, opts, 3, np.float32, seed=400 + rank, max_size=25 if rank else 5)
        got = ex.exchange(trees, np.arange(n) + 0.5, np.arange(n) * 2.0, 7 + rank, [1.0, 2.0, 3.0 + rank], opts,
                          np.float32)
        second = ex.last_overflow
        # a following exchange within capacity takes one round again
        got2 = ex.exchange(trees[:1], [1.0], [2.0], 0, [0.0, 0.0, 0.0], opts, np.float32)
        out = [(nsub, [(srhip.flatten([t], opts, np.float32)[0].tobytes(), s, l) for t, s, l in mem], list(c))
               for nsub, mem, c in got]
        q.put((rank, None, out, (second, ex.last_overflow, len(got2))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(e), None, None))


def test_iteration_exchange_overflow_is_collective_gloo_world2():
    """IterationExchange with one rank past the capacity: no rank raises alone; every rank
    sees the overflow flag, both repeat the exchange once at the largest need, and every rank receives
    every rank's members intact."""
    import multiprocessing as mp

    import srhip

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[2] is not None, r[1]
    opts = srhip.Options(**OPS)
    for rank in range(2):
        n = 2 if rank == 0 else 10
        trees = srhip.random_population(n, opts, 3, np.float32, seed=400 + rank, max_size=25 if rank else 5)
        want = [srhip.flatten([t], opts, np.float32)[0].tobytes() for t in trees]
        for _, _, out, _ in res:
            nsub, mem, counts = out[rank]
            assert nsub == 7 + rank
            assert [m[0] for m in mem] == want
            assert [m[1] for m in mem] == list(np.arange(n) + 0.5)
            assert [m[2] for m in mem] == list(np.arange(n) * 2.0)
            assert counts == [1.0, 2.0, 3.0 + rank]
    for _, _, _, (second, after, n2) in res:
        assert second is not None and second[0] == 10
        assert after is None and n2 == 2
