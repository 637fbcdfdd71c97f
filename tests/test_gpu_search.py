"""Device path of the search: the native coalescer and a search whose every
score runs on the MI355X (A12/A14)."""
import threading

import numpy as np
import pytest

import srhip
from srhip import search as S

pytestmark = pytest.mark.gpu

OPS = dict(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))


def _data(n=100, seed=0, dtype=np.float64):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((2, n)).astype(dtype)
    y = (2 * np.cos(X[1]) + X[0] ** 2 - 2).astype(dtype)
    return X, y


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_coalescer_equals_single_program(dtype):
    """8 threads x 40 single-tree requests: every coalesced result equals the same tree's result in
    one whole-population launch, bit for bit; fewer launches than requests."""
    o = srhip.Options(**OPS)
    X, y = _data(5000, dtype=dtype)
    trees = srhip.random_population(320, o, 2, dtype, seed=3, max_size=20)
    nodes, offs = srhip.flatten(trees, o, dtype)
    ref_ctx = srhip.Context(0)
    ref_loss, ref_ok = srhip.Program(ref_ctx, nodes, offs, o, dtype).eval_loss(
        srhip.DeviceDataset(ref_ctx, X, y), srhip.L2DistLoss())
    ctx = srhip.Context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    co = srhip.Coalescer(ctx, ds, o, srhip.L2DistLoss(), max_batch=64, max_wait_us=500, nclients=8)
    got = [None] * len(trees)

    def client(k):
        for i in range(k, len(trees), 8):
            got[i] = co.score_loss(nodes[offs[i]:offs[i + 1]])

    th = [threading.Thread(target=client, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    st = co.stats()
    co.close()
    for i, (l, ok) in enumerate(got):
        assert ok == bool(ref_ok[i]), i
        if ok:
            assert l == ref_loss[i], (i, l, ref_loss[i])
    assert st["requests"] == len(trees)
    assert st["launches"] < len(trees) // 2, st
    assert st["max_batch"] > 1


def test_coalescer_attributes_errors():
    """A malformed tree in a batch fails only its own request."""
    o = srhip.Options(**OPS)
    X, y = _data(300)
    ctx = srhip.Context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    co = srhip.Coalescer(ctx, ds, o, srhip.L2DistLoss(), max_batch=8, max_wait_us=2000)
    good, _ = srhip.flatten([srhip.Node("x1") * srhip.Node(val=2.0)], o, np.float64)
    bad, _ = srhip.flatten([srhip.Node("x1") * srhip.Node(feature=9)], o, np.float64)  # feature 9 of 2
    t1, t2, t3 = co.submit(good), co.submit(bad), co.submit(good)
    l1, ok1 = co.wait(t1)
    with pytest.raises(srhip.SrhipError):
        co.wait(t2)
    l3, ok3 = co.wait(t3)
    co.close()
    assert ok1 and ok3 and l1 == l3
    assert abs(l1 - np.mean((2 * X[0] - y) ** 2)) <= 1e-12 * l1


def test_device_search_finds_readme_equation():
    """C1-shaped search (README: y = 2cos(x2) + x1^2 - 2, 2 x 100 Float64), every score on the
    device: the best hall-of-fame loss falls far below the constant baseline, and the HoF losses
    equal fresh device evaluations of their trees."""
    X, y = _data()
    o = srhip.Options(populations=8, population_size=33, ncycles_per_iteration=100, maxsize=20,
                      deterministic=True, seed=1, **OPS)
    print("search start", flush=True)
    res = S.equation_search(X, y, o, niterations=10)
    front = res.pareto_frontier()
    best = min(m.loss for m in front)
    base = np.mean((y - y.mean()) ** 2)
    print(f"best loss {best:.3g} (baseline {base:.3g}); coalescer {res.coalescer_stats}", flush=True)
    assert best < 0.05 * base
    assert res.coalescer_stats["launches"] < res.coalescer_stats["requests"]
    d = srhip.Dataset(X, y)
    losses, _ = srhip.eval_loss_batch([m.tree for m in front], d, o)
    for m, l in zip(front, losses):
        assert abs(l - m.loss) <= 1e-12 * max(1.0, abs(l)) or (np.isinf(l) and np.isinf(m.loss))


def test_device_search_multiprocessing_equals_threads():
    """parallelism='multiprocessing' on the device: 4 islands in 2 worker
    processes, each scoring through its own coalescer on its resident dataset and optimising
    constants on its own context, return the threaded device search's hall of fame exactly."""
    X, y = _data()
    o = srhip.Options(populations=4, population_size=20, ncycles_per_iteration=40, maxsize=15,
                      deterministic=True, seed=5, **OPS)
    threaded = S.equation_search(X, y, o, niterations=2)
    mp = S.equation_search(X, y, o, niterations=2, parallelism="multiprocessing", procs=2, devices=[0])
    f0 = [(srhip.string_tree(m.tree, o), m.loss) for m in threaded.pareto_frontier()]
    f1 = [(srhip.string_tree(m.tree, o), m.loss) for m in mp.pareto_frontier()]
    assert f0 == f1
    assert mp.num_evals == threaded.num_evals
    assert mp.coalescer_stats["requests"] == threaded.coalescer_stats["requests"]
    assert mp.node_rows == threaded.node_rows


def test_device_scorer_adds_units_penalty():
    """The search's scorer (score_func -> eval_loss(regularization=true), src/LossFunctions.jl:70-71,
    161-174) adds dimensional_regularization like eval_loss does: a violating tree's coalesced loss
    equals eval_loss on the units dataset, penalty included; a conforming tree pays nothing."""
    X = np.random.default_rng(5).standard_normal((3, 1000))
    y = np.cos(X[2] * 2.1 - 0.2) + 0.5
    opts = srhip.Options(binary_operators=("-", "*", "/", "+"), unary_operators=("cos",))
    ds = srhip.Dataset(X, y, X_units=["m", "1", "kg"], y_units="1")
    x1, x2 = srhip.Node("x1"), srhip.Node("x2")
    good, bad = srhip.cos(3.2 * x1) - x2, srhip.cos(x1) + x2
    sc = S.DeviceScorer(ds, opts)
    try:
        for tree, pen in ((good, 0.0), (bad, 1000.0)):
            _, loss = sc.score(tree)
            assert loss == srhip.eval_loss(tree, ds, opts), srhip.string_tree(tree, opts)
            assert loss - srhip.eval_loss(tree, ds, opts, regularization=False) == pytest.approx(pen)
    finally:
        sc.close()


def test_distributed_search_world1_native_exchange_equals_identity(monkeypatch):
    """The island search's per-iteration exchange through libsrhip's RCCL communicator
    (parallel.IterationExchange over NativeComm.allgather, world size 1) returns the hall of fame the
    same lock-step search returns with the exchange as an in-process identity: every member, score,
    loss and size count survives the fixed-size payload's device round trip unchanged
    (src/SymbolicRegression.jl:910-943, src/Migration.jl:16-38)."""
    from srhip import parallel

    X, y = _data(200, seed=4)

    def run(native):
        monkeypatch.setenv("SRHIP_SEARCH_COMM", "native" if native else "torch")
        calls = []
        orig = parallel.IterationExchange.exchange

        def spy(self, *a, **k):
            calls.append(self.comm is not None)
            return orig(self, *a, **k)

        monkeypatch.setattr(parallel.IterationExchange, "exchange", spy)
        o = srhip.Options(populations=3, population_size=20, ncycles_per_iteration=30, deterministic=True, seed=5,
                          maxsize=15, **OPS)
        res = S.equation_search(X, y, o, niterations=2, distributed=True)
        monkeypatch.setattr(parallel.IterationExchange, "exchange", orig)
        return res, calls

    rn, cn = run(True)
    ri, ci = run(False)
    assert cn == [True, True] and ci == [False, False]  # the library's communicator vs the identity
    fn = [(str(m.tree), m.loss, m.score) for m in rn.pareto_frontier()]
    fi = [(str(m.tree), m.loss, m.score) for m in ri.pareto_frontier()]
    assert fn == fi and len(fn) > 0
