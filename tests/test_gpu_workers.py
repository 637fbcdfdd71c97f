"""Device workers of srhip.workers.GPUWorkerPool (`:multiprocessing` <-> GPU mapping, SURVEY.md
§8(f) row 4): two worker processes on device 0 score populations against a dataset registered
once; every loss and did_succeed equals the in-process evaluation bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_worker_pool_scores_equal_in_process(ctx):
    import srhip
    import srhip.workers as w

    opts = srhip.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    rng = np.random.default_rng(3)
    X = rng.standard_normal((5, 100_000)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    pops = []
    for s in range(4):
        trees = srhip.random_population(64, opts, 5, np.float32, seed=40 + s, max_size=30)
        pops.append(srhip.flatten(trees, opts, np.float32))
    ds = srhip.DeviceDataset(ctx, X, y)
    want = []
    for nodes, offs in pops:
        prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
        want.append(prog.eval_loss(ds, srhip.L2DistLoss()))
        prog.close()
    with w.GPUWorkerPool(2, devices=[0]) as pool:
        key = pool.register_dataset(X, y)
        futs = [pool.submit(w.task_eval_loss, nodes, offs, opts, dataset=key) for nodes, offs in pops]
        got = [f.result(timeout=120) for f in futs]
        info = [pool.submit(w.task_info, worker=i).result(timeout=60) for i in range(2)]
    for (gl, gok), (wl, wok) in zip(got, want):
        assert np.array_equal(gok, wok)
        assert np.array_equal(gl, wl)
    assert [(i, d, u) for i, d, u in info] == [(0, 0, 1), (1, 0, 1)]
