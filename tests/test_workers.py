"""`:multiprocessing` worker <-> GPU mapping and dataset residency (srhip.workers; SURVEY.md §8(f)
row 4, reference src/SymbolicRegression.jl:964-987 / src/Configure.jl:309-343).  The host backend
drives the pool machinery on the CPU; tests/test_gpu_workers.py runs device workers."""
import os

import numpy as np
import pytest


def _sr():
    import srhip.workers as w

    return w


def task_crash(worker, ds):
    os._exit(3)


def task_echo(worker, ds, x):
    return worker.index, x * 2


def test_worker_device_mapping_round_robin():
    w = _sr()
    with w.GPUWorkerPool(4, devices=[0, 1, 2], backend="host") as pool:
        assert [pool.device_of(i) for i in range(4)] == [0, 1, 2, 0]
        info = sorted(pool.map(w.task_info, [None] * 8))
        assert {i for i, _, _ in info} == {0, 1, 2, 3}
        assert all(dev == pool.device_of(i) for i, dev, _ in info)


def test_dataset_resident_once_per_worker():
    """Every worker maps the dataset once at registration; tasks name it by key and carry no
    dataset bytes, so many tasks leave the per-worker upload count at 1."""
    w = _sr()
    X = np.random.default_rng(0).standard_normal((3, 5000)).astype(np.float32)
    y = X[0] * 2
    with w.GPUWorkerPool(2, backend="host") as pool:
        key = pool.register_dataset(X, y)
        sums = [pool.submit(w.task_column_sums, dataset=key).result(timeout=60) for _ in range(6)]
        for s in sums:
            np.testing.assert_array_equal(s, X.sum(axis=1))
        info = pool.map(w.task_info, [None] * 4)
        assert {u for _, _, u in info} == {1}
        assert pool.map(task_echo, [1, 2, 3]) == [(0, 2), (1, 4), (0, 6)]


def test_dead_worker_respawns_with_datasets():
    w = _sr()
    X = np.arange(12, dtype=np.float64).reshape(3, 4)
    with w.GPUWorkerPool(2, backend="host") as pool:
        key = pool.register_dataset(X)
        fut = pool.submit(task_crash, worker=1)
        with pytest.raises(w.WorkerDied):
            fut.result(timeout=60)
        assert pool.ensure_workers() == 1 and pool.respawns == 1
        # the respawned worker re-attached the dataset from shared memory
        np.testing.assert_array_equal(pool.submit(w.task_column_sums, dataset=key, worker=1).result(timeout=60),
                                      X.sum(axis=1))
        assert pool.submit(w.task_info, worker=1).result(timeout=60)[2] == 1


def test_task_error_is_reported():
    w = _sr()
    with w.GPUWorkerPool(1, backend="host") as pool:
        with pytest.raises(RuntimeError, match="KeyError"):
            pool.submit(w.task_column_sums, dataset=99).result(timeout=60)
        assert pool.submit(task_echo, 5).result(timeout=60) == (0, 10)
