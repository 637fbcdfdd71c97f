"""`:multiprocessing` for the device path: worker processes bound to GPUs, datasets resident on
them.

The reference starts Distributed workers (`addprocs`, src/Configure.jl:309-343) and ships every
population's cycle to one with `@spawnat` (src/SymbolicRegression.jl:964-987, through
`@sr_spawner`, src/SearchUtils.jl:108-127).  The spawned closure captures `dataset`, so the whole
dataset is serialized into every task.  Here:

* worker i owns device ``devices[i % len(devices)]`` (one libsrhip context per worker process, the
  one-context-per-task model of device.py);
* ``register_dataset`` copies X / y / weights ONCE into POSIX shared memory; every worker maps it and
  uploads it to its device once, and tasks name the dataset by key -- a task carries only
  populations (node tables, a few KB);
* a worker that died is respawned by ``ensure_workers`` (called before every submit) and re-attaches
  every registered dataset from shared memory (no re-send from the head process); the tasks that
  were in flight on the dead process fail with ``WorkerDied`` (tasks queued for its replacement are
  untouched: reaping goes by process generation).  The pool does not resubmit them, and the island
  search (srhip.search, :multiprocessing) does not either: a worker death ends that search with the
  error, while the pool stays usable for the next call;
* tasks are plain picklable functions ``fn(worker, dataset, *args)`` (module-level, like the
  reference's requirement that user functions be defined on the workers, `move_functions_to_workers`),
  run in submission order per worker; results come back as concurrent.futures.Future objects.

``backend="host"`` runs the same machinery without touching a GPU (the dataset is the mapped numpy
arrays): the CPU tests drive the pool, the residency and the respawn logic with it.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import pickle
import queue
import threading
import traceback
from concurrent.futures import Future
from multiprocessing import shared_memory

import numpy as np


class WorkerDied(RuntimeError):
    pass


class _Shared:
    """One numpy array in a named shared-memory block (the head process owns and unlinks it)."""

    def __init__(self, arr: np.ndarray | None):
        self.name = self.shape = self.dtype = None
        self.shm = None
        if arr is None:
            return
        arr = np.ascontiguousarray(arr)
        self.shm = shared_memory.SharedMemory(create=True, size=max(1, arr.nbytes))
        np.ndarray(arr.shape, arr.dtype, buffer=self.shm.buf)[...] = arr
        self.name, self.shape, self.dtype = self.shm.name, arr.shape, arr.dtype.str

    def spec(self):
        return None if self.name is None else (self.name, self.shape, self.dtype)

    def close(self):
        if self.shm is not None:
            self.shm.close()
            self.shm.unlink()
            self.shm = None


def _attach(spec, keep):
    if spec is None:
        return None
    name, shape, dtype = spec
    # the workers share the head process's resource tracker (spawn passes it on), which already
    # holds this block: attaching re-registers the same name, and the head's unlink releases it
    shm = shared_memory.SharedMemory(name=name)
    keep.append(shm)
    return np.ndarray(shape, np.dtype(dtype), buffer=shm.buf)


class WorkerState:
    """What a task sees: its worker index, device, context (None on the host backend) and the
    resident datasets (key -> DeviceDataset, or the mapped arrays on the host backend)."""

    def __init__(self, index, device, backend):
        self.index, self.device, self.backend = index, device, backend
        self.ctx = None
        self.datasets = {}
        self.arrays = {}
        self.uploads = 0  # datasets uploaded by this worker process (residency accounting)
        self._shm = []

    def attach(self, key, specs):
        X, y, w = (_attach(s, self._shm) for s in specs)
        self.arrays[key] = (X, y, w)
        if self.backend == "srhip":
            from .device import DeviceDataset, get_context

            if self.ctx is None:
                self.ctx = get_context(self.device)
            self.datasets[key] = DeviceDataset(self.ctx, X, y, w)
        else:
            self.datasets[key] = (X, y, w)
        self.uploads += 1


def _worker_main(index, device, backend, inbox, outbox, datasets):
    # a spawned child: nothing GPU-related happened in this process before this point
    state = WorkerState(index, device, backend)
    try:
        for key, specs in datasets:
            state.attach(key, specs)
    except BaseException:
        outbox.put((None, index, False, traceback.format_exc()))
        return
    while True:
        msg = inbox.get()
        if msg is None:
            break
        kind, tid, payload = msg
        try:
            if kind == "attach":
                state.attach(*payload)
                res = None
            else:
                fn, key, args = payload
                res = fn(state, state.datasets[key] if key is not None else None, *args)
            outbox.put((tid, index, True, res))
        except BaseException:
            outbox.put((tid, index, False, traceback.format_exc()))
    for d in state.datasets.values():
        close = getattr(d, "close", None)
        if close:
            close()
    for s in state._shm:
        s.close()


class GPUWorkerPool:
    """``nprocs`` worker processes over ``devices`` (default: every visible GPU; ``[0]`` on the
    host backend).  ``submit(fn, *args, dataset=key, worker=None)`` runs ``fn(worker_state, dataset,
    *args)`` on a worker (round-robin when ``worker`` is None) and returns a Future."""

    def __init__(self, nprocs: int, devices=None, backend: str = "srhip"):
        if backend not in ("srhip", "host"):
            raise ValueError(f"backend {backend!r}")
        if devices is None:
            if backend == "srhip":
                from .device import device_count

                n = device_count()
                if n == 0:
                    raise RuntimeError("no GPU visible to libsrhip (use backend='host' for the host-only pool)")
                devices = list(range(n))
            else:
                devices = [0]
        self.devices = list(devices)
        self.backend = backend
        self.nprocs = int(nprocs)
        self._mp = mp.get_context("spawn")
        self._outbox = self._mp.Queue()
        self._procs = [None] * self.nprocs
        self._inbox = [None] * self.nprocs
        self._shared = {}  # key -> (_Shared X, y, w)
        self._pending = {}  # tid -> (Future, worker, generation of that worker's process)
        self._gen = [0] * self.nprocs  # respawns of each worker slot
        self._lock = threading.Lock()
        self._tids = itertools.count()
        self._keys = itertools.count()
        self._rr = itertools.count()
        self._closed = False
        self.respawns = 0
        for i in range(self.nprocs):
            self._start(i)
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()

    def device_of(self, worker: int) -> int:
        """Worker -> device: worker i on devices[i % ndevices]."""
        return self.devices[worker % len(self.devices)]

    def _start(self, i):
        specs = [(k, tuple(s.spec() for s in sh)) for k, sh in self._shared.items()]
        self._inbox[i] = self._mp.Queue()
        p = self._mp.Process(target=_worker_main, args=(i, self.device_of(i), self.backend, self._inbox[i],
                                                         self._outbox, specs), daemon=True)
        p.start()
        with self._lock:
            self._procs[i] = p
            self._gen[i] += 1

    def _read(self):
        while True:
            try:
                msg = self._outbox.get(timeout=0.2)
            except queue.Empty:
                if self._closed:
                    return
                self._reap()
                continue
            if msg is None:
                return
            tid, worker, ok, res = msg
            with self._lock:
                fut = self._pending.pop(tid, (None, None, None))[0] if tid is not None else None
            if fut is None:
                continue
            if ok:
                fut.set_result(res)
            else:
                fut.set_exception(RuntimeError(f"worker {worker} (device {self.device_of(worker)}):\n{res}"))

    def _reap(self):
        """Fail the tasks of worker processes that died (the slots are respawned on the next submit).
        Under the lock and by generation: a task queued for a slot's NEW process (respawned since the
        old one died) is never failed for the old one's death."""
        with self._lock:
            dead = {(i, self._gen[i]) for i, p in enumerate(self._procs) if p is not None and not p.is_alive()}
            if not dead:
                return
            lost = [tid for tid, (_, w, g) in self._pending.items() if (w, g) in dead]
            futs = [self._pending.pop(tid)[0] for tid in lost]
        for f in futs:
            f.set_exception(WorkerDied("worker process died"))

    def ensure_workers(self) -> int:
        """Respawn dead workers (they re-attach every registered dataset); returns how many."""
        n = 0
        for i, p in enumerate(self._procs):
            if p is None or not p.is_alive():
                self._reap()
                self._start(i)
                n += 1
        self.respawns += n
        return n

    def register_dataset(self, X, y=None, weights=None):
        """Copy the dataset into shared memory once and make it resident on every worker."""
        key = next(self._keys)
        sh = (_Shared(np.asarray(X)), _Shared(None if y is None else np.asarray(y)),
              _Shared(None if weights is None else np.asarray(weights)))
        self._shared[key] = sh
        specs = tuple(s.spec() for s in sh)
        futs = [self._send(i, "attach", (key, specs)) for i in range(self.nprocs)]
        for f in futs:
            f.result()
        return key

    def _send(self, worker, kind, payload):
        pickle.dumps(payload)  # fail here, not silently in the queue's feeder thread
        tid = next(self._tids)
        fut = Future()
        with self._lock:
            self._pending[tid] = (fut, worker, self._gen[worker])
        self._inbox[worker].put((kind, tid, payload))
        return fut

    def submit(self, fn, *args, dataset=None, worker=None) -> Future:
        if self._closed:
            raise RuntimeError("pool is closed")
        self.ensure_workers()
        w = next(self._rr) % self.nprocs if worker is None else int(worker) % self.nprocs
        return self._send(w, "task", (fn, dataset, args))

    def map(self, fn, items, dataset=None):
        """fn(worker, dataset, item) for every item, spread round-robin; results in order."""
        futs = [self.submit(fn, it, dataset=dataset) for it in items]
        return [f.result() for f in futs]

    def close(self):
        if self._closed:
            return
        for i, p in enumerate(self._procs):
            if p is not None and p.is_alive():
                self._inbox[i].put(None)
        for p in self._procs:
            if p is not None:
                p.join(timeout=30)
                if p.is_alive():
                    p.terminate()
                    p.join(timeout=5)
        self._closed = True
        self._reader.join(timeout=5)
        for sh in self._shared.values():
            for s in sh:
                s.close()
        self._shared.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# --- task functions (module level: picklable) ---------------------------------------------------

def task_eval_loss(worker, ds, nodes, offsets, options, loss=None):
    """One population's losses and did_succeed on the worker's device (srhip_eval_loss)."""
    from .device import Program
    from .losses import L2DistLoss

    prog = Program(worker.ctx, nodes, offsets, options, ds.dtype)
    try:
        return prog.eval_loss(ds, loss or L2DistLoss())
    finally:
        prog.close()


def task_column_sums(worker, ds):
    """Host backend: column sums of the resident X (what the worker sees without any re-send)."""
    X = ds[0] if isinstance(ds, tuple) else None
    return None if X is None else X.sum(axis=1)


def task_info(worker, ds, *_):
    """(worker index, device, datasets uploaded by this process): residency accounting."""
    return worker.index, worker.device, worker.uploads
