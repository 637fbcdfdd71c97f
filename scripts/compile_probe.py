"""Fresh-population compile on the GPU box: where does a pipelined compile lose time?
Prints one JSON line: the job's CPU allotment (affinity, cgroup quota), compile of 1024 fresh C2 trees
on the main thread / on a worker thread (device idle), the same with an evaluation loop running on
another context, and the evaluation's wall time alone / beside a compile loop."""
import concurrent.futures as cf
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402


def cpu_info():
    q = None
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            q = open(f).read().strip()
            break
        except OSError:
            pass
    return {"affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "quota": q}


def main():
    opts, X, y, _, _, _ = workloads.c2(0, 1024, 1_000_000)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    loss = srhip.L2DistLoss()
    pops = [workloads.c2(9000 + i, 1024, 4096)[4:] for i in range(52)]
    it = iter(pops)
    med = lambda v: 1e3 * float(np.median(v))  # noqa: E731

    def compile_one(c):
        nd, of = next(it)
        t0 = time.perf_counter()
        p = srhip.Program(c, nd, of, opts, np.float32)
        dt = time.perf_counter() - t0
        return p, dt

    p0, _ = compile_one(ctx)
    for _ in range(40):
        p0.eval_loss(ds, loss)  # steady clocks
    main_c = []
    for _ in range(6):
        p, dt = compile_one(ctx)
        main_c.append(dt)
        p.close()
    with cf.ThreadPoolExecutor(1) as ex:
        worker_c = [ex.submit(lambda: compile_one(ctx)).result() for _ in range(6)]
        for p, _ in worker_c:
            p.close()
        worker_c = [dt for _, dt in worker_c]
    ev_alone = []
    for _ in range(10):
        t0 = time.perf_counter()
        p0.eval_loss(ds, loss)
        ev_alone.append(time.perf_counter() - t0)
    # an evaluation loop on the main thread while a worker compiles
    stop = threading.Event()
    ev_busy = []

    def evals():
        while not stop.is_set():
            t0 = time.perf_counter()
            p0.eval_loss(ds, loss)
            ev_busy.append(time.perf_counter() - t0)

    th = threading.Thread(target=evals)
    th.start()
    time.sleep(0.02)
    ctx2 = srhip.Context(0)
    conc_c = []
    for _ in range(8):
        p, dt = compile_one(ctx2)
        conc_c.append(dt)
        p.close()
    stop.set()
    th.join()
    ctx2.close()
    # the bench's single-context pipeline, phase by phase: next population compiled on a worker thread
    # while this one evaluates on the same context
    ph = {"eval": [], "close": [], "wait": [], "iter": []}
    with cf.ThreadPoolExecutor(1) as ex:
        fut = ex.submit(lambda: compile_one(ctx))
        p, _ = fut.result()
        for i in range(10):
            t0 = time.perf_counter()
            fut = ex.submit(lambda: compile_one(ctx))
            p.eval_loss(ds, loss)
            t1 = time.perf_counter()
            p.close()
            t2 = time.perf_counter()
            p, cdt = fut.result()
            t3 = time.perf_counter()
            ph["eval"].append(t1 - t0)
            ph["close"].append(t2 - t1)
            ph["wait"].append(t3 - t2)
            ph["iter"].append(t3 - t0)
        p.close()
    pipe1 = {k: med(v) for k, v in ph.items()}
    print(json.dumps({"pipe1": pipe1, "cpu": cpu_info(), "compile_main_ms": med(main_c), "compile_worker_ms": med(worker_c),
                      "compile_beside_evals_ms": med(conc_c), "eval_alone_ms": med(ev_alone),
                      "eval_beside_compiles_ms": med(ev_busy), "evals_beside": len(ev_busy)}))


if __name__ == "__main__":
    main()
