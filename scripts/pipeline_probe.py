"""Where does a fresh C2 population's time go beside the evaluation?  (bench.py's population_pipeline
item: pipelined_ms_per_population against the interpreter's kernel_ms.)  One MI355X:
  compile     Program() of 1024 fresh trees alone (host compile + program upload)
  eval_first  the first eval_loss of a fresh program (order upload, probe, persistent launch)
  eval_again  the same program's second eval_loss
  close       Program.close() right after an evaluation (device-memory frees)
  pipe_close  the bench's pipelined loop (next population compiled on a thread during the evaluation,
              each program closed after its evaluation)
  pipe_keep   the same loop with the programs kept alive until the end (no frees inside the loop)
Prints one JSON line of medians in ms."""
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402


def main():
    npop = 8
    opts, X, y, _, _, _ = workloads.c2(0, 1024, 1_000_000)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    loss = srhip.L2DistLoss()
    pops = [workloads.c2(5000 + i, 1024, 4096)[4:] for i in range(4 * npop + 3)]
    it = iter(pops)

    def make():
        nd, of = next(it)
        return srhip.Program(ctx, nd, of, opts, np.float32)

    for _ in range(2):  # warm-up
        p = make()
        p.eval_loss(ds, loss)
        p.eval_loss(ds, loss)
        p.close()
    # the GPU reaches its steady clocks over ~50 ms of work: 60 evaluations before anything is timed
    p = make()
    for _ in range(60):
        p.eval_loss(ds, loss)
    steady = []
    for _ in range(10):
        t0 = time.perf_counter()
        p.eval_loss(ds, loss)
        steady.append(time.perf_counter() - t0)
    p.close()
    comp, first, again, close = [], [], [], []
    for _ in range(npop):
        t0 = time.perf_counter()
        p = make()
        t1 = time.perf_counter()
        p.eval_loss(ds, loss)
        t2 = time.perf_counter()
        p.eval_loss(ds, loss)
        t3 = time.perf_counter()
        p.close()
        t4 = time.perf_counter()
        comp.append(t1 - t0)
        first.append(t2 - t1)
        again.append(t3 - t2)
        close.append(t4 - t3)

    def pipe(keep):
        kept = []
        with cf.ThreadPoolExecutor(1) as ex:
            fut = ex.submit(make)
            t0 = time.perf_counter()
            for i in range(npop):
                p = fut.result()
                if i + 1 < npop:
                    fut = ex.submit(make)
                p.eval_loss(ds, loss)
                if keep:
                    kept.append(p)
                else:
                    p.close()
            dt = (time.perf_counter() - t0) / npop
        for p in kept:
            p.close()
        return dt

    pc = pipe(False)
    pk = pipe(True)
    med = lambda v: 1e3 * float(np.median(v))  # noqa: E731
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("SRHIP_")},
                      "eval_steady": med(steady), "compile": med(comp), "eval_first": med(first),
                      "eval_again": med(again), "close": med(close),
                      "pipe_close": 1e3 * pc, "pipe_keep": 1e3 * pk, "kernel_ms_last": ctx.last_kernel_ms()}))


if __name__ == "__main__":
    main()
