"""Round-trip latency of one small evaluation (C1's regime: one tree x 100 rows F64):
srhip_eval_loss on a persistent program, a fresh program per call, and the coalescer's single-client
path.  python scripts/latency_bench.py [reps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import numpy as np  # noqa: E402

import srhip  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
opts = srhip.Options(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))
rng = np.random.default_rng(0)
X = rng.standard_normal((2, 100))
y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
trees = srhip.random_population(64, opts, 2, np.float64, seed=1, max_size=20)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
loss = srhip.L2DistLoss()
nodes, offs = srhip.flatten(trees[:1], opts, np.float64)
prog = srhip.Program(ctx, nodes, offs, opts, np.float64)


def timeit(fn, n):
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


print(f"persistent program eval_loss: {timeit(lambda: prog.eval_loss(ds, loss), reps):.1f} us")


def fresh():
    p = srhip.Program(ctx, nodes, offs, opts, np.float64)
    p.eval_loss(ds, loss)
    p.close()


print(f"fresh program per call:       {timeit(fresh, reps):.1f} us")
co = srhip.Coalescer(ctx, ds, opts, loss)
one = srhip.flatten(trees[:1], opts, np.float64)[0]
print(f"coalescer score_loss:         {timeit(lambda: co.score_loss(one), reps):.1f} us")
print(f"coalescer stats: {co.stats()}")
co.close()
