"""C4's dual-number gradient launch alone (all 512 trees' loss + d loss / d c over 100k F64 rows),
for kernel A/B and PMC passes: python scripts/grad_bench.py [reps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
opts, X, y, trees, nodes, offs = workloads.c4()
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
prog = srhip.Program(ctx, nodes, offs, opts, np.float64)
loss = srhip.L2DistLoss()
for _ in range(3):
    prog.eval_loss_grad(ds, loss)
ctx.synchronize()
ks = []
t0 = time.perf_counter()
for _ in range(reps):
    f, g, ok = prog.eval_loss_grad(ds, loss)
    ks.append(ctx.last_kernel_ms())
dt = (time.perf_counter() - t0) / reps
print(f"grad launch {dt * 1e3:.3f} ms, kernel {np.mean(ks):.3f} ms (min {np.min(ks):.3f}); ok {int(ok.sum())}; "
      f"checksum {float(np.nansum(np.where(np.isfinite(f), f, 0))):.17g}")
