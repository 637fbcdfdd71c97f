"""Trees whose did_succeed needs the exact precise pass (status 2 of srhip_partials_finalize) for the
C2 population (1M rows) and the row-shard population (10M rows, one rank), and one eval_loss's time:
python scripts/undecided_count.py [c2|rowshard]  (A/B of the decision's bounds across builds: SRHIP_LIB)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "rowshard"
if which == "c2":
    opts, X, y, trees, nodes, offs = workloads.c2()
else:
    X, y = workloads.c3_shard(0, 10_000_000)
    opts, trees, nodes, offs = workloads.rowshard_population(1024)
ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
loss = srhip.L2DistLoss()
psums, pchk = prog.eval_loss_partials(ds, loss)
st = prog.finalize(X.shape[0], psums, pchk)[2]
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    _, ok = prog.eval_loss(ds, loss)
    ts.append(time.perf_counter() - t0)
if len(sys.argv) > 2:  # status, check statistics and the per-tree partial sums for offline comparison
    np.savez(sys.argv[2], st=st, chk=np.asarray(pchk, np.float64))
print(f"{which}: undecided {int(np.sum(st == 2))} of {len(st)}, failed {int(np.sum(st == 1))}, "
      f"eval_loss {1e3 * min(ts):.3f} ms (kernel {ctx.last_kernel_ms():.3f}), ok {int(ok.sum())}", flush=True)
