"""Launch shape against population size on C3's dataset (10 features x 10M rows F32): the search's
coalesced launches carry a few trees each (C3: 2.4 on average), where the C2 population carries 1024.
For nl trees: median wall per srhip_eval_loss and the interpreter's kernel time, with the default
launch choice and with SRHIP_NO_PERSISTENT=1 (the grid launch); losses must be bitwise equal.

  python scripts/small_batch_sweep.py [--rows N] [--reps K] > out.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "symbolicregression.jl_amd")]

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--sizes", default="1,2,3,4,6,8,12,16,32,64,128,256")
    ap.add_argument("--envs", default="default,SRHIP_NO_PERSISTENT=1")
    args = ap.parse_args()
    X, y = workloads.c3_data(args.rows)
    opts, trees, nodes, offs = workloads.c3_population(ntrees=256)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    loss = srhip.L2DistLoss()
    for nl in [int(s) for s in args.sizes.split(",")]:
        sub_nodes = nodes[:offs[nl]]
        prog = srhip.Program(ctx, sub_nodes, offs[:nl + 1], opts, np.float32)
        ref = None
        for env in args.envs.split(","):
            kv = None if env == "default" else env.split("=", 1)
            if kv:
                os.environ[kv[0]] = kv[1]
            try:
                for _ in range(3):
                    prog.eval_loss(ds, loss)
                walls, kms = [], []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    l, ok = prog.eval_loss(ds, loss)
                    walls.append(time.perf_counter() - t0)
                    kms.append(ctx.last_kernel_ms())
            finally:
                if kv:
                    del os.environ[kv[0]]
            same = None
            if ref is None:
                ref = (l.copy(), ok.copy())
            else:
                same = bool(np.array_equal(ref[0].view(np.uint64), l.view(np.uint64)) and np.array_equal(ref[1], ok))
            print(json.dumps({"ntrees": nl, "env": env, "wall_us": 1e6 * float(np.median(walls)),
                              "kernel_us": 1e3 * float(np.median(kms)), "same_bits": same}), flush=True)


if __name__ == "__main__":
    main()
