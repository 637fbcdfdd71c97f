"""Per-operator cost of the Float32 interpreter (C2's kernel variant): populations of 1024 trees of
one shape each (8 operators of one kind, or a feature leaf as the baseline) over C2's 1M x 5
dataset.  Run plain it prints the kernel time per shape; under rocprofv3 --pmc the eval_kernel
dispatches of each eval (between two reduce_kernel dispatches) are attributed to the shape in
gpurun_out/op_costs_order.json, and scripts/op_costs_pmc.py turns them into counters per
operator-node-row.  python scripts/op_costs.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import workloads  # noqa: E402
from srhip.node import Node  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
opts, X, y, _, _, _ = workloads.c2(0, 16, 1_000_000)
B = {o: opts.binary_index(o) for o in ("+", "-", "*", "/")}
U = {o: opts.unary_index(o) for o in ("cos", "exp")}
rng = np.random.default_rng(7)


def f(i):
    return Node(f"x{i % 5 + 1}")


def c(lo=0.5, hi=1.5):
    return Node(val=float(rng.uniform(lo, hi)))


def chain(op, right, n=8):
    t = f(0)
    for i in range(n):
        t = Node(B[op], t, right(i + 1))
    return t


SHAPES = {
    "leaf": lambda: f(0),
    "addf8": lambda: chain("+", f),
    "addc8": lambda: chain("+", lambda i: c()),
    "mulf8": lambda: chain("*", f),
    "subf8": lambda: chain("-", f),
    "divf8": lambda: chain("/", lambda i: Node(B["+"], f(i), c(2.0, 3.0))) ,  # 8 div + 8 add
    "addfc8": lambda: chain("+", lambda i: Node(B["+"], f(i), c(2.0, 3.0))),  # 16 add (divf8's baseline)
    "divc8": lambda: chain("/", lambda i: c(0.9, 1.1)),
    "cos8": lambda: _un("cos", 8),
    "expm8": lambda: _expm(8),
    "mulc8": lambda: chain("*", lambda i: c(0.05, 0.15)),
    "push4": lambda: Node(B["+"], Node(B["+"], Node(B["*"], f(0), f(1)), Node(B["*"], f(2), f(3))),
                          Node(B["+"], Node(B["*"], f(4), f(0)), Node(B["*"], f(1), f(2)))),
    "mulf4": lambda: chain("*", f, 4),
    # round 6: Julia's Float32 cos by argument tier (cos8 above is tier B: cos of a feature, then of
    # values in [-1, 1]); each cos takes A * c, so subtract mulc8's per-node cost for the cos alone
    "cosA8": lambda: _cosm(8, 0.05, 0.15),      # |arg| < pi/4
    "cosC8": lambda: _cosm(8, 40.0, 60.0),      # 9pi/4 < |arg| < 2^28 pi/2 (Cody-Waite)
    "cosS8": lambda: _cosm(8, 0.9e9, 1.1e9),    # Payne-Hanek rows
}


def _un(op, n):
    t = f(0)
    for _ in range(n):
        t = Node(U[op], t)
    return t


def _cosm(n, lo, hi):  # cos(A * c) repeated: n cos + n mul-by-constant
    t = f(0)
    for _ in range(n):
        t = Node(U["cos"], Node(B["*"], t, c(lo, hi)))
    return t


def _expm(n):  # exp(A * c) repeated: n exp + n mul-by-constant
    t = f(0)
    for _ in range(n):
        t = Node(U["exp"], Node(B["*"], t, c(0.05, 0.15)))
    return t


ctx = srhip.get_context(0)
ds = srhip.DeviceDataset(ctx, X, y)
loss = srhip.L2DistLoss()
order = []
res = {}
for name, make in SHAPES.items():
    trees = [make() for _ in range(1024)]
    nodes, offs = srhip.flatten(trees, opts, np.float32)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    st = prog.stats()
    kms = []
    for _ in range(reps):
        _, ok = prog.eval_loss(ds, loss)
        kms.append(ctx.last_kernel_ms())
        order.append(name)
    w = ctx.last_work()
    res[name] = {"kernel_ms": min(kms), "opnodes": st["total_opnodes"], "nodes": st["total_nodes"],
                 "ok": int(np.sum(ok)), "node_rows": w["node_rows"]}
    print(json.dumps({name: res[name]}), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "op_costs_order.json"), "w") as fh:
    json.dump({"order": order, "shapes": res}, fh)
