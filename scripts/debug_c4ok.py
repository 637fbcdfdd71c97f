"""Diagnostic (GPU box): C4 trees where the gradient kernel's did_succeed differs from eval_loss's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import srhip  # noqa: E402
from srhip import workloads  # noqa: E402

opts, X, y, trees, nodes, offs = workloads.c4()
ctx = srhip.get_context(0)
prog = srhip.Program(ctx, nodes, offs, opts, np.float64)
ds = srhip.DeviceDataset(ctx, X, y)
dl, dok = prog.eval_loss(ds, srhip.L2DistLoss())
gl, g, gok = prog.eval_loss_grad(ds, srhip.L2DistLoss())
ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y)
bad = np.nonzero(dok != gok)[0]
print("differ:", len(bad), "of", len(dok))
for t in bad[:20]:
    print(t, "eval", dok[t], dl[t], "grad", gok[t], gl[t], "oracle", ook[t], ol[t], srhip.string_tree(trees[t], opts))
