"""Where do C2's cos arguments fall?  For every cos node of the C2 bench population whose argument is
an operator output (cos of a feature is a derived column, computed once per row block), evaluate the
argument subtree over the 1M rows (oracle, host) and classify each 1024-row wave tile by its max |x|:
  A: all |x| < Float32(pi)/4 (no reduction: one kernel)
  B: all |x| <= 9pi/4 (Julia's +-k pi/2 cases: one-product reduction, both kernels)
  C: all |x| < 2^28 pi/2 (Cody-Waite)
  D: larger / non-finite.
Prints tile counts per tier (the device's per-wave path choice for Julia's Float32 trig).
python scripts/trig_arg_tiers.py [rows per tile, default 1000; 64: the round-6 per-slice study]"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "symbolicregression.jl_amd")]
import oracle
from srhip import workloads
from srhip.node import flatten

TILE = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
opts, X, y, trees, nodes, offs = workloads.c2(0, 1024, 1_000_000)
cos_idx = [i + 1 for i, u in enumerate(opts.unary_operators) if u == "cos"][0]
args = []
def walk(n):
    if n.degree == 1:
        op = n.op if isinstance(n.op, int) else opts.unary_operators.index(n.op) + 1
        if op == cos_idx and n.l.degree > 0:
            args.append(n.l)
        walk(n.l)
    elif n.degree == 2:
        walk(n.l); walk(n.r)
for t in trees:
    walk(t)
tiers = np.zeros(4, dtype=np.int64)
for a in args:
    nd, of = flatten([a], opts, np.float32)
    out, ok = oracle.eval_tree(nd, opts.binop_codes, opts.unaop_codes, X)
    m = np.abs(out).reshape(-1, TILE)  # (1M rows: 1000-row tiles, ~ the device's 1024)
    mx = np.max(np.where(np.isnan(m), np.inf, m), axis=1)
    tiers[0] += np.sum(mx < np.float32(np.pi) / 4)
    tiers[1] += np.sum((mx >= np.float32(np.pi) / 4) & (mx <= np.pi * 9 / 4))
    tiers[2] += np.sum((mx > np.pi * 9 / 4) & (mx < 421657440.0))
    tiers[3] += np.sum(~(mx < 421657440.0))
print("rows per tile:", TILE, "cos-of-operator nodes:", len(args), "tiles per tier A/B/C/D:", tiers.tolist(),
      "fractions:", np.round(tiers / tiers.sum(), 3).tolist())
