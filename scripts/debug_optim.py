"""Diagnostic (GPU box): the device optimiser's trajectory for one tree (SRHIP_OPTIM_TRACE) beside
the oracle's objective calls for the same tree (oracle/optim.py), single start."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import optim  # noqa: E402
import srhip  # noqa: E402


def newton_case():
    opts = srhip.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp", "sin"))
    rng = np.random.default_rng(21)
    trees = []
    while len(trees) < 24:
        t = srhip.gen_random_tree_fixed_size(int(rng.integers(3, 12)), opts, 3, np.float64, rng)
        if srhip.count_constants(t) == 1:
            trees.append(t)
    X = rng.standard_normal((3, 2000))
    y = np.cos(1.3 * X[0]) * 2.0 + X[1] * 0.7 - 0.3
    return opts, trees, X, y


def bfgs_case():
    opts = srhip.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp", "sin"))
    trees = srhip.random_population(32, opts, 3, np.float64, seed=5, max_size=14)
    rng = np.random.default_rng(6)
    X = rng.standard_normal((3, 1500))
    y = np.cos(1.3 * X[0]) * 2.0 + X[1] * 0.7 - 0.3
    return opts, trees, X, y


def run(case, t):
    opts, trees, X, y = case()
    nodes, offs = srhip.flatten([trees[t]], opts, np.float64)
    print("tree", t, srhip.string_tree(trees[t], opts), flush=True)
    ctx = srhip.get_context(0)
    os.environ["SRHIP_OPTIM_TRACE"] = "0"
    prog = srhip.Program(ctx, nodes, offs, opts, np.float64)
    out, imp, fc = prog.optimize_constants(srhip.DeviceDataset(ctx, X, y), srhip.L2DistLoss(), nrestarts=0, seed=3)
    sys.stderr.flush()
    print("device", out, imp, fc, prog.get_constants(), flush=True)
    f0, order = optim._loss_fn(nodes, opts.binop_codes, opts.unaop_codes, X, y)

    def f(c):
        v = f0(c)
        print(f"  oracle f({list(c)}) = {v!r}", flush=True)
        return v

    x0 = np.array([nodes[i]["val"] for i in order])
    algo = optim.newton if len(x0) == 1 else optim.bfgs
    print("oracle", algo(f, x0, 8), flush=True)


if __name__ == "__main__":
    which = sys.argv[1]
    run(newton_case if which == "newton" else bfgs_case, int(sys.argv[2]))
