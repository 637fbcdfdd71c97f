"""ORACLE — TEST INFRASTRUCTURE ONLY (a study, not a checker).

How far do BASELINE.json's configs move when ONLY the transcendental algorithm changes?  The
device and the default oracle share include/srhip_math.h, so the parity tests cannot see this; here
the oracle evaluates the same trees on the same data twice:

  C2 (Float32, 1024 trees x 1M rows): the default Float32 sin / cos (one degree-5 minimax) against
      Julia's own kernels (srm_jtrigf: FreeBSD __kernel_sindf / __kernel_cosdf per quadrant, Julia's
      rem_pio2_kernel) -- the liboracle_jtrig.so variant.
  C4 (Float64, 512 trees x 100k rows) and a C1-shaped population (Float64, X = randn(2, 100)): the
      header's Float64 exp / log / sin / cos against glibc's (liboracle_glibc64.so) -- a second
      near-correctly-rounded libm standing in for Julia's table-driven exp / log, which are not
      restated here.

Reports, per config: did_succeed masks that differ, the worst relative loss deviation over trees
that succeed in both, and how many trees exceed the config's tolerance (1e-6 Float32, 1e-12
Float64).  Usage: python oracle/libm_sensitivity.py [--out profiles/r05_libm_sensitivity.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import oracle  # noqa: E402


def _run(variant, nodes, offs, opts, X, y, threads):
    oracle.use_variant(variant)
    le, _, ok, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, nthreads=threads)
    oracle.use_variant(None)
    return le, ok


def compare(name, variant, nodes, offs, opts, X, y, tol, threads):
    t0 = time.perf_counter()
    la, oka = _run(None, nodes, offs, opts, X, y, threads)
    lb, okb = _run(variant, nodes, offs, opts, X, y, threads)
    both = oka & okb
    rel = np.zeros(len(la))
    fin = both & np.isfinite(la) & np.isfinite(lb)
    rel[fin] = np.abs(la[fin] - lb[fin]) / np.maximum(np.abs(la[fin]), 1e-300)
    order = np.argsort(-rel)
    worst = [{"tree": int(t), "loss_default": float(la[t]), "loss_variant": float(lb[t]), "rel": float(rel[t])}
             for t in order[:5] if rel[t] > 0]
    return {
        "config": name, "variant": variant, "trees": int(len(la)), "rows": int(X.shape[1]),
        "mask_differs": int(np.sum(oka != okb)), "ok_default": int(oka.sum()), "ok_variant": int(okb.sum()),
        "trees_loss_differs": int(np.sum(rel > 0)), "max_rel_loss_dev": float(rel.max()) if len(rel) else 0.0,
        "median_rel_dev_of_differing": float(np.median(rel[rel > 0])) if np.any(rel > 0) else 0.0,
        "tolerance": tol, "trees_over_tolerance": int(np.sum(rel > tol)), "worst": worst,
        "seconds": time.perf_counter() - t0,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--c2-rows", type=int, default=1_000_000)
    a = ap.parse_args()
    from srhip import workloads
    from srhip.options import Options
    from srhip.random_trees import random_population
    from srhip.node import flatten

    res = []
    opts, X, y, _, nodes, offs = workloads.c2(0, 1024, a.c2_rows)
    res.append(compare("C2 bench population (F32)", "jtrig", nodes, offs, opts, X, y, 1e-6, a.threads))
    opts, _, nodes, offs = workloads.rowshard_population(1024)
    X3, y3 = workloads.c3_shard(0, a.c2_rows)
    res.append(compare("rowshard population over 1M C3-shape rows (F32)", "jtrig", nodes, offs, opts, X3, y3, 1e-6,
                       a.threads))
    opts, X, y, _, nodes, offs = workloads.c4()
    res.append(compare("C4 population (F64)", "glibc64", nodes, offs, opts, X, y, 1e-12, a.threads))
    o1 = Options(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))
    rng = np.random.default_rng(0)
    X1 = rng.standard_normal((2, 100))
    y1 = 2 * np.cos(X1[1]) + X1[0] ** 2 - 2
    trees = random_population(4096, o1, 2, np.float64, seed=11, max_size=30)
    n1, f1 = flatten(trees, o1, np.float64)
    res.append(compare("C1-shaped random population (F64, randn(2, 100))", "glibc64", n1, f1, o1, X1, y1, 1e-12,
                       a.threads))
    for r in res:
        print(json.dumps({k: v for k, v in r.items() if k != "worst"}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
