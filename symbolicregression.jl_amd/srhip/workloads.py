"""The synthetic inputs of BASELINE.json's configs, in one place so that
bench.py and the full-size parity tests (tests/test_gpu_configs.py) evaluate the SAME trees on the
SAME data.  Every generator is seeded; nothing here touches the device.

  C2  eval-only: 1024 random trees (size U{1..30}, + - * / cos exp) x 1M rows x 5 features F32
  C3  search data: 10 features x 10M rows F32 (+ the 64-tree population its CPU baseline scores)
  C4  constant optimisation: 512 fixed-size-20 F64 trees with >= 2 constants x 100k rows x 5
  C5  Int32 evaluation (test_integer_evaluation.jl shape) / custom objective
      (test_custom_objectives.jl: X = rand(2, 100) * 10, y = x1 + x2, F64)
"""
from __future__ import annotations

import numpy as np

from .node import count_constants, flatten
from .options import Options
from .random_trees import gen_random_tree_fixed_size, random_population

C2_OPS = dict(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))


def c2(rank: int = 0, ntrees: int = 1024, rows: int = 1_000_000, binops=None, unaops=None):
    """(options, X[5, rows] f32, y[rows] f32, trees, nodes, offsets) of rank `rank`'s C2 island:
    X ~ N(0,1) (seed 0 + 1000 rank), y = 2cos(x4) + x1^2 - 2 + 0.1 N(0,1) (seed 1 + 1000 rank),
    trees from random_population(seed 2 + 1000 rank)."""
    opts = Options(binary_operators=tuple(binops or C2_OPS["binary_operators"]),
                   unary_operators=tuple(C2_OPS["unary_operators"] if unaops is None else unaops))
    nfeat = 5
    rng = np.random.default_rng(0 + 1000 * rank)
    X = rng.standard_normal((nfeat, rows)).astype(np.float32)
    rng_y = np.random.default_rng(1 + 1000 * rank)
    y = (2 * np.cos(X[3].astype(np.float64)) + X[0].astype(np.float64) ** 2 - 2
         + 0.1 * rng_y.standard_normal(rows)).astype(np.float32)
    trees = random_population(ntrees, opts, nfeat, np.float32, seed=2 + 1000 * rank, max_size=30)
    nodes, offs = flatten(trees, opts, np.float32)
    return opts, X, y, trees, nodes, offs


C3_OPS = dict(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))


def c3_data(rows: int = 10_000_000):
    """C3's dataset (replicated on every rank): X ~ N(0,1) 10 x rows F32 (seed 0),
    y = 2cos(x4) + x1^2 - 2 + 0.5 x7 x3 - exp(x10 / 4)."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((10, rows)).astype(np.float32)
    y = np.empty(rows, dtype=np.float32)
    step = 1 << 20
    for a in range(0, rows, step):  # in slices: no 10 x rows float64 temporary
        Xd = X[:, a:a + step].astype(np.float64)
        y[a:a + step] = 2 * np.cos(Xd[3]) + Xd[0] ** 2 - 2 + 0.5 * Xd[6] * Xd[2] - np.exp(Xd[9] / 4)
    return X, y


def c3_shard(lo: int, hi: int, nfeat: int = 10):
    """Rows [lo, hi) of the row-sharded C3-shape dataset (bench.py --mode rowshard): generated in
    fixed 2^20-row chunks, chunk c from seed 100 + c, so a shard's rows do not depend on how many
    ranks share the dataset.  X ~ N(0,1) nfeat x rows F32, y as c3_data's formula."""
    step = 1 << 20
    X = np.empty((nfeat, hi - lo), dtype=np.float32)
    for c in range(lo // step, (hi + step - 1) // step):
        a, b = c * step, (c + 1) * step
        Xc = np.random.default_rng(100 + c).standard_normal((nfeat, step)).astype(np.float32)
        s0, s1 = max(a, lo), min(b, hi)
        X[:, s0 - lo:s1 - lo] = Xc[:, s0 - a:s1 - a]
    y = np.empty(hi - lo, dtype=np.float32)
    for a in range(0, hi - lo, step):
        Xd = X[:, a:a + step].astype(np.float64)
        y[a:a + step] = 2 * np.cos(Xd[3]) + Xd[0] ** 2 - 2 + 0.5 * Xd[6] * Xd[2] - np.exp(Xd[9] / 4)
    return X, y


def rowshard_population(ntrees: int = 1024, nfeat: int = 10):
    """bench.py --mode rowshard's population: random trees (size U{1..30}, C3's operators) over
    nfeat features, seed 7."""
    opts = Options(**C3_OPS)
    trees = random_population(ntrees, opts, nfeat, np.float32, seed=7, max_size=30)
    nodes, offs = flatten(trees, opts, np.float32)
    return opts, trees, nodes, offs


def c3_population(opts=None, ntrees: int = 64):
    """The 64-tree population (size <= 20, the search's default maxsize) C3's CPU baseline scores."""
    opts = opts or Options(**C3_OPS)
    trees = random_population(ntrees, opts, 10, np.float32, seed=6, max_size=20)
    nodes, offs = flatten(trees, opts, np.float32)
    return opts, trees, nodes, offs


C4_OPS = dict(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))


def c4(ntrees: int = 512, rows: int = 100_000):
    """(options, X[5, rows] f64, y, trees, nodes, offsets): fixed-size-20 trees with >= 2 constants
    (benchmark/benchmarks.jl:96-114's shape), X ~ N(0,1), y = 2cos(x4) + x1^2 - 2 + 0.1 N(0,1); one
    generator (seed 4) draws the trees first, then X and the noise."""
    opts = Options(**C4_OPS)
    rng = np.random.default_rng(4)
    trees = []
    while len(trees) < ntrees:
        t = gen_random_tree_fixed_size(20, opts, 5, np.float64, rng)
        if count_constants(t) >= 2:
            trees.append(t)
    nodes, offs = flatten(trees, opts, np.float64)
    X = rng.standard_normal((5, rows))
    y = 2 * np.cos(X[3]) + X[0] ** 2 - 2 + 0.1 * rng.standard_normal(rows)
    return opts, X, y, trees, nodes, offs


def c5_custom_objective_data(seed: int = 0, n: int = 100):
    """test/test_custom_objectives.jl:39-40: X = rand(2, 100) .* 10, y = x1 + x2 (Float64)."""
    rng = np.random.default_rng(seed)
    X = rng.random((2, n)) * 10
    return X, X[0] + X[1]
