"""Edge cases at the evaluation boundary: empty populations, empty / one-row inputs, populations that
fail statically, the longest and widest trees, and the stack limit.

The reference evaluates any tree recursively (DynamicExpressions `_eval_tree_array`,
src/InterfaceDynamicExpressions.jl:56-63) on any dataset its constructor accepts
(src/Dataset.jl:98-225).  Here: an empty population is a valid program whose results are empty; a
dataset of zero rows and an empty row subset are errors (srhip_dataset_create / the idx check); a
tree that needs more than K_MAX = 8 interpreter stack slots (a balanced tree of at least 2^10 leaves,
>= 2047 nodes) is rejected with SRHIP_ERR_UNSUPPORTED naming the tree, loudly, never evaluated by a
CPU path.  Everything evaluable is checked against the oracle: did_succeed masks identical, losses
within north_star's 1e-6 (Float32) / 1e-12 (Float64) relative, predictions bit for bit.

The host-only cases (no `gpu` marker) compile through `srhip_program_create` with no context.
"""
import math

import numpy as np
import pytest

F32_REL = 1e-6
F64_REL = 1e-12
K_MAX = 8  # include/srhip_isa.h (csrc/srhip_isa.h K_MAX): stack slots of the largest kernel variant


def _sr():
    import srhip

    return srhip


def _rel(a, b):
    if a == b or (math.isnan(a) and math.isnan(b)):
        return 0.0
    return abs(a - b) / max(abs(b), 1e-300)


def _balanced(sr, depth, nfeat, k=1):
    """A perfect binary tree of `depth` levels of + and * (cos between levels) over feature leaves:
    Strahler number depth + 1; with leaf operands read in place the interpreter needs depth - 1
    stack slots."""
    if depth == 0:
        return sr.Node(f"x{1 + k % nfeat}")
    l, r = _balanced(sr, depth - 1, nfeat, 2 * k), _balanced(sr, depth - 1, nfeat, 2 * k + 1)
    if depth == 1:  # (no unary operator on a leaf: a derived column would be a leaf operand)
        return l + r
    return sr.cos(l) + r if depth % 2 else l * sr.cos(r)


def _chains(sr, nfeat, length, seed):
    """Long left- and right-deep chains over many features (bounded values: cos between products)."""
    rng = np.random.default_rng(seed)
    feats = rng.integers(1, nfeat + 1, size=length)
    left = sr.Node(f"x{feats[0]}")
    for i, f in enumerate(feats[1:]):
        x = sr.Node(f"x{f}")
        op = i % 4
        left = left + x if op == 0 else (left - x if op == 1 else (sr.cos(left) * x if op == 2 else sr.cos(left)))
    right = sr.Node(f"x{feats[-1]}")
    for i, f in enumerate(feats[-2::-1]):
        x = sr.Node(f"x{f}")
        op = i % 3
        right = x - right if op == 0 else (x + sr.cos(right) if op == 1 else x * sr.cos(right))
    return [left, right]


# ---- host-only (no device) ------------------------------------------------------------------------
def test_empty_population_compiles():
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos",))
    for dt in (np.float32, np.float64, np.int32):
        nodes, offs = sr.flatten([], opts, dt)
        assert len(nodes) == 0 and list(offs) == [0]
        prog = sr.Program(None, nodes, offs, opts, dt)
        assert prog.ntrees == 0
        assert prog.stats()["total_nodes"] == 0


def test_stack_limit_is_loud():
    """A tree at K_MAX stack slots compiles; one past it fails with SRHIP_ERR_UNSUPPORTED naming the
    slots it needs -- the whole program, never a silent partial result."""
    sr = _sr()
    from srhip._lib import ERR_UNSUPPORTED, SrhipError

    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos",))
    ok_tree = _balanced(sr, K_MAX + 1, 3)
    nodes, offs = sr.flatten([ok_tree], opts, np.float32)
    prog = sr.Program(None, nodes, offs, opts, np.float32)
    assert prog.stats()["max_stack"] == K_MAX
    big = _balanced(sr, K_MAX + 2, 3)
    nodes, offs = sr.flatten([sr.Node("x1"), big], opts, np.float32)
    with pytest.raises(SrhipError) as e:
        sr.Program(None, nodes, offs, opts, np.float32)
    assert e.value.code == ERR_UNSUPPORTED and "stack slots" in str(e.value)


def test_long_chains_compile():
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("cos",))
    trees = _chains(sr, 300, 1500, seed=3)
    nodes, offs = sr.flatten(trees, opts, np.float64)
    prog = sr.Program(None, nodes, offs, opts, np.float64)
    assert prog.stats()["total_nodes"] == len(nodes)
    assert prog.stats()["max_stack"] <= 2  # chains need no stack beyond the accumulator's partner


# ---- on the device ----------------------------------------------------------------------------------
@pytest.mark.gpu
def test_empty_population_evaluates_to_empty(ctx):
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos",))
    X = np.random.default_rng(0).standard_normal((2, 100)).astype(np.float32)
    y = X[0].copy()
    ds = sr.DeviceDataset(ctx, X, y)
    nodes, offs = sr.flatten([], opts, np.float32)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    loss, ok = prog.eval_loss(ds, sr.L2DistLoss())
    assert loss.shape == (0,) and ok.shape == (0,)
    pred, ok = prog.eval_predict(sr.DeviceDataset(ctx, X))
    assert pred.shape == (0, 100) and ok.shape == (0,)


@pytest.mark.gpu
def test_zero_rows_and_empty_subset_fail_loudly(ctx):
    sr = _sr()
    from srhip._lib import ERR_INVALID, SrhipError

    with pytest.raises(SrhipError) as e:
        sr.DeviceDataset(ctx, np.zeros((2, 0), dtype=np.float32), np.zeros(0, dtype=np.float32))
    assert e.value.code == ERR_INVALID
    opts = sr.Options(binary_operators=("+",), unary_operators=("cos",))
    X = np.ones((2, 10), dtype=np.float32)
    ds = sr.DeviceDataset(ctx, X, X[0].copy())
    nodes, offs = sr.flatten([sr.Node("x1") + sr.Node("x2")], opts, np.float32)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    with pytest.raises(SrhipError) as e:
        prog.eval_loss(ds, sr.L2DistLoss(), idx=np.zeros(0, dtype=np.int64))
    assert e.value.code == ERR_INVALID
    # the context stays usable after the errors
    loss, ok = prog.eval_loss(ds, sr.L2DistLoss())
    assert ok[0] and loss[0] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_one_row_dataset_and_repeated_subset(ctx, oracle, dtype):
    """n = 1, and batching's sample-with-replacement subset (src/LossFunctions.jl:125-127) that picks
    the same row batch_size times: the loss of the gathered rows, as the oracle computes it on them."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    trees = sr.random_population(48, opts, 3, dtype, 41, 20)
    nodes, offs = sr.flatten(trees, opts, dtype)
    rng = np.random.default_rng(42)
    X = rng.standard_normal((3, 1)).astype(dtype)
    y = rng.standard_normal(1).astype(dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    tol = F32_REL if dtype == np.float32 else F64_REL
    ds = sr.DeviceDataset(ctx, X, y)
    for idx in (None, np.zeros(50, dtype=np.int64)):
        dl, dok = prog.eval_loss(ds, sr.L2DistLoss(), idx=idx)
        Xs, ys = (X, y) if idx is None else (X[:, idx], y[idx])
        ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, Xs, ys, None, 0, 0.0)
        assert np.array_equal(dok, ook)
        assert not [t for t in np.nonzero(ook)[0] if _rel(dl[t], ol[t]) > tol]
        assert np.all(np.isinf(dl[~dok]))


@pytest.mark.gpu
def test_population_that_fails_statically(ctx, oracle):
    """Every tree fails before any row is evaluated (a non-finite constant leaf, a constant subtree
    that overflows): no launch runs, every tree is not ok with loss L(Inf), as in the oracle."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*", "/"), unary_operators=("cos", "exp"))
    x1 = sr.Node("x1")
    trees = [x1 * sr.Node(val=float("inf")), x1 + sr.exp(sr.exp(sr.Node(val=100.0))),
             sr.cos(x1) + sr.Node(val=float("nan")), sr.Node(val=3e38) * sr.Node(val=10.0) + x1]
    X = np.random.default_rng(1).standard_normal((1, 5000)).astype(np.float32)
    y = X[0].copy()
    nodes, offs = sr.flatten(trees, opts, np.float32)
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    dl, dok = prog.eval_loss(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    _, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert not ook.any() and not dok.any()
    assert np.all(np.isinf(dl))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_longest_and_widest_trees(ctx, oracle, dtype):
    """1500-node chains over 300 features (the staged row block does not fit LDS: the launch reads
    X from global memory) and the deepest balanced tree the stack holds (1278 nodes, K_MAX slots),
    beside a C2-shaped population in the same program: losses and predictions against the oracle."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("cos",))
    nfeat, n = 300, 3000
    trees = _chains(sr, nfeat, 1500, seed=7) + [_balanced(sr, K_MAX + 1, nfeat)]
    trees += sr.random_population(32, opts, nfeat, dtype, 8, 30)
    nodes, offs = sr.flatten(trees, opts, dtype)
    rng = np.random.default_rng(9)
    X = rng.standard_normal((nfeat, n)).astype(dtype)
    y = rng.standard_normal(n).astype(dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    assert prog.stats()["max_stack"] == K_MAX
    dl, dok = prog.eval_loss(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook)
    assert dok[:3].all()
    tol = F32_REL if dtype == np.float32 else F64_REL
    assert not [(t, dl[t], ol[t]) for t in np.nonzero(ook)[0] if _rel(dl[t], ol[t]) > tol]
    pred, pok = prog.eval_predict(sr.DeviceDataset(ctx, X))
    it = np.uint32 if dtype == np.float32 else np.uint64
    for t in range(len(trees)):
        ref, rok = oracle.eval_tree(nodes[offs[t]:offs[t + 1]], opts.binop_codes, opts.unaop_codes, X)
        assert bool(pok[t]) == rok, t
        if rok:
            assert np.array_equal(pred[t].view(it), ref.view(it)), t
