"""Every BASELINE.json config at its full size, device vs oracle.

The workloads come from srhip.workloads, the module bench.py measures, so each test evaluates
exactly the trees and data of its config:
  C2  the bench's 1024-tree population x 1M rows x 5 features F32 (every tree, not a subset)
  C3  the 10 features x 10M rows F32 dataset with the 64-tree population its CPU baseline scores
  C4  the 512 fixed-size-20 F64 trees x 100k rows: losses, the dual-number gradient against oracle
      central differences, and the batched optimiser's outcome against oracle/optim.py
  C5  random Int32 trees over 1M rows (bit-exact) and test_custom_objectives.jl's user loss_function
Tolerances (north_star): identical did_succeed masks; losses 1e-6 relative (F32) / 1e-12 (F64)
against the oracle's exact-sum loss; Int32 bit-exact.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F32_REL = 1e-6
F64_REL = 1e-12


def _sr():
    import srhip

    return srhip


def _rel(a, b):
    if a == b:
        return 0.0
    return abs(a - b) / max(abs(b), 1e-300)


def _check_losses(dl, dok, ol, ook, tol):
    assert np.array_equal(dok, ook), np.nonzero(dok != ook)[0][:10]
    bad = [(int(t), dl[t], ol[t]) for t in np.nonzero(ook)[0] if not _rel(dl[t], ol[t]) <= tol]
    assert not bad, bad[:8]
    assert np.all(np.isinf(dl[~dok]))


def test_c2_bench_population_matches_oracle(ctx, oracle):
    """C2 exactly as bench.py runs it: the 1024-tree population (seed 2) over 5 x 1M F32."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, trees, nodes, offs = workloads.c2()
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    assert prog.stats()["total_nodes"] == 15952  # the bench line's nodes_per_step
    dl, dok = prog.eval_loss(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    _check_losses(dl, dok, ol, ook, F32_REL)
    assert int(dok.sum()) == 808  # the bench line's trees_ok


def test_c2_full_size_predictions_bitwise(ctx, oracle):
    """A1 at C2's full size: all 1024 bench trees x 1M rows through srhip_eval_predict
    (eval_tree_array: the path MMI.predict and user loss_functions consume) -- did_succeed equal to the
    oracle's and every prediction of every succeeding tree equal to the oracle's bit for bit.  Four
    programs of 256 trees keep the host copies at 1 GB each."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, trees, nodes, offs = workloads.c2()
    ds = sr.DeviceDataset(ctx, X)
    nt = len(offs) - 1
    nok = 0
    for lo in range(0, nt, 256):
        hi = min(nt, lo + 256)
        sub = nodes[offs[lo]:offs[hi]]
        soffs = offs[lo:hi + 1] - offs[lo]
        prog = sr.Program(ctx, sub, soffs, opts, np.float32)
        pred, ok = prog.eval_predict(ds)

        def one(t):
            ref, rok = oracle.eval_tree(sub[soffs[t]:soffs[t + 1]], opts.binop_codes, opts.unaop_codes, X)
            if bool(ok[t]) != rok:
                return (lo + t, "did_succeed", bool(ok[t]), rok)
            if rok:
                d = np.nonzero(pred[t].view(np.uint32) != ref.view(np.uint32))[0]
                if len(d):
                    return (lo + t, "rows differ", len(d), [(int(i), pred[t][i], ref[i]) for i in d[:4]])
            return None

        with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
            bad = [r for r in ex.map(one, range(hi - lo)) if r is not None]
        assert not bad, bad[:8]
        nok += int(ok.sum())
        del pred, prog
    assert nok == 808  # the loss evaluation's trees_ok: the same mask


def test_c2_plain_program_equals_derived(ctx, monkeypatch):
    """Derived columns (forced with SRHIP_DERIVE_ALWAYS=1 -- C2's launch prefers the
    plain program's longer row blocks) return the same bits as the plain program (SRHIP_NO_DERIVE=1),
    which evaluates every node."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, _, nodes, offs = workloads.c2()
    ds = sr.DeviceDataset(ctx, X, y)
    monkeypatch.setenv("SRHIP_DERIVE_ALWAYS", "1")
    dprog = sr.Program(ctx, nodes, offs, opts, np.float32)
    assert len(dprog.derived_columns()) == 10
    a, aok = dprog.eval_loss(ds, sr.L2DistLoss())
    monkeypatch.setenv("SRHIP_NO_DERIVE", "1")
    plain = sr.Program(ctx, nodes, offs, opts, np.float32)
    assert plain.derived_columns() == []
    b, bok = plain.eval_loss(ds, sr.L2DistLoss())
    assert np.array_equal(aok, bok) and np.array_equal(a.view(np.uint64), b.view(np.uint64))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_early_exit_equals_full_evaluation(ctx, monkeypatch, dtype):
    """A wave stops a tree's row block once the check statistic is non-finite (the reference's
    early return); SRHIP_NO_EARLY_EXIT=1 evaluates every row.  Both give the same bits and masks,
    on the C2 population (216 of 1024 trees fail, most of them on every row block)."""
    sr = _sr()
    from srhip import workloads

    opts, X, y, trees, nodes, offs = workloads.c2(rows=200_000)
    if dtype == np.float64:
        X, y = X.astype(np.float64), y.astype(np.float64)
        nodes, offs = sr.flatten(trees, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    a, aok = prog.eval_loss(ds, sr.L2DistLoss())
    monkeypatch.setenv("SRHIP_NO_EARLY_EXIT", "1")
    b, bok = prog.eval_loss(ds, sr.L2DistLoss())
    assert (~aok).sum() > 100
    assert np.array_equal(aok, bok) and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_c3_shape_matches_oracle(ctx, oracle):
    """C3's dataset (10 features x 10M rows F32) with its 64-tree population."""
    sr = _sr()
    from srhip import workloads

    X, y = workloads.c3_data()
    opts, _, nodes, offs = workloads.c3_population()
    prog = sr.Program(ctx, nodes, offs, opts, np.float32)
    dl, dok = prog.eval_loss(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    _check_losses(dl, dok, ol, ook, F32_REL)
    assert dok.sum() >= 40


@pytest.fixture(scope="module")
def c4():
    from srhip import workloads

    return workloads.c4()


def test_c4_losses_and_grad_kernel_loss(ctx, oracle, c4):
    """C4's 512 trees x 100k F64: eval_loss vs the oracle (1e-12), and the dual-number kernel's
    loss equals eval_loss (the optimiser's objective is the evaluator's)."""
    sr = _sr()
    opts, X, y, _, nodes, offs = c4
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    dl, dok = prog.eval_loss(ds, sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    _check_losses(dl, dok, ol, ook, F64_REL)
    gl, grads, gok = prog.eval_loss_grad(ds, sr.L2DistLoss())
    assert np.array_equal(gok, dok)
    for t in np.nonzero(dok)[0]:
        assert _rel(gl[t], dl[t]) <= F64_REL, (t, gl[t], dl[t])
        assert np.all(np.isfinite(grads[t])) or not np.isfinite(gl[t])


def _const_order(nodes):
    out = []

    def rec(i):
        n = nodes[i]
        if n["degree"] == 0:
            if n["constant"]:
                out.append(i)
            return
        rec(int(n["l"]))
        if n["degree"] == 2:
            rec(int(n["r"]))

    rec(0)
    return out


def test_c4_gradient_vs_oracle_differences(ctx, oracle, c4):
    """d loss / d c of C4 trees (dual numbers, 100k F64 rows) vs Richardson-extrapolated central
    differences of the oracle's loss, on every constant of 64 sampled trees whose differences are
    self-consistent (huge intermediates make c + h round to c inside them: skipped, counted)."""
    sr = _sr()
    opts, X, y, _, nodes, offs = c4
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    loss, grads, ok = prog.eval_loss_grad(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    sample = [t for t in np.random.default_rng(9).permutation(len(offs) - 1) if ok[t] and loss[t] < 1e6][:64]

    def check(t):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        o1 = np.array([0, len(tn)], dtype=np.int64)
        res = []
        for k, i in enumerate(_const_order(tn)):
            def fd(h):
                fp, fm = tn.copy(), tn.copy()
                fp[i]["val"] += h
                fm[i]["val"] -= h
                lp = oracle.eval_loss_batch(fp, o1, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0, nthreads=1)[0][0]
                lm = oracle.eval_loss_batch(fm, o1, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0, nthreads=1)[0][0]
                return (lp - lm) / (2 * h)

            h = 1e-5 * max(1.0, abs(tn[i]["val"]))
            d1, d2 = fd(h), fd(h / 4)
            ref = (16 * d2 - d1) / 15
            if not np.isfinite(ref) or abs(d1 - d2) > 1e-3 * max(1.0, abs(ref)):
                res.append(None)
                continue
            res.append((t, k, grads[t][k], ref))
        return res

    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        results = [r for rs in ex.map(check, sample) for r in rs]
    checked = [r for r in results if r is not None]
    bad = [r for r in checked if not abs(r[2] - r[3]) <= 1e-5 * max(1.0, abs(r[3]))]
    assert not bad, bad[:8]
    assert len(checked) >= 150 and len(checked) >= 0.7 * len(results), (len(checked), len(results))


def test_c4_optimizer_outcome_vs_oracle(ctx, oracle, c4):
    """C4's 512 trees, BFGS(8) / Newton + 2 restarts -- the bench's call itself (bench.py --config c4:
    nrestarts=2, seed=7): never worse than the baseline on any tree, improves most; and on a 32-tree
    sample the outcome equals the exact-gradient restatement's (oracle/optim.py
    optimize_constants_exact over the oracle's dual-number gradient, row sums in the device's order)
    run from the SAME three starts the device used (its own constants, then the two perturbed points
    it reports) with the reference's selection (src/ConstantOptimization.jl:50-78: the first start's
    result unless a restart is strictly better, accepted only if it beats the baseline): loss to
    1e-12 relative, the improved flag, and the returned constants (1e-9) on EVERY sampled tree -- no
    exclusions."""
    import optim

    sr = _sr()
    opts, X, y, _, nodes, offs = c4
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    base, base_ok = prog.eval_loss(ds, sr.L2DistLoss())
    nconst = prog.num_constants().astype(np.int64)
    coff = np.concatenate([[0], np.cumsum(nconst)])
    out, improved, fcalls, starts = prog.optimize_constants(ds, sr.L2DistLoss(), iterations=8, nrestarts=2, seed=7,
                                                           return_starts=True)
    final = prog.get_constants()
    assert np.all(out[base_ok] <= base[base_ok] * (1 + 1e-12))
    assert improved.sum() >= 0.6 * base_ok.sum()
    sample = [t for t in np.random.default_rng(10).permutation(len(offs) - 1) if base_ok[t] and nconst[t] > 0][:32]
    assert len(sample) == 32

    def orc(t):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        x0 = np.array([tn[i]["val"] for i in _const_order(tn)], dtype=np.float64)
        st = [x0] + [starts[r, coff[t]:coff[t + 1]] for r in range(starts.shape[0])]
        return optim.optimize_constants_exact(tn, opts.binop_codes, opts.unaop_codes, X, y, starts=st,
                                              device_order=True)

    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        ref = list(ex.map(orc, sample))
    off = []
    for t, (rx, rl, rimp, _) in zip(sample, ref):
        t = int(t)
        same_loss = out[t] == rl or abs(out[t] - rl) <= 1e-12 * max(abs(out[t]), abs(rl))
        same_x = np.allclose(final[t], rx, rtol=1e-9, atol=0.0)
        if not (same_loss and bool(improved[t]) == bool(rimp) and same_x):
            off.append((t, out[t], rl, bool(improved[t]), bool(rimp), final[t], rx))
    assert not off, off


def test_c4_restart_points_are_reported_and_replayable(ctx, c4):
    """The restart points the device draws are x0 * (1 + randn/2) of the tree's own constants, and
    handing the reported points back as caller-supplied starts reproduces the outcome bit for bit."""
    sr = _sr()
    opts, X, y, _, nodes, offs = c4
    sub = [int(t) for t in range(64)]
    sn = np.concatenate([nodes[offs[t]:offs[t + 1]] for t in sub])
    so = np.concatenate([[0], np.cumsum([offs[t + 1] - offs[t] for t in sub])]).astype(np.int64)
    ds = sr.DeviceDataset(ctx, X, y)
    a = sr.Program(ctx, sn, so, opts, np.float64)
    x0 = np.concatenate(a.get_constants())
    oa, ia, fa, st = a.optimize_constants(ds, sr.L2DistLoss(), nrestarts=2, seed=3, return_starts=True)
    assert st.shape == (2, len(x0))
    ratio = st[:, x0 != 0] / x0[x0 != 0]
    assert np.all(np.isfinite(ratio)) and abs(float(np.mean(ratio)) - 1.0) < 0.2 and 0.3 < float(np.std(ratio)) < 0.7
    b = sr.Program(ctx, sn, so, opts, np.float64)
    ob, ib, fb, st2 = b.optimize_constants(ds, sr.L2DistLoss(), nrestarts=2, seed=999, starts=st, return_starts=True)
    assert np.array_equal(st, st2)
    assert np.array_equal(oa, ob) and np.array_equal(ia, ib) and np.array_equal(fa, fb)
    assert all(np.array_equal(u, v) for u, v in zip(a.get_constants(), b.get_constants()))


def test_c4_restart_selection_float32(ctx):
    """Float32 restart path: the library perturbs in Float32 (val * (1f + 0.5f randn), rounded to
    Float32), and the outcome with nrestarts=2 is the reference's selection over the three single-start
    runs the device makes from the same points (src/ConstantOptimization.jl:50-78): the first start's
    result unless a restart's minimum is strictly smaller, kept only if it beats the baseline.  The
    single-start runs are pinned separately (test_batched_optimizer_equals_per_tree)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    rng = np.random.default_rng(21)
    X = rng.standard_normal((3, 20000)).astype(np.float32)
    y = (2.1 * np.cos(1.3 * X[0]) + 0.7 * X[1] * X[2] - 0.4).astype(np.float32)
    trees = sr.random_population(96, opts, 3, np.float32, seed=22, max_size=16)
    nodes, offs = sr.flatten(trees, opts, np.float32)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    p = sr.Program(ctx, nodes, offs, opts, np.float32)
    x0 = [c.copy() for c in p.get_constants()]
    base, base_ok = p.eval_loss(ds, loss)
    out, imp, fc, st = p.optimize_constants(ds, loss, nrestarts=2, seed=5, return_starts=True)
    assert np.array_equal(st, st.astype(np.float32).astype(np.float64))  # Float32 points
    nconst = np.array([len(c) for c in x0])
    coff = np.concatenate([[0], np.cumsum(nconst)])
    res = []  # (minimum, constants) per start, single-start device runs from each point
    for s in range(3):
        q = sr.Program(ctx, nodes, offs, opts, np.float32)
        if s > 0:
            q.set_constants(st[s - 1])
        # the minimum of a single start: run without acceptance against the baseline by reading the
        # optimiser's best point and re-evaluating it
        ql, qi, _ = q.optimize_constants(ds, loss, nrestarts=0, seed=0)
        res.append((ql, qi, [c.copy() for c in q.get_constants()]))
    final = p.get_constants()
    checked = 0
    for t in range(len(nconst)):
        if nconst[t] == 0 or not base_ok[t]:
            continue
        # a single-start run from point s keeps its own start unless its minimum beats that start's
        # loss, so its reported loss is min(start loss, minimum); only trees where every start's run
        # improved on its own start expose the minimum itself
        if not all(res[s][1][t] for s in range(3)):
            continue
        mins = [res[s][0][t] for s in range(3)]
        # (the reported minima are the evaluator's re-scores, within 1e-6 of the optimiser's own
        # objective values for Float32: near-ties are not decidable from outside and are skipped)
        if any(abs(mins[a] - mins[b]) <= 1e-5 * max(abs(mins[a]), abs(mins[b])) for a in range(3) for b in range(a)):
            continue
        if abs(min(mins) - base[t]) <= 1e-5 * abs(base[t]):
            continue
        best = 0
        for s in (1, 2):
            if mins[s] < mins[best]:
                best = s
        if mins[best] < base[t]:
            assert imp[t], t
            assert np.array_equal(final[t], res[best][2][t]), (t, best, final[t], res[best][2][t])
        else:
            assert not imp[t], t
            assert np.array_equal(final[t], x0[t])
        checked += 1
    assert checked >= 20, checked


def test_c4_restart_float32_vs_oracle(ctx, oracle):
    """The Float32 restart path pinned to the oracle (no near-tie exclusions): a Float32 population,
    BFGS / Newton + 2 restarts drawn in Float32 (val * (1f + 0.5f randn)), and on >= 32 trees the
    outcome equals oracle/optim.py optimize_constants_exact run from the device's own three starts
    over the oracle's Float32 dual-number objective in the device's row order
    (sr_oracle_grad.h oracle_loss_grad_devorder_f32: constants rounded to Float32 per call, values and
    tangents in Float32) with the reference's selection (src/ConstantOptimization.jl:50-78): the
    improved flag, the returned Float32 constants, and the loss to 1e-6 relative."""
    import optim

    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp"))
    rng = np.random.default_rng(21)
    X = rng.standard_normal((3, 20000)).astype(np.float32)
    y = (2.1 * np.cos(1.3 * X[0]) + 0.7 * X[1] * X[2] - 0.4).astype(np.float32)
    trees = sr.random_population(96, opts, 3, np.float32, seed=22, max_size=16)
    nodes, offs = sr.flatten(trees, opts, np.float32)
    ds = sr.DeviceDataset(ctx, X, y)
    p = sr.Program(ctx, nodes, offs, opts, np.float32)
    base, base_ok = p.eval_loss(ds, sr.L2DistLoss())
    nconst = p.num_constants().astype(np.int64)
    coff = np.concatenate([[0], np.cumsum(nconst)])
    out, improved, _, starts = p.optimize_constants(ds, sr.L2DistLoss(), iterations=8, nrestarts=2, seed=5,
                                                   return_starts=True)
    final = p.get_constants()
    sample = [int(t) for t in range(len(nconst)) if base_ok[t] and nconst[t] > 0][:40]
    assert len(sample) >= 32, len(sample)

    def orc(t):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        x0 = np.array([tn[i]["val"] for i in _const_order(tn)], dtype=np.float64)
        st = [x0] + [starts[r, coff[t]:coff[t + 1]] for r in range(starts.shape[0])]
        return optim.optimize_constants_exact(tn, opts.binop_codes, opts.unaop_codes, X, y, starts=st,
                                              device_order=True)

    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        ref = list(ex.map(orc, sample))
    off = []
    for t, (rx, rl, rimp, _) in zip(sample, ref):
        same_loss = out[t] == rl or abs(out[t] - rl) <= 1e-6 * max(abs(out[t]), abs(rl))
        same_x = np.array_equal(np.asarray(final[t], np.float32), np.asarray(rx, np.float64).astype(np.float32))
        if not (same_loss and bool(improved[t]) == bool(rimp) and same_x):
            off.append((t, out[t], rl, bool(improved[t]), bool(rimp), final[t], rx))
    assert not off, off


def test_c5_int32_population_1m_rows_bit_exact(ctx, oracle):
    """C5 Int32: random + - * trees with small integer constants over 3 x 1M Int32 rows (wrap-around
    arithmetic): predictions' loss and masks bit-exact against the oracle."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("square", "neg"))
    rng = np.random.default_rng(13)
    trees = sr.random_population(128, opts, 3, np.float64, seed=14, max_size=20)
    for tr in trees:
        for nd in tr:
            if nd.degree == 0 and nd.constant:
                nd.val = int(rng.integers(-5, 6))
    nodes, offs = sr.flatten(trees, opts, np.int32)
    X = rng.integers(-5, 6, size=(3, 1_000_000)).astype(np.int32)  # test_integer_evaluation.jl's range
    y = rng.integers(-50, 50, size=1_000_000).astype(np.int32)
    prog = sr.Program(ctx, nodes, offs, opts, np.int32)
    dl, dok = prog.eval_loss(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook) and dok.all()
    assert np.array_equal(dl, ol)


def _custom_objective_options(sr, **kw):
    """test/test_custom_objectives.jl:5-35: the user loss multiplies the tree by 2 and sums |out - y|
    over eval_tree_array's predictions; elementwise_loss = nothing."""
    def my_custom_loss(tree, dataset, options):
        tree = sr.Node(1, tree, sr.Node(val=2.0))  # binary op #1 = "*"
        out, completed = sr.eval_tree_array(tree, dataset.X, options)
        if not completed:
            return np.inf
        return float(np.sum(np.abs(out - dataset.y)))

    return sr.Options(binary_operators=("*", "/", "+", "-"), unary_operators=("cos", "sin"),
                      loss_function=my_custom_loss, maxsize=10, **kw)


def test_c5_custom_objective_loss_function(ctx, oracle):
    """C5 custom objective (test/test_custom_objectives.jl): eval_loss / score_func route to the user
    loss_function (src/LossFunctions.jl:97-112), whose eval_tree_array runs on the device; values
    match the oracle's eval_tree of the same doubled tree, and 0.5 * (x1 + x2) -- the reference
    test's expected optimum -- scores ~0."""
    sr = _sr()
    from srhip import workloads

    opts = _custom_objective_options(sr)
    X, y = workloads.c5_custom_objective_data()
    ds = sr.Dataset(X, y)
    x1, x2 = sr.Node("x1"), sr.Node("x2")
    trees = [sr.Node(val=0.5) * (x1 + x2), x1 + x2, x1 * x2 - sr.cos(x2), sr.sin(x1) / x2, x1 / sr.Node(val=0.0)]
    for tree in trees:
        got = sr.eval_loss(tree, ds, opts)
        doubled = sr.Node(1, tree, sr.Node(val=2.0))
        nodes, _ = sr.flatten([doubled], opts, np.float64)
        pred, ok = oracle.eval_tree(nodes, opts.binop_codes, opts.unaop_codes, X)
        want = float(np.sum(np.abs(pred - y))) if ok else np.inf
        assert got == want or abs(got - want) <= 1e-12 * abs(want), (sr.string_tree(tree, opts), got, want)
        assert sr.score_func(ds, tree, opts)[1] == got
    assert sr.eval_loss(trees[0], ds, opts) < 1e-10
    # batching with a 3-argument loss_function is an error (src/LossFunctions.jl:84-90)
    with pytest.raises(RuntimeError):
        sr.eval_loss(trees[0], ds, _custom_objective_options(sr, batching=True))


def test_c5_custom_objective_optimize_constants(ctx, oracle):
    """optimize_constants with a user loss_function (src/ConstantOptimization.jl:48: the objective is
    eval_loss, i.e. the user's function): host Newton / BFGS with finite differences over device
    predictions (srhip.host_optim).  (a) with a user loss equal to the mean squared error the outcome
    matches the reference procedure on L2 (oracle/optim.py) -- same algorithm, same objective; (b)
    test_custom_objectives.jl's own loss improves c * (x1 + x2) towards 0.5.  Improved members get a
    new birth (:76) and are re-scored with regularization (:73)."""
    import optim

    sr = _sr()
    from srhip import workloads

    X, y = workloads.c5_custom_objective_data()
    ds = sr.Dataset(X, y)
    x1, x2 = sr.Node("x1"), sr.Node("x2")

    def mse(tree, dataset, options):
        out, ok = sr.eval_tree_array(tree, dataset.X, options)
        return float(np.mean((out - dataset.y) ** 2)) if ok else np.inf

    base = dict(binary_operators=("*", "/", "+", "-"), unary_operators=("cos", "sin"), optimizer_nrestarts=0)
    user = sr.Options(loss_function=mse, **base)
    for start in (sr.Node(val=0.2) * x1 + sr.Node(val=1.7) * sr.cos(x2 * sr.Node(val=0.1)),  # BFGS
                  sr.Node(val=0.3) * (x1 + x2),                                              # Newton
                  sr.sin(x1) * sr.Node(val=2.0) + x2):                                       # Newton
        m = sr.PopMember(start.copy(), np.inf, np.inf)
        b0 = m.birth
        m, ne = sr.optimize_constants(ds, m, user, rng=np.random.default_rng(1))
        nodes, _ = sr.flatten([start], user, np.float64)
        _, ol, oimp = optim.optimize_constants(nodes, user.binop_codes, user.unaop_codes, X, y, nrestarts=0)
        assert oimp and m.birth > b0 and ne > 0
        assert abs(m.loss - ol) <= 1e-6 * ol + 1e-12, (sr.string_tree(start, user), m.loss, ol)
        assert m.loss == sr.eval_loss(m.tree, ds, user)
    # (b) the reference test's objective
    opts = _custom_objective_options(sr, optimizer_nrestarts=1)
    m = sr.PopMember(sr.Node(val=0.3) * (x1 + x2), np.inf, np.inf)
    before = sr.eval_loss(m.tree, ds, opts)
    m, _ = sr.optimize_constants(ds, m, opts, rng=np.random.default_rng(2))
    assert m.loss < 0.1 * before and abs(sr.get_constants(m.tree)[0] - 0.5) < 0.05


def test_units_penalty_added_to_device_loss(ctx):
    """_eval_loss adds dimensional_regularization to the device loss when the dataset has units
    (src/LossFunctions.jl:70-72): a violating tree pays 1000 on top of its L2 loss, eval_loss and
    score_func_batch agree, and regularization=false leaves the device loss alone."""
    sr = _sr()
    X = np.random.default_rng(5).standard_normal((3, 1000))
    y = np.cos(X[2] * 2.1 - 0.2) + 0.5
    opts = sr.Options(binary_operators=("-", "*", "/", "+"), unary_operators=("cos",))
    ds = sr.Dataset(X, y, X_units=["m", "1", "kg"], y_units="1")
    plain = sr.Dataset(X, y)
    x1, x2 = sr.Node("x1"), sr.Node("x2")
    good, bad = sr.cos(3.2 * x1) - x2, sr.cos(x1) + x2
    for tree, pen in ((good, 0.0), (bad, 1000.0)):
        raw = sr.eval_loss(tree, plain, opts)
        assert sr.eval_loss(tree, ds, opts, regularization=False) == raw
        assert sr.eval_loss(tree, ds, opts) == np.float64(raw) + pen
    _, losses = sr.score_func_batch(ds, [good, bad], opts)
    assert losses[1] - sr.eval_loss(bad, plain, opts) == pytest.approx(1000.0)
