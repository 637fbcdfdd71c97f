"""Device constant gradients (dual numbers) and the batched constant optimiser vs the oracle.

Parity for the optimiser is at the outcome: the reference differentiates by
finite differences, the device exactly, so iterates differ; the bar is the optimised loss.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OPS = dict(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp", "sin"))


def _sr():
    import srhip

    return srhip


def _problem(sr, dtype, ntrees=40, n=3000, seed=11, max_size=20):
    opts = sr.Options(**OPS)
    trees = sr.random_population(ntrees, opts, 3, dtype, seed=seed, max_size=max_size)
    nodes, offs = sr.flatten(trees, opts, dtype)
    rng = np.random.default_rng(seed + 1)
    X = rng.standard_normal((3, n)).astype(dtype)
    y = (np.cos(1.3 * X[0]) * 2.0 + X[1] * 0.7 - 0.3).astype(dtype)
    return opts, trees, nodes, offs, X, y


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_grad_kernel_loss_equals_eval_loss(ctx, dtype):
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    el, eok = prog.eval_loss(ds, sr.L2DistLoss())
    gl, _, gok = prog.eval_loss_grad(ds, sr.L2DistLoss())
    assert np.array_equal(eok, gok)
    tol = 1e-6 if dtype == np.float32 else 1e-12
    for t in np.nonzero(eok)[0]:
        assert abs(gl[t] - el[t]) <= tol * abs(el[t]) + 1e-300, (t, gl[t], el[t])


def test_grad_matches_central_differences(ctx, oracle):
    """d loss / d c from the dual-number kernel vs central differences of the oracle's loss (F64).
    Operators without huge intermediates (no exp, no /): where an intermediate is ~1e300, c + h
    rounds to c inside it and differences see no change while the exact derivative does not vanish."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("cos", "sin"))
    trees = sr.random_population(24, opts, 3, np.float64, seed=11, max_size=20)
    nodes, offs = sr.flatten(trees, opts, np.float64)
    rng = np.random.default_rng(12)
    X = rng.standard_normal((3, 1500))
    y = np.cos(1.3 * X[0]) * 2.0 + X[1] * 0.7 - 0.3
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    loss, grads, ok = prog.eval_loss_grad(ds, sr.L2DistLoss())
    checked = 0
    for t in np.nonzero(ok)[0]:
        tn = nodes[offs[t]:offs[t + 1]].copy()
        cidx = [i for i in _order(tn)]
        if not cidx or not np.isfinite(loss[t]) or loss[t] > 1e6:
            continue
        one = np.array([0, len(tn)], dtype=np.int64)

        def fd(i, h):
            fp, fm = tn.copy(), tn.copy()
            fp[i]["val"] += h
            fm[i]["val"] -= h
            lp = oracle.eval_loss_batch(fp, one, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)[0][0]
            lm = oracle.eval_loss_batch(fm, one, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)[0][0]
            return (lp - lm) / (2 * h)

        for k, i in enumerate(cidx):
            h = 1e-5 * max(1.0, abs(tn[i]["val"]))
            d1, d2 = fd(i, h), fd(i, h / 4)
            # Richardson: the two steps' O(h^2) errors cancel; skip where differences are unreliable
            ref = (16 * d2 - d1) / 15
            if not np.isfinite(ref) or abs(d1 - d2) > 1e-3 * max(1.0, abs(ref)):
                continue
            assert abs(grads[t][k] - ref) <= 1e-5 * max(1.0, abs(ref)), (t, k, grads[t][k], ref)
            checked += 1
    assert checked >= 20


def _order(nodes):
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


def test_grad_of_scaled_feature_is_the_feature(ctx):
    """test/test_derivatives.jl:85-93: d/dC sum(C * x1) = sum(x1)  ->  for L2: dL/dC = mean(2 (C x1 - y) x1)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("*",), unary_operators=())
    X = np.random.default_rng(0).standard_normal((3, 1000))
    y = np.zeros(1000)
    tree = sr.Node(val=3.2) * sr.Node("x1")
    nodes, offs = sr.flatten([tree], opts, np.float64)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    _, grads, ok = prog.eval_loss_grad(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss())
    assert ok[0]
    expect = np.mean(2 * (3.2 * X[0]) * X[0])
    assert abs(grads[0][0] - expect) <= 1e-12 * abs(expect)


def test_optimizer_recovers_reference_constants(ctx):
    """test/test_optimizer_mutation.jl:8-42 on the device optimiser."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("sin",))
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, 100))
    y = np.sin(X[0] * 2.1 + 0.8) + X[1] ** 2
    x1, x2 = sr.Node("x1"), sr.Node("x2")
    tree = sr.sin(x1 * sr.Node(val=1.9) + sr.Node(val=0.2)) + x2 * x2
    nodes, offs = sr.flatten([tree], opts, np.float64)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    loss, improved, _ = prog.optimize_constants(sr.DeviceDataset(ctx, X, y), sr.L2DistLoss(), seed=1)
    c = prog.get_constants()[0]
    assert improved[0]
    for k in (0.0, 0.2, 0.5, 1.0):
        assert abs(np.sin(c[0] * k + c[1]) - np.sin(2.1 * k + 0.8)) < 1e-3
    assert loss[0] < 1e-8


def test_optimizer_outcome_vs_exact_oracle(ctx, oracle):
    """Batched device BFGS / Newton vs the same optimiser restated over the oracle's exact gradient
    (oracle/optim.py optimize_constants_exact: Optim's BFGS / Newton + LineSearches' BackTracking in
    their source's arithmetic order, forward-mode dual-number gradient, sr_oracle_grad.h), single
    start, on EVERY tree with constants: the optimum agrees to 1e-12 relative.  The oracle sums its
    per-row losses and tangents in the device kernel's row order (device_order=True): with exact
    sums instead, line searches that compare phi at the rounding noise (tiny steps on chaotic trees)
    decide differently and the trajectories part -- by the sums' last bits, not by the algorithm."""
    import optim

    sr = _sr()
    opts, trees, nodes, offs, X, y = _problem(sr, np.float64, ntrees=32, n=1500, seed=5, max_size=14)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    base, base_ok = prog.eval_loss(ds, sr.L2DistLoss())
    dl, improved, _ = prog.optimize_constants(ds, sr.L2DistLoss(), nrestarts=0, seed=3)
    checked, off = 0, []
    for t in range(len(trees)):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        if not base_ok[t] or not _order(tn):
            continue
        _, ol, _, _ = optim.optimize_constants_exact(tn, opts.binop_codes, opts.unaop_codes, X, y,
                                               device_order=True)
        checked += 1
        if not _rel_close(dl[t], ol, 1e-12):
            off.append((t, sr.string_tree(trees[t], opts), dl[t], ol, base[t]))
    assert checked >= 20
    assert not off, off


def _rel_close(a, b, tol):
    if a == b:
        return True
    if not (np.isfinite(a) and np.isfinite(b)):
        return False
    return abs(a - b) <= tol * max(abs(a), abs(b))


def test_optimizer_outcome_vs_fd_reference_procedure(ctx, oracle):
    """The documented deviation from the reference: libsrhip differentiates exactly, the reference
    by finite differences (Optim with only f).  Against the finite-difference restatement
    (oracle/optim.py), single start: never worse than the baseline, and at least as good as the
    oracle's optimum (1e-6 relative) on every tree whose finite-difference optimum is resolved
    (optim.reference_outcome: reproduced with 4x the difference step); on the others the two
    differentiations follow different, equally valid trajectories (they are listed)."""
    import optim

    sr = _sr()
    opts, trees, nodes, offs, X, y = _problem(sr, np.float64, ntrees=32, n=1500, seed=5, max_size=14)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    base, base_ok = prog.eval_loss(ds, sr.L2DistLoss())
    dl, improved, _ = prog.optimize_constants(ds, sr.L2DistLoss(), nrestarts=0, seed=3)
    assert np.all(dl[base_ok] <= base[base_ok] * (1 + 1e-12))
    total, lost, unresolved = 0, [], []
    for t in range(len(trees)):
        tn = nodes[offs[t]:offs[t + 1]].copy()
        if not base_ok[t] or not _order(tn):
            continue
        ol, stable = optim.reference_outcome(tn, opts.binop_codes, opts.unaop_codes, X, y)
        total += 1
        if not stable:
            unresolved.append((t, sr.string_tree(trees[t], opts)))
        elif not dl[t] <= ol * (1 + 1e-6) + 1e-12:
            lost.append((t, len(_order(tn)), dl[t], ol, base[t]))
    assert total >= 10 and total - len(unresolved) >= 8
    assert len(unresolved) <= total // 3, unresolved
    assert not lost, (lost, unresolved)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_grad_program_patch_equals_full_compile(ctx, dtype):
    """After set_constants, the gradient program recompiles only the trees whose constants moved
    (in place, srhip_host.cpp patch_grad_t); its losses, gradients and masks equal, bit for bit, a
    fresh program compiled in full with the same constants — including a tree whose new constant
    is NaN (a static did_succeed failure), a second patch on top of the first, and that tree patched
    back into its kept slot once its constants are finite again."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=48)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    ok0 = prog.eval_loss_grad(ds, loss)[2]  # full compile of the gradient program
    c = prog.get_constants()
    rng = np.random.default_rng(3)
    with_c = [t for t in range(len(c)) if len(c[t]) > 0]
    assert len(with_c) >= 6
    victim = next(t for t in with_c[1:] if ok0[t])
    with_c.remove(victim)
    with_c.insert(1, victim)
    keep = c[with_c[1]].copy()
    for step in range(3):
        for t in with_c[step::3]:
            if t != with_c[1]:
                c[t] = c[t] * (1.0 + 0.25 * rng.standard_normal(len(c[t])))
        if step == 0:
            c[with_c[1]][0] = np.nan  # a static failure: the tree keeps its slot
        if step == 2:
            c[with_c[1]] = keep.copy()  # finite again, same code length: patched back into its slot
        flat = np.concatenate(c)
        prog.set_constants(flat)
        pl, pg, pok = prog.eval_loss_grad(ds, loss)
        fresh = sr.Program(ctx, nodes, offs, opts, dtype)
        fresh.set_constants(flat)
        fl, fg, fok = fresh.eval_loss_grad(ds, loss)
        fresh.close()
        assert np.array_equal(pok, fok)
        assert pok[with_c[1]] == (step == 2)
        assert np.array_equal(pl.view(np.uint64), fl.view(np.uint64))
        assert np.array_equal(np.concatenate(pg).view(np.uint64), np.concatenate(fg).view(np.uint64))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_batched_optimizer_equals_per_tree(ctx, dtype):
    """The pipelined optimiser (srhip_optim.cpp bfgs_pipelined: every tree runs its own
    start / Hessian-probe / line-search state machine, one launch per round over the trees still
    active) returns, bit for bit, the losses, improvement flags, evaluation counts and constants that
    optimising each tree alone returns -- a tree's loss and gradient do not depend on which trees
    share a launch.  The population mixes Newton (one constant) and BFGS trees."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=40)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    nconst = prog.num_constants()
    assert (nconst == 1).sum() >= 3 and (nconst >= 2).sum() >= 10
    out, improved, fcalls = prog.optimize_constants(ds, loss, iterations=8, nrestarts=0, seed=11)
    consts = prog.get_constants()
    assert improved[nconst == 1].any() and improved[nconst >= 2].any()
    for t in range(len(offs) - 1):
        one = sr.Program(ctx, nodes[offs[t]:offs[t + 1]], np.array([0, offs[t + 1] - offs[t]]), opts, dtype)
        o1, i1, f1 = one.optimize_constants(ds, loss, iterations=8, nrestarts=0, seed=11)
        assert i1[0] == improved[t] and f1[0] == fcalls[t], t
        assert np.asarray(o1[0], np.float64).view(np.uint64) == np.asarray(out[t], np.float64).view(np.uint64), t
        assert np.array_equal(one.get_constants()[0].view(np.uint64), consts[t].view(np.uint64)), t
        one.close()


def test_optimizer_fcalls_accounting(ctx):
    """num_evals bookkeeping (src/ConstantOptimization.jl:51,65,79): no constants -> 0;
    otherwise the objective calls of every start, + 1 when the tree was improved (its re-score)."""
    sr = _sr()
    opts = sr.Options(binary_operators=("+", "*"), unary_operators=("cos",))
    x1 = sr.Node("x1")
    X = np.random.default_rng(1).standard_normal((1, 500))
    y = 2.5 * X[0] + 0.5
    trees = [sr.cos(x1) + x1,                              # no constants
             sr.Node(val=1.0) * x1 + sr.Node(val=0.1),     # BFGS, improves
             sr.Node(val=2.5) * x1 + sr.Node(val=0.5)]     # already optimal: gradient 0 at start
    nodes, offs = sr.flatten(trees, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    _, improved, fcalls = prog.optimize_constants(ds, sr.L2DistLoss(), nrestarts=2, seed=5)
    assert fcalls[0] == 0 and not improved[0]
    assert improved[1] and fcalls[1] >= 3 * 2 + 1  # >= initial + one trial per start, + the re-score
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    _, improved, fcalls = prog.optimize_constants(ds, sr.L2DistLoss(), nrestarts=0, seed=5)
    assert fcalls[0] == 0 and not improved[0]
    assert not improved[2] and fcalls[2] == 1  # zero gradient at the start: one call, nothing accepted


def test_newton_outcome_vs_oracle(ctx, oracle):
    """One-constant trees take Newton (src/ConstantOptimization.jl:27-31) on the device and in the
    oracle: the device optimum matches or beats the oracle's (1e-6 relative) on every tree whose
    reference optimum is resolved (optim.reference_outcome)."""
    import optim

    sr = _sr()
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp", "sin"))
    rng = np.random.default_rng(21)
    trees = []
    while len(trees) < 24:
        t = sr.gen_random_tree_fixed_size(int(rng.integers(3, 12)), opts, 3, np.float64, rng)
        if sr.count_constants(t) == 1:
            trees.append(t)
    nodes, offs = sr.flatten(trees, opts, np.float64)
    X = rng.standard_normal((3, 2000))
    y = np.cos(1.3 * X[0]) * 2.0 + X[1] * 0.7 - 0.3
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    ds = sr.DeviceDataset(ctx, X, y)
    base, base_ok = prog.eval_loss(ds, sr.L2DistLoss())
    dl, improved, _ = prog.optimize_constants(ds, sr.L2DistLoss(), nrestarts=0, seed=3)
    checked, unresolved = 0, []
    for t in range(len(trees)):
        if not base_ok[t]:
            continue
        tn = nodes[offs[t]:offs[t + 1]].copy()
        assert dl[t] <= base[t] * (1 + 1e-12)
        ol, stable = optim.reference_outcome(tn, opts.binop_codes, opts.unaop_codes, X, y)
        if not stable:  # e.g. sin(exp(c - (x2 - exp(x1)))): the loss oscillates below the difference step
            unresolved.append((t, sr.string_tree(trees[t], opts)))
            continue
        assert dl[t] <= ol * (1 + 1e-6) + 1e-12, (t, dl[t], ol, base[t])
        checked += 1
    assert checked >= 12 and improved.sum() >= 8, (checked, unresolved)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_grad_tangent_width_4_equals_8(ctx, dtype, monkeypatch):
    """Gradient launches carry 4 or 8 tangents per chunk (chosen per launch from the population's
    constant counts, srhip_optim.cpp eval_grad); losses, gradients and masks are bit-identical
    either way (independent tangent components over the same primal code)."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=48)
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    res = []
    for kt in ("4", "8"):
        monkeypatch.setenv("SRHIP_GRAD_KT", kt)
        res.append(prog.eval_loss_grad(ds, sr.L2DistLoss()))
    (l4, g4, o4), (l8, g8, o8) = res
    assert max(len(c) for c in prog.get_constants()) > 4  # some trees span several 4-wide chunks
    assert np.array_equal(o4, o8)
    assert np.array_equal(l4.view(np.uint64), l8.view(np.uint64))
    assert np.array_equal(np.concatenate(g4).view(np.uint64), np.concatenate(g8).view(np.uint64))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_speculative_trials_equal_sequential(ctx, dtype, monkeypatch, capfd):
    """Value-only trial points (SRHIP_OPTIM_VALUE_TRIALS: a line search's later trials without
    tangents, the gradient fetched at the accepted point) and speculative line-search points (SRHIP_OPTIM_SPEC slots: the next alphas a backtracking tree
    would try, evaluated in spare program slots of the same launch and consumed only while the line
    search asks for exactly that alpha) change nothing: losses, flags, objective-call counts and
    constants equal the sequential pipeline's bit for bit, on C4-shaped trees whose overflowing
    directions backtrack for hundreds of trials -- and the speculation is really used."""
    import re

    import srhip.workloads as wl

    sr = _sr()
    opts, X, y, trees, nodes, offs = wl.c4(ntrees=96, rows=2000)
    if dtype == np.float32:
        nodes, offs = sr.flatten(trees, opts, np.float32)
        X, y = X.astype(np.float32), y.astype(np.float32)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    res = {}
    # (speculative slots, value-only trials): the plain pipeline first
    for spec, vt in (("0", "0"), ("0", "1"), ("256", "0"), ("256", "1")):
        monkeypatch.setenv("SRHIP_OPTIM_SPEC", spec)
        monkeypatch.setenv("SRHIP_OPTIM_VALUE_TRIALS", vt)
        monkeypatch.setenv("SRHIP_OPTIM_TIMING", "2")
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        out, improved, fcalls = prog.optimize_constants(ds, loss, iterations=8, nrestarts=2, seed=5)
        res[spec, vt] = (np.asarray(out, np.float64), improved.copy(), fcalls.copy(), prog.get_constants())
        prog.close()
        err = capfd.readouterr().err
        m = re.findall(r"speculative points (\d+) evaluated, (\d+) used", err)
        assert m, err[-2000:]
        res[spec, vt, "used"] = int(m[-1][1])
    assert res["0", "0", "used"] == 0 and res["256", "1", "used"] > 0 and res["256", "0", "used"] > 0
    a = res["0", "0"]
    for key in (("0", "1"), ("256", "0"), ("256", "1")):
        b = res[key]
        assert np.array_equal(a[0].view(np.uint64), b[0].view(np.uint64)), key
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]), key
        for ca, cb in zip(a[3], b[3]):
            assert np.array_equal(np.asarray(ca).view(np.uint64), np.asarray(cb).view(np.uint64)), key


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_split_optimizer_equals_single_group(ctx, dtype, monkeypatch):
    """The optimiser splits populations of >= 64 trees into SRHIP_OPTIM_SPLIT groups, each group but
    the first a program of its own on an auxiliary context driven from its own host thread
    (srhip_optim.cpp optimize_split).  Losses, improvement flags, evaluation counts and constants are
    bit-identical to one group (a tree's trajectory does not depend on its launch companions)."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=96)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    res = []
    for g in ("1", "2", "3"):
        monkeypatch.setenv("SRHIP_OPTIM_SPLIT", g)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        out, improved, fcalls = prog.optimize_constants(ds, loss, iterations=8, nrestarts=1, seed=3)
        res.append((np.asarray(out, np.float64), improved, fcalls, np.concatenate(prog.get_constants())))
        prog.close()
    base = res[0]
    assert base[1].sum() > 10
    for r in res[1:]:
        assert np.array_equal(r[0].view(np.uint64), base[0].view(np.uint64))
        assert np.array_equal(r[1], base[1]) and np.array_equal(r[2], base[2])
        assert np.array_equal(r[3].view(np.uint64), base[3].view(np.uint64))


@pytest.mark.parametrize("kind_name,args", [("LogitMarginLoss", ()), ("L2MarginLoss", ()), ("ExpLoss", ()),
                                            ("SigmoidLoss", ()), ("ModifiedHuberLoss", ()), ("L2HingeLoss", ()),
                                            ("SmoothedL1HingeLoss", (0.6,)), ("DWDMarginLoss", (1.5,)),
                                            ("HuberLoss", (0.5,)), ("LogitDistLoss", ())])
def test_loss_kind_gradients_match_differences(ctx, kind_name, args):
    """d loss / d c of the dual-number kernel for the other loss kinds (margin losses through the chain
    rule target * dL/da) vs Richardson central differences of the device's own loss (F64)."""
    sr = _sr()
    loss = getattr(sr, kind_name)(*args)
    opts = sr.Options(binary_operators=("+", "-", "*"), unary_operators=("cos",))
    trees = sr.random_population(16, opts, 2, np.float64, seed=5, max_size=12)
    nodes, offs = sr.flatten(trees, opts, np.float64)
    rng = np.random.default_rng(6)
    X = rng.standard_normal((2, 800))
    margin = isinstance(loss, sr.MarginLoss)
    y = np.where(X[0] + 0.3 * X[1] > 0, 1.0, -1.0) if margin else np.cos(X[0]) + 0.5 * X[1]
    ds = sr.DeviceDataset(ctx, X, y)
    prog = sr.Program(ctx, nodes, offs, opts, np.float64)
    l0, grads, ok = prog.eval_loss_grad(ds, loss)
    checked = 0
    for t in np.nonzero(ok)[0]:
        tn = nodes[offs[t]:offs[t + 1]].copy()
        cidx = _order(tn)
        if not cidx or not np.isfinite(l0[t]):
            continue
        one = np.array([0, len(tn)], dtype=np.int64)

        def f(nd):
            p = sr.Program(ctx, nd, one, opts, np.float64)
            v = p.eval_loss(ds, loss)[0][0]
            p.close()
            return v

        for k, i in enumerate(cidx):
            h = 1e-5 * max(1.0, abs(tn[i]["val"]))

            def fd(hh):
                fp, fm = tn.copy(), tn.copy()
                fp[i]["val"] += hh
                fm[i]["val"] -= hh
                return (f(fp) - f(fm)) / (2 * hh)

            d1, d2 = fd(h), fd(h / 4)
            ref = (16 * d2 - d1) / 15
            if not np.isfinite(ref) or abs(d1 - d2) > 1e-3 * max(1.0, abs(ref)):
                continue
            assert abs(grads[t][k] - ref) <= 1e-5 * max(1.0, abs(ref)), (t, k, grads[t][k], ref)
            checked += 1
    assert checked >= 6


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_inline_chunk_list_equals_staged_copy(ctx, dtype, monkeypatch):
    """Gradient launches of at most 96 chunks carry their (tree, first constant) list in the kernel
    arguments; SRHIP_GRAD_INLINE_MAX=0 stages it through a host-to-device copy instead.  Losses,
    gradients and did_succeed are bitwise the same either way, and so is an optimize_constants run
    (whose many small launches take the inline form)."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    res = {}
    for lim in ("0", "96"):
        monkeypatch.setenv("SRHIP_GRAD_INLINE_MAX", lim)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, sr.L2DistLoss())
        out, imp, fc = prog.optimize_constants(ds, sr.L2DistLoss(), iterations=8, nrestarts=1, seed=3)
        res[lim] = (np.asarray(l, np.float64), np.concatenate(g), ok, np.asarray(out, np.float64), imp, fc,
                    np.concatenate(prog.get_constants()))
        prog.close()
    a, b = res["0"], res["96"]
    for u, v in zip(a, b):
        u, v = np.asarray(u), np.asarray(v)
        if u.dtype.kind == "f":
            assert np.array_equal(u.view(np.uint64 if u.itemsize == 8 else np.uint32),
                                  v.view(np.uint64 if v.itemsize == 8 else np.uint32))
        else:
            assert np.array_equal(u, v)


def _bits_equal(u, v):
    u, v = np.asarray(u), np.asarray(v)
    if u.dtype.kind == "f":
        return np.array_equal(u.view(np.uint64 if u.itemsize == 8 else np.uint32),
                              v.view(np.uint64 if v.itemsize == 8 else np.uint32))
    return np.array_equal(u, v)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_value_only_screening_is_exact(ctx, dtype, monkeypatch):
    """Value-only passes evaluate row block 0 of every chunk first (a launch of its own) and skip the
    other blocks of a chunk whose block-0 check statistic is already non-finite (SRHIP_GRAD_SCREEN,
    0 = one launch).  Losses and did_succeed are bitwise those of the unscreened pass: a tree that
    overflows in block 0 (skipped), one that overflows only in a later block (not skipped, still
    fails), finite trees (unchanged sums); and an optimize_constants run ends identically."""
    sr = _sr()
    n = 3000  # 12 row blocks of 256
    rng = np.random.default_rng(5)
    X = rng.uniform(-1.0, 1.0, (3, n)).astype(dtype)
    X[1, 17] = 1000.0    # exp(x1) overflows in block 0
    X[0, 2100] = 1000.0  # exp(x0) overflows only in block 8
    y = (X[0] * 0.5 + X[2]).astype(dtype)
    opts = sr.Options(**OPS)
    exp_op = opts.unary_operators.index("exp") + 1
    E = lambda ch: sr.Node(exp_op, ch)  # noqa: E731
    trees = [sr.Node(3, E(sr.Node(feature=2)), sr.Node(val=1.5)),   # exp(x1) * 1.5: fails in block 0
             sr.Node(1, E(sr.Node(feature=1)), sr.Node(val=0.25)),  # exp(x0) + 0.25: fails in block 8
             sr.Node(1, sr.Node(feature=3), sr.Node(val=0.5))]      # x2 + 0.5: finite
    trees = trees * 3 + sr.random_population(24, opts, 3, dtype, seed=19, max_size=16)
    nodes, offs = sr.flatten(trees, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    monkeypatch.setenv("SRHIP_GRAD_VALUE_ONLY", "1")
    res = {}
    for scr in ("0", "1"):
        monkeypatch.setenv("SRHIP_GRAD_SCREEN", scr)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, _, ok = prog.eval_loss_grad(ds, sr.L2DistLoss())
        res[scr] = (np.asarray(l, np.float64), np.asarray(ok))
        prog.close()
    assert list(res["1"][1][:3]) == [0, 0, 1], res["1"][1][:3]
    for u, v in zip(res["0"], res["1"]):
        assert _bits_equal(u, v)
    monkeypatch.delenv("SRHIP_GRAD_VALUE_ONLY")
    opts, _, nodes, offs, X, y = _problem(sr, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    res = {}
    for scr in ("0", "1"):
        monkeypatch.setenv("SRHIP_GRAD_SCREEN", scr)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        out, imp, fc = prog.optimize_constants(ds, sr.L2DistLoss(), iterations=8, nrestarts=1, seed=3)
        res[scr] = (np.asarray(out, np.float64), imp, fc, np.concatenate(prog.get_constants()))
        prog.close()
    for u, v in zip(res["0"], res["1"]):
        assert _bits_equal(u, v)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_derived_view_is_exact(ctx, dtype, monkeypatch):
    """Constant-gradient launches read every heavy operator of a feature (cos(x), exp(x), ...) from a
    derived view's column, computed once per call with the kernel's own value function, with the
    operator's check fold and precise-sum ordinal on the load (srhip_optim.cpp derived_view).  Losses,
    gradients, did_succeed (an exp(x) overflowing in one row included), value-only passes and a
    split optimize_constants run are bitwise those of the per-row operators (SRHIP_GRAD_DERIVED=0);
    per-row derivatives after an optimiser call on the same program (which compiles it back without
    derived columns) equal a fresh program's."""
    sr = _sr()
    monkeypatch.setenv("SRHIP_GRAD_DERIVED_MIN_ROWS", "0")
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=96)
    exp_op = opts.unary_operators.index("exp") + 1
    extra = [sr.Node(3, sr.Node(exp_op, sr.Node(feature=2)), sr.Node(val=1.5)),
             sr.Node(1, sr.Node(exp_op, sr.Node(feature=1)), sr.Node(val=0.25))]
    en, eo = sr.flatten(extra, opts, dtype)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    X = np.array(X, copy=True)
    X[1, 17] = 1000.0 if dtype == np.float64 else 100.0  # exp(x1) overflows in one row
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    res = {}
    for d in ("0", "1"):
        monkeypatch.setenv("SRHIP_GRAD_DERIVED", d)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, loss)
        idx = np.random.default_rng(2).integers(0, X.shape[1], 1500)  # a batched (gathered) view
        bl, bg, bok = prog.eval_loss_grad(ds, loss, idx=idx)
        monkeypatch.setenv("SRHIP_GRAD_VALUE_ONLY", "1")
        vl, _, vok = prog.eval_loss_grad(ds, loss)
        monkeypatch.delenv("SRHIP_GRAD_VALUE_ONLY")
        out, imp, fc = prog.optimize_constants(ds, loss, iterations=8, nrestarts=1, seed=3)
        consts = np.concatenate(prog.get_constants())
        pred, pgrad, pok = prog.eval_grad_predict(ds, variable=True)
        flat = lambda a: np.concatenate([np.ravel(x) for x in a])  # noqa: E731
        res[d] = [np.asarray(l, np.float64), flat(g), np.asarray(ok), np.asarray(vl, np.float64), np.asarray(vok),
                  np.asarray(out, np.float64), imp, fc, consts, np.asarray(pred), flat(pgrad), np.asarray(pok),
                  np.asarray(bl, np.float64), flat(bg), np.asarray(bok)]
        prog.close()
    assert not res["1"][2][-2] and res["1"][2][-1], res["1"][2][-2:]
    assert res["1"][6].sum() > 5
    for i, (u, v) in enumerate(zip(res["0"], res["1"])):
        assert _bits_equal(u, v), i


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_uniform_constant_subtrees_are_exact(ctx, dtype, monkeypatch):
    """Operators whose operands are constant subtrees (cos(c), c1 / c2, ...) are evaluated once per lane
    and copied to the lane's rows (UN_UNIFORM_FLAG); losses, gradients, did_succeed, value-only
    passes and an optimize_constants run are bitwise those of the per-row evaluation
    (SRHIP_GRAD_UNIFORM=0)."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=80, max_size=24)
    cos_op = opts.unary_operators.index("cos") + 1
    extra = [sr.Node(3, sr.Node(cos_op, sr.Node(val=0.7)), sr.Node(feature=1)),            # cos(c) * x0
             sr.Node(1, sr.Node(4, sr.Node(val=2.0), sr.Node(val=3.0)), sr.Node(feature=2)),  # c1 / c2 + x1
             sr.Node(3, sr.Node(1, sr.Node(val=1e30), sr.Node(val=1e30)), sr.Node(feature=3))]
    en, eo = sr.flatten(extra, opts, dtype)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    res = {}
    for u in ("0", "1"):
        monkeypatch.setenv("SRHIP_GRAD_UNIFORM", u)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, loss)
        monkeypatch.setenv("SRHIP_GRAD_VALUE_ONLY", "1")
        vl, _, vok = prog.eval_loss_grad(ds, loss)
        monkeypatch.delenv("SRHIP_GRAD_VALUE_ONLY")
        out, imp, fc = prog.optimize_constants(ds, loss, iterations=8, nrestarts=1, seed=3)
        flat = lambda a: np.concatenate([np.ravel(x) for x in a])  # noqa: E731
        res[u] = [np.asarray(l, np.float64), flat(g), np.asarray(ok), np.asarray(vl, np.float64), np.asarray(vok),
                  np.asarray(out, np.float64), imp, fc, np.concatenate(prog.get_constants())]
        prog.close()
    assert res["1"][6].sum() > 5
    for i, (a, b) in enumerate(zip(res["0"], res["1"])):
        assert _bits_equal(a, b), i


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_gradient_program_forms_exact_on_domain_operators(ctx, dtype, monkeypatch):
    """Derived-view columns and once-per-lane constant subtrees over operators with restricted domains
    (safe log / sqrt return NaN below 0, tanh, sin): losses, gradients and did_succeed of a full and
    a value-only pass are bitwise those of the plain per-row program (SRHIP_GRAD_DERIVED=0,
    SRHIP_GRAD_UNIFORM=0), NaN columns and infinite derivative factors included."""
    sr = _sr()
    monkeypatch.setenv("SRHIP_GRAD_DERIVED_MIN_ROWS", "0")
    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("log", "sqrt", "sin", "tanh", "exp"))
    trees = sr.random_population(120, opts, 3, dtype, seed=23, max_size=22)
    nodes, offs = sr.flatten(trees, opts, dtype)
    rng = np.random.default_rng(24)
    X = (rng.standard_normal((3, 2500)) * 2.0).astype(dtype)
    X[0, :8] = 0.0  # log(0) = -Inf, sqrt'(0) = Inf
    y = (np.sin(X[1]) + 0.5 * X[2]).astype(dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    res = {}
    for form in ("plain", "fast"):
        monkeypatch.setenv("SRHIP_GRAD_DERIVED", "0" if form == "plain" else "1")
        monkeypatch.setenv("SRHIP_GRAD_UNIFORM", "0" if form == "plain" else "1")
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, loss)
        monkeypatch.setenv("SRHIP_GRAD_VALUE_ONLY", "1")
        vl, _, vok = prog.eval_loss_grad(ds, loss)
        monkeypatch.delenv("SRHIP_GRAD_VALUE_ONLY")
        flat = lambda a: np.concatenate([np.ravel(x) for x in a])  # noqa: E731
        res[form] = [np.asarray(l, np.float64), flat(g), np.asarray(ok), np.asarray(vl, np.float64), np.asarray(vok)]
        prog.close()
    assert res["fast"][2].sum() > 10 and (~res["fast"][2]).sum() > 3
    for i, (a, b) in enumerate(zip(res["plain"], res["fast"])):
        assert _bits_equal(a, b), i


def test_derived_view_is_exact_weighted(ctx, monkeypatch):
    """The derived view over a weighted Float64 dataset, whole and batched (gathered rows and weights):
    losses, gradients, did_succeed and an optimize_constants run bitwise those of the per-row
    operators."""
    sr = _sr()
    monkeypatch.setenv("SRHIP_GRAD_DERIVED_MIN_ROWS", "0")
    dtype = np.float64
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=72)
    w = np.random.default_rng(9).uniform(0.1, 2.0, X.shape[1]).astype(dtype)
    ds = sr.DeviceDataset(ctx, X, y, w)
    loss = sr.L2DistLoss()
    idx = np.random.default_rng(10).integers(0, X.shape[1], 1200)
    res = {}
    for d in ("0", "1"):
        monkeypatch.setenv("SRHIP_GRAD_DERIVED", d)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, loss)
        bl, bg, bok = prog.eval_loss_grad(ds, loss, idx=idx)
        out, imp, fc = prog.optimize_constants(ds, loss, iterations=8, nrestarts=1, seed=5)
        flat = lambda a: np.concatenate([np.ravel(x) for x in a])  # noqa: E731
        res[d] = [np.asarray(l), flat(g), np.asarray(ok), np.asarray(bl), flat(bg), np.asarray(bok),
                  np.asarray(out), imp, fc, np.concatenate(prog.get_constants())]
        prog.close()
    assert res["1"][7].sum() > 5
    for i, (a, b) in enumerate(zip(res["0"], res["1"])):
        assert _bits_equal(a, b), i


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_grad_superinstructions_are_exact(ctx, dtype, monkeypatch):
    """The gradient program's superinstructions (round 6: leaf-leaf FF / FC / CF forms with the constant's
    index in the upper half, pushes fused with the plain leaf load after them) return bitwise the plain
    forms' results (SRHIP_GRAD_NO_SUPER=1): losses, gradients, did_succeed of a full and a value-only pass,
    per-row derivatives with respect to the constants and the features, and an optimize_constants run
    (speculative slots patch the fused instructions' constants), near-overflow trees included (the
    precise pass runs the gradient program with operator ordinals counted, not read).  The default build
    emits none of them (srhip_isa.h SRHIP_GRAD_SUPER_LEVEL, measured slower); a build with
    EXTRA=-DSRHIP_GRAD_SUPER_LEVEL=2 runs the comparison proper."""
    sr = _sr()
    opts, _, nodes, offs, X, y = _problem(sr, dtype, ntrees=96, max_size=24)
    big = 3.0e37 if dtype == np.float32 else 1.0e306
    x0, x1, x2 = (sr.Node(feature=i) for i in (1, 2, 3))
    c = lambda v: sr.Node(val=v)  # noqa: E731
    extra = [sr.Node(3, sr.Node(1, x0, c(0.5)), sr.Node(2, c(1.5), x1)),         # (x0 + c) * (c - x1)
             sr.Node(1, sr.Node(3, x0, x1), sr.Node(4, x2, c(3.0))),              # x0 * x1 + x2 / c
             sr.Node(3, x0, c(big)), sr.Node(1, sr.Node(3, x1, c(big)), c(1.0))]  # near-overflow sums
    en, eo = sr.flatten(extra, opts, dtype)
    nodes = np.concatenate([nodes, en])
    offs = np.concatenate([offs, eo[1:] + offs[-1]])
    ds = sr.DeviceDataset(ctx, X, y)
    loss = sr.L2DistLoss()
    flat = lambda a: np.concatenate([np.ravel(x) for x in a])  # noqa: E731
    res = {}
    for ns in ("1", "0"):
        monkeypatch.setenv("SRHIP_GRAD_NO_SUPER", ns)
        prog = sr.Program(ctx, nodes, offs, opts, dtype)
        l, g, ok = prog.eval_loss_grad(ds, loss)
        monkeypatch.setenv("SRHIP_GRAD_VALUE_ONLY", "1")
        vl, _, vok = prog.eval_loss_grad(ds, loss)
        monkeypatch.delenv("SRHIP_GRAD_VALUE_ONLY")
        pc, gc, okc = prog.eval_grad_predict(ds, variable=False)
        pf, gf, okf = prog.eval_grad_predict(ds, variable=True)
        out, imp, fc = prog.optimize_constants(ds, loss, iterations=8, nrestarts=1, seed=3)
        res[ns] = [np.asarray(l, np.float64), flat(g), np.asarray(ok), np.asarray(vl, np.float64), np.asarray(vok),
                   pc, flat(gc), okc, pf, flat(gf), okf,
                   np.asarray(out, np.float64), imp, fc, np.concatenate(prog.get_constants())]
        prog.close()
    assert res["0"][12].sum() > 5
    for i, (a, b) in enumerate(zip(res["1"], res["0"])):
        assert _bits_equal(a, b), i
