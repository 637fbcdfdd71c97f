"""The reference's hot-path API, backed by libsrhip:

  eval_tree_array(tree, X, options)        src/InterfaceDynamicExpressions.jl:56-63
  eval_diff_tree_array / eval_grad_tree_array   src/InterfaceDynamicExpressions.jl:90-95,118-124
  eval_loss(tree, dataset, options; ...)   src/LossFunctions.jl:97-112 (-> _eval_loss :45-75)
  eval_loss_batched / batch_sample         src/LossFunctions.jl:114-127
  loss_to_score                            src/LossFunctions.jl:138-158
  score_func / score_func_batched          src/LossFunctions.jl:161-194
  update_baseline_loss!                    src/LossFunctions.jl:201-215
  compute_complexity                       src/Complexity.jl:17-50

plus the batched entry points the device is built for (one launch per population):
  eval_tree_array_batch, eval_loss_batch, score_func_batch.
Same argument meaning and error behaviour as the reference; there is no CPU fallback.
"""
from __future__ import annotations

import inspect

import numpy as np

from .dataset import Dataset
from .device import Program, get_context
from .losses import is_device_loss
from .node import Node, count_nodes, flatten


def _ctx(options):
    return get_context(getattr(options, "device", 0))


def _as_trees(trees):
    if isinstance(trees, Node):
        return [trees]
    return [t.tree if hasattr(t, "tree") else t for t in trees]


def compile_trees(trees, options, dtype) -> Program:
    nodes, offsets = flatten(_as_trees(trees), options, dtype)
    return Program(_ctx(options), nodes, offsets, options, dtype)


# ---- eval_tree_array ---------------------------------------------------------------------------
def eval_tree_array_batch(trees, X, options, idx=None):
    """Evaluate many trees over X: returns (out[ntrees, n] in T, ok[ntrees])."""
    ctx = _ctx(options)
    if isinstance(X, Dataset):
        ds = X
    else:
        ds = Dataset(np.asarray(X))
    prog = compile_trees(trees, options, ds.X.dtype)
    try:
        return prog.eval_predict(ds.device(ctx), idx)
    finally:
        prog.close()


def eval_tree_array(tree, X, options, **kws):
    """(output::Vector{T}, complete::Bool) for one tree (src/InterfaceDynamicExpressions.jl:56-63)."""
    out, ok = eval_tree_array_batch([tree], X, options)
    return out[0], bool(ok[0])


def eval_grad_tree_array(tree, X, options, variable: bool = False, **kws):
    """(output, gradient, complete) -- src/InterfaceDynamicExpressions.jl:118-124.  gradient is
    [nfeatures, n] (variable=True: d output / d x_f) or [nconst, n] (variable=False: d output / d c in
    get_constants order); forward-mode dual numbers on the device."""
    ds = X if isinstance(X, Dataset) else Dataset(np.asarray(X))
    prog = compile_trees([tree], options, ds.X.dtype)
    try:
        out, grads, ok = prog.eval_grad_predict(ds.device(_ctx(options)), variable=variable)
    finally:
        prog.close()
    return out[0], grads[0], bool(ok[0])


def eval_diff_tree_array(tree, X, options, direction: int):
    """(output, d output / d x_direction, complete) -- src/InterfaceDynamicExpressions.jl:90-95
    (direction is 1-based, as in Julia)."""
    ds = X if isinstance(X, Dataset) else Dataset(np.asarray(X))
    if not 1 <= int(direction) <= ds.nfeatures:
        raise ValueError(f"direction {direction} out of range 1..{ds.nfeatures}")
    prog = compile_trees([tree], options, ds.X.dtype)
    try:
        out, grads, ok = prog.eval_grad_predict(ds.device(_ctx(options)), variable=True, direction=int(direction))
    finally:
        prog.close()
    return out[0], grads[0][0], bool(ok[0])


# ---- losses ------------------------------------------------------------------------------------
def _host_elementwise_loss(pred, y, w, loss):
    """User-defined elementwise loss (a Julia function in the reference): evaluated on the host
    over device predictions, with _loss / _weighted_loss's normalisation (src/LossFunctions.jl:13-33)."""
    T = pred.dtype.type
    if w is None:
        vals = np.array([loss(pred[i], y[i]) for i in range(len(pred))], dtype=pred.dtype)
        return float(np.sum(vals.astype(np.float64)) / len(pred))
    vals = np.array([loss(pred[i], y[i], w[i]) for i in range(len(pred))], dtype=pred.dtype)
    return float(np.sum(vals.astype(np.float64)) / np.sum(w.astype(np.float64)))


def dimensional_regularization(tree, dataset: Dataset, options):
    """src/LossFunctions.jl:217-227: 0 unless the tree violates the dataset's units (checked on row 1,
    srhip.units), then options.dimensional_constraint_penalty (default 1000)."""
    L = dataset.loss_type.type
    if not dataset.has_units():
        return L(0)
    from .units import violates_dimensional_constraints

    if not violates_dimensional_constraints(tree, dataset, options):
        return L(0)
    pen = options.dimensional_constraint_penalty
    return L(1000) if pen is None else L(pen)


def eval_loss_batch(trees, dataset: Dataset, options, regularization: bool = True, idx=None):
    """_eval_loss for every tree in one device launch: returns (loss[ntrees] float64, ok[ntrees]).

    Loss is +Inf where did_succeed is false (L(Inf), src/LossFunctions.jl:55-57); with units and
    regularization, dimensional_regularization is added to the finite losses (:70-72)."""
    trees = _as_trees(trees)
    if options.loss_function is not None:
        out = np.array([eval_loss(t, dataset, options, regularization=regularization, idx=idx) for t in trees],
                       dtype=np.float64)
        return out, np.isfinite(out)
    out, ok = _eval_loss_batch_device(trees, dataset, options, idx)
    if regularization and dataset.has_units():
        # in the loss type L, as _eval_loss adds L(loss) + L(penalty) (src/LossFunctions.jl:70-72)
        L = dataset.loss_type.type
        for t in np.nonzero(ok)[0]:
            out[t] = float(L(out[t]) + dimensional_regularization(trees[t], dataset, options))
    return out, ok


def _eval_loss_batch_device(trees, dataset: Dataset, options, idx):
    ctx = _ctx(options)
    loss = options.elementwise_loss
    prog = compile_trees(trees, options, dataset.X.dtype)
    try:
        if is_device_loss(loss):
            return prog.eval_loss(dataset.device(ctx), loss, idx)
        pred, ok = prog.eval_predict(dataset.device(ctx), idx)
        y = dataset.y if idx is None else dataset.y[np.asarray(idx)]
        w = None if not dataset.weighted else (dataset.weights if idx is None else dataset.weights[np.asarray(idx)])
        out = np.full(len(trees), np.inf)
        for t in range(len(trees)):
            if ok[t]:
                out[t] = _host_elementwise_loss(pred[t], y, w, loss)
        return out, ok
    finally:
        prog.close()


def _evaluator(f, tree, dataset, options, idx):
    """src/LossFunctions.jl:78-94: user loss_function dispatch on whether it accepts idx."""
    try:
        nparams = len(inspect.signature(f).parameters)
    except (TypeError, ValueError):
        nparams = 4
    if nparams >= 4:
        return f(tree, dataset, options, idx)
    if options.batching:
        raise RuntimeError(
            "User-defined loss function must accept batching indices if `options.batching == true`. "
            "For example, `f(tree, dataset, options, idx)`, where `idx` is `nothing` if full dataset is "
            "to be used, and a vector of indices otherwise.")
    return f(tree, dataset, options)


def eval_loss(tree, dataset: Dataset, options, regularization: bool = True, idx=None):
    """src/LossFunctions.jl:97-112. Returns a scalar of the dataset's loss type L."""
    L = dataset.loss_type.type
    if options.loss_function is not None:
        return L(_evaluator(options.loss_function, tree, dataset, options, idx))
    loss, _ = eval_loss_batch([tree], dataset, options, regularization=regularization, idx=idx)
    return L(loss[0])


def batch_sample(dataset: Dataset, options, rng=None):
    """StatsBase.sample(1:n, batch_size; replace=true) (src/LossFunctions.jl:125-127), 0-based."""
    rng = np.random.default_rng() if rng is None else rng
    return rng.integers(0, dataset.n, size=options.batch_size)


def eval_loss_batched(tree, dataset, options, regularization=True, idx=None, rng=None):
    _idx = batch_sample(dataset, options, rng) if idx is None else idx
    return eval_loss(tree, dataset, options, regularization=regularization, idx=_idx)


# ---- complexity / scoring ----------------------------------------------------------------------
def compute_complexity(tree: Node, options) -> int:
    """count_nodes, or the custom complexity mapping (src/Complexity.jl:17-50)."""
    cm = options.complexity_mapping
    if not cm.use:
        return count_nodes(tree)
    total = 0.0
    for n in tree:
        if n.degree == 0:
            if n.constant:
                total += cm.constant_complexity
            else:
                vc = cm.variable_complexity
                total += vc[n.feature - 1] if isinstance(vc, (list, tuple, np.ndarray)) else vc
        elif n.degree == 1:
            total += cm.unaop_complexities[options.unary_index(n.op) - 1]
        else:
            total += cm.binop_complexities[options.binary_index(n.op) - 1]
    return int(round(total))


def loss_to_score(loss, use_baseline, baseline, member, options, complexity=None):
    """src/LossFunctions.jl:138-158."""
    L = type(loss) if isinstance(loss, np.floating) else np.float64
    normalization = baseline if (baseline >= L(0.01) and use_baseline) else L(0.01)
    loss_val = L(loss) / L(normalization)
    size = compute_complexity(member.tree if hasattr(member, "tree") else member, options) \
        if complexity is None else complexity
    parsimony_term = size * options.parsimony
    return L(loss_val + L(parsimony_term))


def score_func(dataset: Dataset, member, options, complexity=None):
    """(score, loss) — src/LossFunctions.jl:161-174."""
    tree = member.tree if hasattr(member, "tree") else member
    result_loss = eval_loss(tree, dataset, options)
    score = loss_to_score(result_loss, dataset.use_baseline, dataset.baseline_loss, member, options, complexity)
    return score, result_loss


def score_func_batched(dataset, member, options, complexity=None, idx=None, rng=None):
    """src/LossFunctions.jl:177-194."""
    tree = member.tree if hasattr(member, "tree") else member
    result_loss = eval_loss_batched(tree, dataset, options, idx=idx, rng=rng)
    score = loss_to_score(result_loss, dataset.use_baseline, dataset.baseline_loss, member, options, complexity)
    return score, result_loss


def score_func_batch(dataset: Dataset, members, options, idx=None):
    """score_func over a whole population in one device launch: (scores, losses) arrays in L."""
    trees = _as_trees(members)
    L = dataset.loss_type.type
    losses, _ = eval_loss_batch(trees, dataset, options, idx=idx)
    losses = losses.astype(dataset.loss_type)
    scores = np.array([loss_to_score(L(l), dataset.use_baseline, dataset.baseline_loss, t, options)
                       for l, t in zip(losses, trees)], dtype=dataset.loss_type)
    return scores, losses


# ---- the batching-mode batch seams (options.batching): one launch per population ----------------
def trees_equal(a: Node, b: Node) -> bool:
    """DynamicExpressions' structural == on nodes (degree, operator, feature, constant value)."""
    if a is b:
        return True
    if a is None or b is None or a.degree != b.degree:
        return False
    if a.degree == 0:
        if a.constant != b.constant:
            return False
        return a.val == b.val if a.constant else a.feature == b.feature
    if a.op != b.op or not trees_equal(a.l, b.l):
        return False
    return a.degree == 1 or trees_equal(a.r, b.r)


class LossCache:
    """s_r_cycle's loss_cache (src/SingleIteration.jl:47-50): per population slot, the tree last
    scored on the cycle's fixed batch and that score."""

    def __init__(self, n: int, L=np.float64):
        self.oid = [None] * n
        self.score = np.zeros(n, dtype=L)


def rescore_population_batched(dataset: Dataset, members, options, idx, cache: LossCache, first_loop: bool):
    """The batched re-score of s_r_cycle (src/SingleIteration.jl:64-82) for a whole population in ONE
    device launch: on the first loop every member, afterwards every member whose tree differs from
    its cache entry, is scored on the fixed batch ``idx`` (score_func_batched on each: eval_loss with
    idx, regularization, loss_to_score with the member's complexity) by a single eval_loss_batch(idx)
    launch; the others keep their cached score.  Returns (scores[n], number of trees evaluated)."""
    members = list(members)
    stale = [i for i, m in enumerate(members)
             if first_loop or cache.oid[i] is None or not trees_equal(cache.oid[i], _tree_of(m))]
    if stale:
        scores, _ = score_func_batch(dataset, [members[i] for i in stale], options, idx=idx)
        for i, sc in zip(stale, scores):
            cache.oid[i] = _tree_of(members[i]).copy()
            cache.score[i] = sc
    return cache.score.copy(), len(stale)


def finalize_scores(dataset: Dataset, members, options) -> float:
    """finalize_scores (src/Population.jl:162-176): with options.batching every member's score and
    loss are recomputed on the full dataset -- here one score_func_batch launch for the population
    (members get .score / .loss).  Returns num_evals (pop.n, or 0 without batching)."""
    members = list(members)
    if not options.batching or not members:
        return 0.0
    scores, losses = score_func_batch(dataset, members, options)
    for m, sc, lo in zip(members, scores, losses):
        m.score, m.loss = sc, lo
    return float(len(members))


def rescore_hall_of_fame(dataset: Dataset, members, exists, options) -> float:
    """_dispatch_s_r_cycle's best_seen re-score (src/SymbolicRegression.jl:1120-1127): with
    options.batching each hall-of-fame entry's score and loss are recomputed on the full dataset --
    one launch over the entries that exist (the reference also re-scores the placeholder entries,
    whose values are never read; num_evals counts every entry as it does)."""
    if not options.batching:
        return 0.0
    live = [m for m, e in zip(members, exists) if e and m is not None]
    if live:
        scores, losses = score_func_batch(dataset, live, options)
        for m, sc, lo in zip(live, scores, losses):
            m.score, m.loss = sc, lo
    return float(len(members))


def _tree_of(member):
    return member.tree if hasattr(member, "tree") else member


def update_baseline_loss(dataset: Dataset, options) -> None:
    """update_baseline_loss! (src/LossFunctions.jl:201-215): loss of the constant tree avg_y."""
    example_tree = Node(val=dataset.avg_y)
    baseline_loss = eval_loss(example_tree, dataset, options)
    if np.isfinite(baseline_loss):
        dataset.baseline_loss = baseline_loss
        dataset.use_baseline = True
    else:
        dataset.baseline_loss = dataset.loss_type.type(1)
        dataset.use_baseline = False


# ---- constant optimisation ---------------------------------------------------------------------
def eval_grad_loss_batch(trees, dataset: Dataset, options, idx=None):
    """Loss and its exact gradient w.r.t. each tree's constants (get_constants order), one launch:
    (loss[T], [grad per tree], ok[T]).  The loss-level counterpart of eval_grad_tree_array
    (src/InterfaceDynamicExpressions.jl:118-124, variable=false)."""
    trees = _as_trees(trees)
    prog = compile_trees(trees, options, dataset.X.dtype)
    try:
        return prog.eval_loss_grad(dataset.device(_ctx(options)), options.elementwise_loss, idx)
    finally:
        prog.close()


def optimize_constants(dataset: Dataset, members, options, rng=None, idx=None):
    """optimize_constants (src/ConstantOptimization.jl:11-81) for one member or a whole list at once.

    Members are PopMember-like objects (``.tree``, ``.loss``, ``.score``, ``.birth``) or bare Nodes.
    Where the optimised constants beat the member's baseline loss, its tree constants are replaced,
    loss and score re-computed on the same rows (:70-78) and its birth renewed (:76).  Returns
    (members, num_evals) like the reference (num_evals summed over the members).

    Built-in distance losses: one batched device call (srhip_optimize_constants: dual-number
    gradients, Newton / BFGS per tree).  With ``options.batching`` every member draws its own
    minibatch (src/ConstantOptimization.jl:14-16), so members are optimised one device call each.
    A user ``loss_function`` (or a Python elementwise loss): host Newton / BFGS with finite
    differences over ``eval_loss`` (srhip.host_optim), whose evaluations run on the device."""
    from .node import get_constants, set_constants
    from .utils import get_birth_order

    single = not isinstance(members, (list, tuple))
    mlist = [members] if single else list(members)
    trees = [m.tree if hasattr(m, "tree") else m for m in mlist]
    rng = np.random.default_rng() if rng is None else rng
    eval_fraction = (options.batch_size / dataset.n) if options.batching else 1.0
    L = dataset.loss_type.type
    if idx is not None or not options.batching:
        groups = [(list(range(len(mlist))), idx)]
    else:
        groups = [([i], batch_sample(dataset, options, rng)) for i in range(len(mlist))]
    num_evals = 0.0
    for members_idx, gidx in groups:
        if options.loss_function is not None or not is_device_loss(options.elementwise_loss):
            results = _optimize_constants_host(dataset, [trees[i] for i in members_idx], options, rng, gidx)
        else:
            seed = int(rng.integers(0, 2**63 - 1))
            prog = compile_trees([trees[i] for i in members_idx], options, dataset.X.dtype)
            try:
                losses, improved, fcalls = prog.optimize_constants(
                    dataset.device(_ctx(options)), options.elementwise_loss, iterations=options.optimizer_iterations,
                    nrestarts=options.optimizer_nrestarts, seed=seed, idx=gidx)
                consts = prog.get_constants()
            finally:
                prog.close()
            results = list(zip(improved, consts, losses, fcalls))
        for i, (ok, c, lo, fc) in zip(members_idx, results):
            num_evals += float(fc) * eval_fraction
            if not ok:
                continue
            set_constants(trees[i], c)
            m = mlist[i]
            if hasattr(m, "tree"):
                if options.loss_function is not None or not is_device_loss(options.elementwise_loss):
                    lo = eval_loss(trees[i], dataset, options, regularization=True, idx=gidx)
                elif dataset.has_units():
                    lo = lo + dimensional_regularization(trees[i], dataset, options)
                m.loss = L(lo)
                m.score = loss_to_score(m.loss, dataset.use_baseline, dataset.baseline_loss, m, options)
                if hasattr(m, "birth"):
                    m.birth = get_birth_order()
    return (mlist[0] if single else mlist), num_evals


def _optimize_constants_host(dataset, trees, options, rng, idx):
    """Host Newton / BFGS with finite differences over eval_loss(regularization=false), per tree:
    [(improved, constants, loss, f_calls)] (src/ConstantOptimization.jl:43-81)."""
    from . import host_optim
    from .node import get_constants, set_constants

    out = []
    for tree in trees:
        x0 = np.asarray(get_constants(tree), dtype=np.float64)
        if len(x0) == 0:
            out.append((False, x0, np.inf, 0))
            continue
        work = tree.copy()

        def objective(c, work=work):
            set_constants(work, c)
            return eval_loss(work, dataset, options, regularization=False, idx=idx)

        x, fx, improved, calls, _ = host_optim.optimize(objective, x0, iterations=options.optimizer_iterations,
                                                        nrestarts=options.optimizer_nrestarts, rng=rng)
        out.append((improved, x, fx, calls + (1 if improved else 0)))
    return out
