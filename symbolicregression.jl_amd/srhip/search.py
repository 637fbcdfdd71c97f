"""The search loop around the hot path: regularized evolution over islands, every score through
the device (SURVEY.md §8(a) A12 scoring call sites, A14 ``s_r_cycle``, A15 migration; §8(f)-1
cross-population request coalescer).

Restated from the reference, file by file:
  * ``s_r_cycle``                      src/SingleIteration.jl:24-98
  * ``optimize_and_simplify_population`` src/SingleIteration.jl:100-127
  * ``reg_evol_cycle``                 src/RegularizedEvolution.jl:13-111
  * ``next_generation`` / ``crossover_generation`` / ``condition_mutation_weights!``
                                       src/Mutate.jl:34-431
  * mutation operators                 src/MutationFunctions.jl:33-318
  * ``MutationWeights`` / ``sample_mutation``  src/MutationWeights.jl:42-66
  * ``best_of_sample`` / ``best_sub_pop``      src/Population.jl:107-187
  * ``RunningSearchStatistics``        src/AdaptiveParsimony.jl:22-97
  * ``HallOfFame`` / ``calculate_pareto_frontier`` / ``update_hall_of_fame!``
                                       src/HallOfFame.jl:30-96, src/SearchUtils.jl:513-531
  * ``check_constraints`` (size, depth, per-operator complexity)  src/CheckConstraints.jl:69-97
  * ``migrate!``                       src/Migration.jl:16-38
  * ``get_cur_maxsize``                src/SearchUtils.jl:458-470
  * the main loop (populations as concurrent tasks, results processed as they complete, HoF /
    frequency / migration updates, re-dispatch)  src/SymbolicRegression.jl:870-1000, 1088-1129
  * ``simplify_tree!`` / ``combine_operators``: DynamicExpressions v0.16 (external, absent from
    the container; restated: constant folding of all-constant operator nodes, and merging of
    constants through nested + and *) — parity unpinned.

The reference scores ONE tree per mutation from every population task concurrently; here the
island threads call :class:`srhip.Coalescer` (a native batcher in libsrhip), which turns the
concurrent single-tree requests into one device launch.  NumPy Generators replace Julia's RNG:
searches are statistically, not bit-, equivalent to the reference; with ``deterministic=True``
a search is reproducible run to run (islands iterate in lock step, fixed processing order).
"""
from __future__ import annotations

import functools
import itertools
import math
import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from .api import (compute_complexity, dimensional_regularization, loss_to_score, optimize_constants,
                  update_baseline_loss)
from .dataset import Dataset
from .node import Node, count_constants, count_depth, count_nodes, flatten, string_tree
from .random_trees import make_random_leaf

MAX_DEGREE = 2

# ---- search options (src/Options.jl:379-440 defaults) -------------------------------------------


@dataclass
class MutationWeights:
    """src/MutationWeights.jl:42-55 (form/break_connection only apply to GraphNode: always 0 here)."""
    mutate_constant: float = 0.048
    mutate_operator: float = 0.47
    swap_operands: float = 0.1
    add_node: float = 0.79
    insert_node: float = 5.1
    delete_node: float = 1.7
    simplify: float = 0.0020
    randomize: float = 0.00023
    do_nothing: float = 0.21
    optimize: float = 0.0

    def copy(self) -> "MutationWeights":
        return MutationWeights(**self.__dict__)


MUTATIONS = tuple(MutationWeights.__dataclass_fields__)

SEARCH_DEFAULTS = dict(
    populations=15, population_size=33, ncycles_per_iteration=550, tournament_selection_n=12,
    tournament_selection_p=0.86, topn=12, alpha=0.1, perturbation_factor=0.076, annealing=False,
    crossover_probability=0.066, warmup_maxsize_by=0.0, use_frequency=True, use_frequency_in_tournament=True,
    adaptive_parsimony_scaling=20.0, fraction_replaced=0.00036, fraction_replaced_hof=0.035,
    probability_negate_constant=0.01, maxdepth=None, migration=True, hof_migration=True, should_simplify=True,
    should_optimize_constants=True, skip_mutation_failures=True, bin_constraints=None, una_constraints=None,
    mutation_weights=None,
)


def search_option(options, name):
    if hasattr(options, name):
        return getattr(options, name)
    return options.unused.get(name, SEARCH_DEFAULTS[name])


@functools.lru_cache(maxsize=64)
def _tournament_cdf(n: int, p: float) -> tuple:
    w = tournament_selection_weights(n, p)
    return tuple(np.cumsum(w))


def tournament_selection_weights(n: int, p: float) -> np.ndarray:
    """src/Options.jl: weights p (1-p)^(k-1), k = 1..n, normalised."""
    w = np.array([p * (1 - p) ** k for k in range(n)])
    return w / w.sum()


def _draw(cdf, u: float) -> int:
    """Index k with cdf[k-1] <= u * cdf[-1] < cdf[k] (inverse-CDF draw on a short list)."""
    t = u * cdf[-1]
    for k, c in enumerate(cdf):
        if t < c:
            return k
    return len(cdf) - 1


# ---- members, populations, statistics ------------------------------------------------------------
from .utils import get_birth_order  # noqa: E402  (shared with api.optimize_constants)


@dataclass
class PopMember:
    """src/PopMember.jl:7-16."""
    tree: Node
    score: float
    loss: float
    birth: int = field(default_factory=get_birth_order)
    complexity: int = -1
    ref: int = -1
    parent: int = -1

    def copy(self) -> "PopMember":
        return PopMember(self.tree.copy(), self.score, self.loss, self.birth, self.complexity, self.ref, self.parent)

    def get_complexity(self, options) -> int:
        """compute_complexity cached on the member, as the reference caches it in PopMember
        (src/PopMember.jl:7-16, recompute_complexity!); reset to -1 whenever ``tree`` changes."""
        if self.complexity < 0:
            self.complexity = compute_complexity(self.tree, options)
        return self.complexity


class RunningSearchStatistics:
    """src/AdaptiveParsimony.jl:22-97."""

    def __init__(self, options, window_size: int = 100000):
        size = options.maxsize + MAX_DEGREE
        self.window_size = window_size
        self.frequencies = np.ones(size)
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()

    def copy(self):
        c = RunningSearchStatistics.__new__(RunningSearchStatistics)
        c.window_size, c.frequencies, c.normalized_frequencies = (
            self.window_size, self.frequencies.copy(), self.normalized_frequencies.copy())
        return c

    def update_frequencies(self, size: int) -> None:
        if 0 < size <= len(self.frequencies):
            self.frequencies[size - 1] += 1

    def move_window(self) -> None:
        smallest = 1.0
        f = self.frequencies
        total = f.sum()
        if total <= self.window_size:
            return
        diff = total - self.window_size
        for _ in range(1000):
            if diff <= 0:
                break
            sel = f > smallest
            nrem = int(sel.sum())
            if nrem == 0:
                break
            amount = min(diff / nrem, f[sel].min() - smallest)
            f[sel] -= amount
            tot = amount * nrem
            diff -= tot
            if tot < 1e-6:
                break

    def normalize_frequencies(self) -> None:
        self.normalized_frequencies = self.frequencies / self.frequencies.sum()


class HallOfFame:
    """src/HallOfFame.jl:30-60: best member per complexity."""

    def __init__(self, options):
        n = options.maxsize + MAX_DEGREE
        self.members = [None] * n
        self.exists = [False] * n

    def update(self, members, options) -> None:
        """update_hall_of_fame! (src/SearchUtils.jl:513-531)."""
        for m in members:
            size = m.get_complexity(options)
            if not (0 < size < options.maxsize + MAX_DEGREE):
                continue
            if not self.exists[size - 1] or m.score < self.members[size - 1].score:
                self.members[size - 1] = m.copy()
                self.exists[size - 1] = True

    def pareto_frontier(self):
        """calculate_pareto_frontier (src/HallOfFame.jl:73-96)."""
        dominating = []
        for size, m in enumerate(self.members):
            if not self.exists[size]:
                continue
            if all(not self.exists[i] or m.loss < self.members[i].loss for i in range(size)):
                dominating.append(m.copy())
        return dominating


# ---- tree sampling and mutation operators (src/MutationFunctions.jl) ---------------------------
def _sample(tree: Node, rng, pred=None):
    """rand(NodeSampler(; tree, filter)): uniform over the (filtered) nodes."""
    nodes = [n for n in tree if pred is None or pred(n)]
    return nodes[int(rng.integers(0, len(nodes)))] if nodes else None


def swap_operands(tree, rng):
    node = _sample(tree, rng, lambda t: t.degree == 2)
    if node is not None:
        node.l, node.r = node.r, node.l
    return tree


def mutate_operator(tree, options, rng):
    node = _sample(tree, rng, lambda t: t.degree != 0)
    if node is None:
        return tree
    node.op = int(rng.integers(1, (options.nuna if node.degree == 1 else options.nbin) + 1))
    return tree


def mutate_constant(tree, temperature, options, dtype, rng):
    """src/MutationFunctions.jl:63-92 (factor in T, negation with probability_negate_constant)."""
    node = _sample(tree, rng, lambda t: t.degree == 0 and t.constant)
    if node is None:
        return tree
    T = np.dtype(dtype).type
    bottom = 0.1
    max_change = search_option(options, "perturbation_factor") * temperature + 1 + bottom
    factor = T(max_change ** T(rng.random()))
    v = T(node.val)
    v = v * factor if rng.random() < 0.5 else v / factor
    if rng.random() > search_option(options, "probability_negate_constant"):
        v = v * T(-1)
    node.val = float(v)
    return tree


def _new_op(options, nfeatures, dtype, rng, left=None, make_bin=None):
    if make_bin is None:
        make_bin = rng.random() < options.nbin / (options.nuna + options.nbin)
    if make_bin:
        op = int(rng.integers(1, options.nbin + 1))
        l = left if left is not None else make_random_leaf(nfeatures, dtype, rng)
        return Node(op, l, make_random_leaf(nfeatures, dtype, rng))
    op = int(rng.integers(1, options.nuna + 1))
    return Node(op, left if left is not None else make_random_leaf(nfeatures, dtype, rng))


def append_random_op(tree, options, nfeatures, dtype, rng, make_bin=None):
    node = _sample(tree, rng, lambda t: t.degree == 0)
    node.set_node(_new_op(options, nfeatures, dtype, rng, make_bin=make_bin))
    return tree


def insert_random_op(tree, options, nfeatures, dtype, rng):
    node = _sample(tree, rng)
    make_bin = rng.random() < options.nbin / (options.nuna + options.nbin)
    node.set_node(_new_op(options, nfeatures, dtype, rng, left=node.copy(), make_bin=make_bin))
    return tree


def prepend_random_op(tree, options, nfeatures, dtype, rng):
    make_bin = rng.random() < options.nbin / (options.nuna + options.nbin)
    tree.set_node(_new_op(options, nfeatures, dtype, rng, left=tree.copy(), make_bin=make_bin))
    return tree


def random_node_and_parent(tree, rng):
    if tree.degree == 0:
        return tree, tree, "n"
    parent = _sample(tree, rng, lambda t: t.degree != 0)
    if parent.degree == 1 or rng.random() < 0.5:
        return parent.l, parent, "l"
    return parent.r, parent, "r"


def delete_random_op(tree, options, nfeatures, dtype, rng):
    node, parent, side = random_node_and_parent(tree, rng)
    isroot = side == "n"
    if node.degree == 0:
        node.set_node(make_random_leaf(nfeatures, dtype, rng))
        return tree
    child = node.l if (node.degree == 1 or rng.random() < 0.5) else node.r
    if isroot:
        return child
    if side == "l":
        parent.l = child
    else:
        parent.r = child
    return tree


def gen_random_tree(length, options, nfeatures, dtype, rng):
    """src/MutationFunctions.jl:227-240."""
    tree = Node(val=1.0)
    for _ in range(length):
        tree = append_random_op(tree, options, nfeatures, dtype, rng)
    return tree


def gen_random_tree_fixed_size(node_count, options, nfeatures, dtype, rng):
    from .random_trees import gen_random_tree_fixed_size as g

    return g(node_count, options, nfeatures, dtype, rng)


def crossover_trees(tree1, tree2, rng):
    """src/MutationFunctions.jl:271-303."""
    tree1, tree2 = tree1.copy(), tree2.copy()
    node1, parent1, side1 = random_node_and_parent(tree1, rng)
    node2, parent2, side2 = random_node_and_parent(tree2, rng)
    node1 = node1.copy()
    if side1 == "l":
        parent1.l = node2.copy()
    elif side1 == "r":
        parent1.r = node2.copy()
    else:
        tree1 = node2.copy()
    if side2 == "l":
        parent2.l = node1
    elif side2 == "r":
        parent2.r = node1
    else:
        tree2 = node1
    return tree1, tree2


# ---- simplification (DynamicExpressions v0.16 simplify_tree! / combine_operators, restated) ------
def _fold(name, vals, dtype):
    from .operators import scalar_op

    with np.errstate(all="ignore"):
        out = scalar_op(name, [np.dtype(dtype).type(v) for v in vals])
    return float(out) if np.isfinite(out) else None


def simplify_tree(tree, options, dtype):
    """Operator nodes whose children are all (finite) constants become the constant result
    (kept only if finite), bottom-up."""
    if tree.degree == 0:
        return tree
    tree.l = simplify_tree(tree.l, options, dtype)
    if tree.degree == 2:
        tree.r = simplify_tree(tree.r, options, dtype)
    kids = [tree.l] if tree.degree == 1 else [tree.l, tree.r]
    if all(k.degree == 0 and k.constant and math.isfinite(k.val) for k in kids):
        names = options.unary_operators if tree.degree == 1 else options.binary_operators
        name = names[(options.unary_index(tree.op) if tree.degree == 1 else options.binary_index(tree.op)) - 1]
        v = _fold(name, [k.val for k in kids], dtype)
        if v is not None:
            return Node(val=v)
    return tree


def combine_operators(tree, options, dtype):
    """Merge constants through nested + and *: (c1 op (c2 op x)) -> ((c1 op c2) op x) for
    op in {+, *} (either operand order), bottom-up."""
    if tree.degree == 0:
        return tree
    tree.l = combine_operators(tree.l, options, dtype)
    if tree.degree == 2:
        tree.r = combine_operators(tree.r, options, dtype)
    if tree.degree != 2:
        return tree
    name = options.binary_operators[options.binary_index(tree.op) - 1]
    if name not in ("+", "*"):
        return tree
    is_c = lambda n: n.degree == 0 and n.constant  # noqa: E731
    for c, other in ((tree.l, tree.r), (tree.r, tree.l)):
        if not is_c(c) or other.degree != 2:
            continue
        if options.binary_operators[options.binary_index(other.op) - 1] != name:
            continue
        for c2, x in ((other.l, other.r), (other.r, other.l)):
            if is_c(c2):
                v = _fold(name, [c.val, c2.val], dtype)
                if v is None:
                    return tree
                return Node(tree.op, Node(val=v), x)
    return tree


# ---- constraints (src/CheckConstraints.jl) --------------------------------------------------------
def check_constraints(tree, options, maxsize, cursize=None) -> bool:
    size = compute_complexity(tree, options) if cursize is None else cursize
    if size > maxsize:
        return False
    maxdepth = search_option(options, "maxdepth") or options.maxsize
    if count_depth(tree) > maxdepth:
        return False
    bc = search_option(options, "bin_constraints")
    uc = search_option(options, "una_constraints")
    if bc or uc:
        for n in tree:
            if n.degree == 2 and bc:
                cons = bc[options.binary_index(n.op) - 1]
                if cons[0] > -1 and compute_complexity(n.l, options) > cons[0]:
                    return False
                if cons[1] > -1 and compute_complexity(n.r, options) > cons[1]:
                    return False
            elif n.degree == 1 and uc:
                cons = uc[options.unary_index(n.op) - 1]
                if cons > -1 and compute_complexity(n.l, options) > cons:
                    return False
    return True


# ---- scoring through the device ----------------------------------------------------------------
class DeviceScorer:
    """score_func (src/LossFunctions.jl:161-174) for one tree at a time, served by the native
    coalescer so concurrent islands share device launches."""

    def __init__(self, dataset: Dataset, options, nclients: int = 0, max_batch: int = 256, max_wait_us=None,
                 ctx=None, device_dataset=None):
        """``ctx`` / ``device_dataset``: score on an existing context and resident dataset (a
        :multiprocessing worker's, see task_island_iteration) instead of a new context and upload."""
        import os

        from .device import Coalescer, Context

        # flush as soon as the worker is free (requests that arrive during a flush form the next
        # batch): with the ~35 us flush path, C1 1.55-1.64e7 node-row evals/s at 0 us against
        # 0.9-1.1e7 at 50 us (same box); SRHIP_COALESCE_WAIT_US overrides (tuning)
        if max_wait_us is None:
            max_wait_us = int(os.environ.get("SRHIP_COALESCE_WAIT_US", "0"))
        self.dataset, self.options = dataset, options
        self._own_ctx = ctx is None
        self.ctx = Context(options.device) if ctx is None else ctx
        self.ds = dataset.device(self.ctx) if device_dataset is None else device_dataset
        self.coalescer = Coalescer(self.ctx, self.ds, options, options.elementwise_loss, max_batch=max_batch,
                                   max_wait_us=max_wait_us, nclients=nclients)
        self.L = dataset.loss_type.type
        self.dtype = dataset.X.dtype
        self._lock = threading.Lock()
        self.trees_scored = 0
        self.node_rows = 0

    def score(self, tree, complexity=None, idx=None):
        nodes, _ = flatten([tree], self.options, self.dtype)
        loss, ok = self.coalescer.score_loss(nodes, idx)
        with self._lock:  # work counters (bench: node-row evaluations)
            self.trees_scored += 1
            self.node_rows += len(nodes) * (self.dataset.n if idx is None else len(idx))
        loss = self.L(loss) if ok else self.L(np.inf)
        if ok and self.dataset.has_units():
            # score_func -> eval_loss(regularization=true) adds the units penalty to a finite loss
            # (src/LossFunctions.jl:70-71), as eval_loss / eval_loss_batch do
            loss = self.L(loss + dimensional_regularization(tree, self.dataset, self.options))
        score = loss_to_score(loss, self.dataset.use_baseline, self.dataset.baseline_loss, tree, self.options,
                              complexity)
        return score, loss

    def close(self):
        self.coalescer.close()
        if self._own_ctx:
            self.dataset.release_device(self.ctx)
            self.ctx.close()


# ---- one mutation / crossover (src/Mutate.jl) ----------------------------------------------------
def condition_mutation_weights(w: MutationWeights, member: PopMember, options, curmaxsize) -> None:
    """src/Mutate.jl:34-76."""
    tree = member.tree
    if tree.degree == 0:
        w.mutate_operator = w.swap_operands = w.delete_node = w.simplify = 0.0
        if not tree.constant:
            w.optimize = 0.0
            w.mutate_constant = 0.0
        return
    if not any(n.degree == 2 for n in tree):
        w.swap_operands = 0.0
    w.mutate_constant *= min(8, count_constants(tree)) / 8.0
    if compute_complexity(tree, options) >= curmaxsize:
        w.add_node = 0.0
        w.insert_node = 0.0
    if not search_option(options, "should_simplify"):
        w.simplify = 0.0


def sample_mutation(w: MutationWeights, rng) -> str:
    cdf = list(itertools.accumulate(getattr(w, k) for k in MUTATIONS))
    return MUTATIONS[_draw(cdf, rng.random())]


class Island:
    """One population and its evolution state (the body of a reference population task)."""

    def __init__(self, k, dataset, options, scorer, rng, dtype):
        self.k, self.dataset, self.options, self.scorer, self.rng, self.dtype = k, dataset, options, scorer, rng, dtype
        self.nfeatures = dataset.nfeatures
        self.num_evals = 0.0

    # src/Mutate.jl:78-346
    def next_generation(self, member, temperature, curmaxsize, stats):
        o, rng = self.options, self.rng
        before_score, before_loss = member.score, member.loss
        w = (search_option(o, "mutation_weights") or MutationWeights()).copy()
        condition_mutation_weights(w, member, o, curmaxsize)
        choice = sample_mutation(w, rng)
        successful = False
        attempts = 0
        tree = None
        while not successful and attempts < 10:
            tree = member.tree.copy()
            successful = True
            if choice == "mutate_constant":
                tree = mutate_constant(tree, temperature, o, self.dtype, rng)
            elif choice == "mutate_operator":
                tree = mutate_operator(tree, o, rng)
            elif choice == "swap_operands":
                tree = swap_operands(tree, rng)
            elif choice == "add_node":
                if rng.random() < 0.5:
                    tree = append_random_op(tree, o, self.nfeatures, self.dtype, rng)
                else:
                    tree = prepend_random_op(tree, o, self.nfeatures, self.dtype, rng)
            elif choice == "insert_node":
                tree = insert_random_op(tree, o, self.nfeatures, self.dtype, rng)
            elif choice == "delete_node":
                tree = delete_random_op(tree, o, self.nfeatures, self.dtype, rng)
            elif choice == "simplify":
                tree = combine_operators(simplify_tree(tree, o, self.dtype), o, self.dtype)
                return PopMember(tree, before_score, before_loss, parent=member.ref), True
            elif choice == "randomize":
                size = int(rng.integers(1, curmaxsize + 1))
                tree = gen_random_tree_fixed_size(size, o, self.nfeatures, self.dtype, rng)
            elif choice == "optimize":
                cur = PopMember(tree, before_score, before_loss, parent=member.ref)
                cur, ne = self._optimizer()(self.dataset, cur, o, rng=rng)
                self.num_evals += ne
                return cur, True
            elif choice == "do_nothing":
                return PopMember(tree, before_score, before_loss, parent=member.ref), True
            successful = successful and check_constraints(tree, o, curmaxsize)
            attempts += 1
        if not successful:
            return PopMember(member.tree.copy(), before_score, before_loss, complexity=member.complexity,
                             parent=member.ref), False
        after_score, after_loss = self.scorer.score(tree)
        self.num_evals += 1
        if math.isnan(after_score):
            return PopMember(member.tree.copy(), before_score, before_loss, complexity=member.complexity,
                             parent=member.ref), False
        prob = 1.0
        if search_option(o, "annealing"):
            delta = after_score - before_score
            prob *= math.exp(-delta / (temperature * search_option(o, "alpha")))
        if search_option(o, "use_frequency"):
            old_size = member.get_complexity(o)
            new_size = compute_complexity(tree, o)
            nf = stats.normalized_frequencies
            old_f = nf[old_size - 1] if 0 < old_size <= o.maxsize else 1e-6
            new_f = nf[new_size - 1] if 0 < new_size <= o.maxsize else 1e-6
            prob *= old_f / new_f
        if prob < rng.random():
            return PopMember(member.tree.copy(), before_score, before_loss, complexity=member.complexity,
                             parent=member.ref), False
        return PopMember(tree, after_score, after_loss, parent=member.ref), True

    # src/Mutate.jl:349-429
    def crossover_generation(self, m1, m2, curmaxsize):
        o = self.options
        c1, c2 = crossover_trees(m1.tree, m2.tree, self.rng)
        tries = 1
        while True:
            s1, s2 = compute_complexity(c1, o), compute_complexity(c2, o)
            if check_constraints(c1, o, curmaxsize, s1) and check_constraints(c2, o, curmaxsize, s2):
                break
            if tries > 10:
                return m1, m2, False
            c1, c2 = crossover_trees(m1.tree, m2.tree, self.rng)
            tries += 1
        sc1, l1 = self.scorer.score(c1, s1)
        sc2, l2 = self.scorer.score(c2, s2)
        self.num_evals += 2
        return PopMember(c1, sc1, l1, parent=m1.ref), PopMember(c2, sc2, l2, parent=m2.ref), True

    # src/Population.jl:107-160
    def best_of_sample(self, pop, stats):
        o, rng = self.options, self.rng
        n = search_option(o, "tournament_selection_n")
        # n distinct members uniformly at random (argsort of uniform keys: one RNG call)
        sample = [pop[i] for i in np.argsort(rng.random(len(pop)))[:min(n, len(pop))]]
        if search_option(o, "use_frequency_in_tournament"):
            a = search_option(o, "adaptive_parsimony_scaling")
            scores = []
            for m in sample:
                size = m.get_complexity(o)
                freq = stats.normalized_frequencies[size - 1] if 0 < size <= o.maxsize else 0.0
                scores.append(m.score * math.exp(a * freq))
        else:
            scores = [m.score for m in sample]
        p = search_option(o, "tournament_selection_p")
        if p == 1.0:
            return sample[int(np.argmin(scores))]
        k = _draw(_tournament_cdf(len(sample), float(p)), rng.random())
        order = sorted(range(len(scores)), key=scores.__getitem__)  # stable
        return sample[order[k]]

    # src/RegularizedEvolution.jl:13-111
    def reg_evol_cycle(self, pop, temperature, curmaxsize, stats):
        o, rng = self.options, self.rng
        n_cycles = math.ceil(len(pop) / search_option(o, "tournament_selection_n"))
        skip = search_option(o, "skip_mutation_failures")
        for _ in range(n_cycles):
            if rng.random() > search_option(o, "crossover_probability"):
                allstar = self.best_of_sample(pop, stats)
                baby, accepted = self.next_generation(allstar, temperature, curmaxsize, stats)
                if not accepted and skip:
                    continue
                oldest = min(range(len(pop)), key=lambda i: pop[i].birth)
                pop[oldest] = baby
            else:
                a1, a2 = self.best_of_sample(pop, stats), self.best_of_sample(pop, stats)
                b1, b2, accepted = self.crossover_generation(a1, a2, curmaxsize)
                if not accepted and skip:
                    continue
                oldest = min(range(len(pop)), key=lambda i: pop[i].birth)
                pop[oldest] = b1
                oldest = min(range(len(pop)), key=lambda i: pop[i].birth)
                pop[oldest] = b2
        return pop

    # src/SingleIteration.jl:24-98 (batching=false form: the member's own score)
    def s_r_cycle(self, pop, ncycles, curmaxsize, stats):
        o = self.options
        max_temp, min_temp = 1.0, (0.0 if search_option(o, "annealing") else 1.0)
        best_seen = HallOfFame(o)
        for temperature in np.linspace(max_temp, min_temp, ncycles):
            pop = self.reg_evol_cycle(pop, float(temperature), curmaxsize, stats)
            for m in pop:
                size = m.get_complexity(o)
                if 0 < size <= o.maxsize and (not best_seen.exists[size - 1]
                                              or m.score < best_seen.members[size - 1].score):
                    best_seen.exists[size - 1] = True
                    best_seen.members[size - 1] = m.copy()
        return pop, best_seen

    # src/SingleIteration.jl:100-127: simplify every member, optimise constants of a random 14 %
    # (one batched device optimisation for the population instead of one per member)
    def optimize_and_simplify_population(self, pop):
        o, rng = self.options, self.rng
        do_opt = rng.random(len(pop)) < o.optimizer_probability
        if search_option(o, "should_simplify"):
            for m in pop:
                m.tree = combine_operators(simplify_tree(m.tree, o, self.dtype), o, self.dtype)
                m.complexity = -1
        if search_option(o, "should_optimize_constants"):
            chosen = [m for m, d in zip(pop, do_opt) if d and count_constants(m.tree) > 0]
            if chosen:
                _, ne = self._optimizer()(self.dataset, chosen, o, rng=rng)
                self.num_evals += ne
        return pop

    def _optimizer(self):
        """optimize_constants, or the scorer's own (testing / CPU-baseline hook: a scorer object may
        carry ``optimize_constants(dataset, members, options, rng=...)`` with the same contract)."""
        return getattr(self.scorer, "optimize_constants", None) or optimize_constants

    def run_iteration(self, pop, curmaxsize, stats):
        """_dispatch_s_r_cycle (src/SymbolicRegression.jl:1088-1129)."""
        stats = stats.copy()
        stats.normalize_frequencies()
        pop, best_seen = self.s_r_cycle(pop, search_option(self.options, "ncycles_per_iteration"), curmaxsize, stats)
        pop = self.optimize_and_simplify_population(pop)
        return pop, best_seen


def migrate(candidates, pop, options, frac, rng) -> None:
    """migrate! (src/Migration.jl:16-38)."""
    n = len(pop)
    num = int(rng.poisson(n * frac))
    num = min(num, len(candidates), n)
    if num == 0:
        return
    locs = rng.integers(0, n, size=num)
    mig = rng.integers(0, len(candidates), size=num)
    for i, j in zip(locs, mig):
        m = candidates[int(j)].copy()
        m.birth = get_birth_order()
        pop[int(i)] = m


def get_cur_maxsize(options, total_cycles, cycles_remaining) -> int:
    """src/SearchUtils.jl:458-470."""
    w = search_option(options, "warmup_maxsize_by")
    frac = (total_cycles - cycles_remaining) / total_cycles
    if w > 0 and frac <= w:
        return 3 + int(math.floor((options.maxsize - 3) * frac / w))
    return options.maxsize


@dataclass
class SearchResult:
    hall_of_fame: HallOfFame
    populations: list
    num_evals: float
    coalescer_stats: dict
    node_rows: float = 0.0  # tree-node x row evaluations scored on the device (all ranks)

    def pareto_frontier(self):
        return self.hall_of_fame.pareto_frontier()


# ---- :multiprocessing islands (src/SymbolicRegression.jl:964-987) ----------
def _worker_search(worker, key, meta, options, factory):
    """The worker-process side of an island task: a host Dataset over the shared-memory arrays with
    the worker's resident device copy attached (no second upload), and one scorer per dataset --
    a coalescer on a context of its own over the resident dataset (one client: max_wait 0), or
    ``factory``'s."""
    cache = worker.__dict__.setdefault("search", {})
    if worker.backend == "srhip":
        options.device = worker.device
    st = cache.get(key)
    if st is None:
        X, y, w = worker.arrays[key]
        d = Dataset(X, y, w, loss_type=meta["loss_type"])
        d.X_units, d.y_units = meta["X_units"], meta["y_units"]
        dev = None
        if worker.backend == "srhip":
            dev = worker.datasets[key]
            d._dev[(id(worker.ctx), worker.ctx.device)] = dev
        if factory is not None:
            sc = factory(worker, d, options)
        else:
            # the coalescer on a context of its own (over the worker's resident dataset: any context
            # on its device may read it), not the worker's: api.optimize_constants / eval_loss on
            # this thread use the worker's context, and the coalescer's worker threads never share it
            sc = DeviceScorer(d, options, nclients=1, max_wait_us=0, device_dataset=dev)
        st = cache[key] = (d, sc)
    d, sc = st
    if "baseline_loss" in meta:
        d.baseline_loss, d.use_baseline = meta["baseline_loss"], meta["use_baseline"]
    return d, sc


def _scorer_counters(sc):
    c = sc.coalescer.stats() if hasattr(sc, "coalescer") else {}
    return float(getattr(sc, "node_rows", 0)), c


def _counter_delta(before, after):
    (r0, c0), (r1, c1) = before, after
    return r1 - r0, {k: c1[k] - c0.get(k, 0) for k in c1 if k != "max_batch"} | (
        {"max_batch": c1["max_batch"]} if "max_batch" in c1 else {})


def task_search_baseline(worker, ds, key, meta, options, factory=None):
    """update_baseline_loss! on the worker's resident dataset: (baseline_loss, use_baseline)."""
    d, sc = _worker_search(worker, key, meta, options, factory)
    if factory is None:
        update_baseline_loss(d, options)
        return d.baseline_loss, d.use_baseline
    _, loss = sc.score(Node(val=d.avg_y))  # the same constant tree through the factory's scorer
    if np.isfinite(loss):
        return d.loss_type.type(loss), True
    return d.loss_type.type(1), False


def task_score_trees(worker, ds, key, meta, options, trees, factory=None):
    """score_func of each tree (an initial population): ([(score, loss)], counter deltas)."""
    _, sc = _worker_search(worker, key, meta, options, factory)
    before = _scorer_counters(sc)
    out = [sc.score(t) for t in trees]
    return out, _counter_delta(before, _scorer_counters(sc))


def task_island_iteration(worker, ds, key, meta, options, k, rng, num_evals, pop, curmaxsize, stats,
                          factory=None):
    """One island iteration (s_r_cycle + optimize_and_simplify_population) in a worker process:
    (pop, best_seen, rng, num_evals, counter deltas)."""
    from .utils import advance_birth_order

    d, sc = _worker_search(worker, key, meta, options, factory)
    advance_birth_order(max([m.birth for m in pop], default=-1))
    isl = Island(k, d, options, sc, rng, d.X.dtype)
    isl.num_evals = num_evals
    before = _scorer_counters(sc)
    pop, best_seen = isl.run_iteration(pop, curmaxsize, stats)
    return pop, best_seen, isl.rng, isl.num_evals, _counter_delta(before, _scorer_counters(sc))


class _MPIslands:
    """Head-process side: the dataset registered once on the pool, island k pinned to worker
    k % procs (its scorer and resident dataset stay on that worker), counters summed."""

    def __init__(self, pool, dataset, options, factory):
        self.pool, self.options, self.factory = pool, options, factory
        self.key = pool.register_dataset(dataset.X, dataset.y, dataset.weights)
        self.meta = dict(loss_type=dataset.loss_type, X_units=dataset.X_units, y_units=dataset.y_units)
        bl, ub = pool.submit(task_search_baseline, self.key, self.meta, options, factory, dataset=self.key,
                             worker=0).result()
        dataset.baseline_loss, dataset.use_baseline = bl, ub
        self.meta.update(baseline_loss=bl, use_baseline=ub)
        self.node_rows = 0.0
        self.cstats = {}

    def _add(self, delta):
        rows, c = delta
        self.node_rows += rows
        for name, v in c.items():
            self.cstats[name] = max(self.cstats.get(name, 0), v) if name == "max_batch" else self.cstats.get(name, 0) + v

    def score_trees(self, k, trees):
        return self.pool.submit(task_score_trees, self.key, self.meta, self.options, trees, self.factory,
                                dataset=self.key, worker=k % self.pool.nprocs)

    def scores(self, fut):
        out, delta = fut.result()
        self._add(delta)
        return out

    def iterate(self, isl, pop, curmaxsize, stats):
        return self.pool.submit(task_island_iteration, self.key, self.meta, self.options, isl.k, isl.rng,
                                isl.num_evals, pop, curmaxsize, stats, self.factory, dataset=self.key,
                                worker=isl.k % self.pool.nprocs)

    def collect(self, isl, fut):
        from .utils import advance_birth_order

        pop, best_seen, isl.rng, isl.num_evals, delta = fut.result()
        self._add(delta)
        advance_birth_order(max([m.birth for m in pop], default=-1))
        return pop, best_seen


def equation_search(X, y, options, niterations: int = 10, weights=None, seed=None, scorer=None,
                    verbosity: int = 0, distributed=None, group=None, parallelism: str = "multithreading",
                    procs=None, devices=None, worker_backend: str = "srhip", scorer_factory=None) -> SearchResult:
    """equation_search (src/SymbolicRegression.jl:357-1000) for one output, populations as
    concurrent island threads, every score through the device.  ``scorer`` (testing hook):
    any object with ``score(tree, complexity=None) -> (score, loss)``; default: the device
    coalescer.

    Multi-GPU: under torch.distributed with world size > 1 (or
    ``distributed=True``), rank r owns the populations k with k % world == r on its own GPU
    (device = LOCAL_RANK) with a full dataset replica; no collective touches evaluation.  After
    every iteration the ranks exchange their best_sub_pops and hall-of-fame frontiers as node
    tables (:func:`srhip.parallel.exchange_members`, an all-gather over RCCL / xGMI), fold the
    remote members into their hall of fame, all-reduce the adaptive-parsimony size counts, and
    migrate from the global candidate set (src/Migration.jl:16-38).  Islands run in lock step
    across ranks; every rank returns the same global hall of fame.

    ``parallelism="multiprocessing"`` (the reference's `:multiprocessing` with `procs` workers,
    src/SymbolicRegression.jl:964-987): every island's iteration runs in a
    worker process of a :class:`srhip.workers.GPUWorkerPool` (``procs`` workers, default
    min(populations, 16); worker i on ``devices[i % len(devices)]``).  The dataset is copied once into
    shared memory and uploaded once per worker; a task carries one population (node tables) and the
    island's RNG, and returns the evolved population, its best_seen, the RNG and its counters.  Each
    worker scores through its own coalescer on its resident dataset, so islands no longer share one
    interpreter lock.  Island state and processing order are those of the threaded mode, so a
    deterministic search returns the same hall of fame either way (tests/test_gpu_search.py).
    ``worker_backend="host"`` + ``scorer_factory(worker, dataset, options)`` (testing hook): the same
    process machinery without a GPU (tests/test_search.py)."""
    from . import parallel

    dataset = X if isinstance(X, Dataset) else Dataset(X, y, weights)
    dtype = dataset.X.dtype
    npops = search_option(options, "populations")
    psize = search_option(options, "population_size")
    rank, ws = parallel.world()
    if distributed is False:
        rank, ws = 0, 1
    # distributed=True at world size 1: the same lock-step protocol through the exchange (tests)
    dist_mode = ws > 1 or distributed is True
    det = bool(options.deterministic) or dist_mode
    base_seed = options.seed if seed is None else seed
    ss = np.random.SeedSequence(base_seed)
    rngs = [np.random.default_rng(s) for s in ss.spawn(npops + 1)]
    head_rng = rngs[-1] if not dist_mode else np.random.default_rng([int(base_seed or 0), rank, 7919])
    local = [k for k in range(npops) if k % ws == rank]
    mp_mode = parallelism == "multiprocessing"
    if parallelism not in ("multithreading", "multiprocessing"):
        raise ValueError(f"parallelism {parallelism!r}")
    if mp_mode and scorer is not None:
        raise ValueError("parallelism='multiprocessing' scores on the workers: use scorer_factory, not scorer")
    own_scorer = scorer is None and not mp_mode
    if dist_mode:
        import os

        options.device = int(os.environ.get("LOCAL_RANK", options.device))
    pool = mpx = xchg = None
    if own_scorer:
        update_baseline_loss(dataset, options)
        scorer = DeviceScorer(dataset, options, nclients=len(local))
    elif mp_mode:
        from .workers import GPUWorkerPool

        nprocs = int(procs or min(len(local), 16))
        pool = GPUWorkerPool(nprocs, devices=devices if devices is not None else
                             ([options.device] if worker_backend == "srhip" else None), backend=worker_backend)
        mpx = _MPIslands(pool, dataset, options, scorer_factory)
    try:
        islands = {k: Island(k, dataset, options, scorer, rngs[k], dtype) for k in local}
        # initial populations: gen_random_tree(3, ...) scored (src/Population.jl:40-63)
        pops = {}
        init = {}
        for k in local:
            isl = islands[k]
            trees = [gen_random_tree(3, options, dataset.nfeatures, dtype, isl.rng) for _ in range(psize)]
            if mp_mode:
                init[k] = (trees, mpx.score_trees(k, trees))
                continue
            members = []
            for t in trees:
                sc, lo = scorer.score(t)
                members.append(PopMember(t, sc, lo))
            pops[k] = members
        for k, (trees, fut) in init.items():
            pops[k] = [PopMember(t, sc, lo) for t, (sc, lo) in zip(trees, mpx.scores(fut))]
        stats = RunningSearchStatistics(options)
        hof = HallOfFame(options)
        best_sub_pops = {k: [] for k in local}
        total_cycles = npops * niterations
        cycles_remaining = total_cycles
        curmaxsize = get_cur_maxsize(options, total_cycles, cycles_remaining)
        num_evals = float(len(local) * psize)
        topn = search_option(options, "topn")
        if dist_mode and xchg is None:
            from . import device as _device_mod

            # libsrhip's communicator when the search runs on the device (its own scorer or device workers)
            on_device = own_scorer or (mp_mode and worker_backend == "srhip")
            xchg = parallel.IterationExchange.for_search(
                options, npops, ws, topn, len(stats.frequencies), lambda: _device_mod.get_context(options.device),
                group, native=on_device)

        def process(k, pop, best_seen):
            nonlocal cycles_remaining, curmaxsize, num_evals
            best_sub_pops[k] = [m for m in sorted(pop, key=lambda m: m.score)][:topn]
            for m in pop:
                stats.update_frequencies(m.get_complexity(options))
            hof.update(pop, options)
            hof.update([m for m, e in zip(best_seen.members, best_seen.exists) if e], options)
            dominating = hof.pareto_frontier()
            if search_option(options, "migration"):
                cands = [m for sp in best_sub_pops.values() for m in sp]
                migrate(cands, pop, options, search_option(options, "fraction_replaced"), head_rng)
            if search_option(options, "hof_migration") and dominating:
                migrate(dominating, pop, options, search_option(options, "fraction_replaced_hof"), head_rng)
            cycles_remaining -= 1
            curmaxsize = get_cur_maxsize(options, total_cycles, cycles_remaining)
            stats.move_window()
            pops[k] = pop

        def process_distributed(results, it):
            """One lock-step iteration's bookkeeping across ranks (see the docstring)."""
            nonlocal cycles_remaining, curmaxsize
            nbin = len(stats.frequencies)
            counts = np.zeros(nbin)
            for k in local:
                pop, best_seen = results[k]
                best_sub_pops[k] = [m for m in sorted(pop, key=lambda m: m.score)][:topn]
                for m in pop:
                    size = m.get_complexity(options)
                    if 0 < size <= nbin:
                        counts[size - 1] += 1
                hof.update(pop, options)
                hof.update([m for m, e in zip(best_seen.members, best_seen.exists) if e], options)
                pops[k] = pop
            mine = [m for k in local for m in best_sub_pops[k]]
            front = hof.pareto_frontier()
            sent = mine + front
            # ONE fixed-size all-gather per iteration: every rank's best_sub_pops, then its frontier,
            # with (score, loss), and its adaptive-parsimony size counts (parallel.IterationExchange)
            got = xchg.exchange([m.tree for m in sent], [m.score for m in sent], [m.loss for m in sent],
                                len(mine), counts, options, dtype)
            for _, _, cnt in got:  # rank order; integer counts: the sum is exact in any order
                stats.frequencies += cnt
            stats.move_window()
            cands, remote_front = [], []
            for ns, members, _ in got:
                chunk = [PopMember(t, sc, lo) for t, sc, lo in members]
                cands.extend(chunk[:ns])
                remote_front.extend(chunk[ns:])
            hof.update(cands + remote_front, options)
            dominating = hof.pareto_frontier()
            for k in local:
                if search_option(options, "migration"):
                    migrate(cands, pops[k], options, search_option(options, "fraction_replaced"), head_rng)
                if search_option(options, "hof_migration") and dominating:
                    migrate(dominating, pops[k], options, search_option(options, "fraction_replaced_hof"), head_rng)
            cycles_remaining = total_cycles - (it + 1) * npops
            curmaxsize = get_cur_maxsize(options, total_cycles, cycles_remaining)

        with ThreadPoolExecutor(max_workers=max(1, len(local))) as ex:
            def submit(k):
                if mp_mode:
                    return mpx.iterate(islands[k], pops[k], curmaxsize, stats)
                return ex.submit(islands[k].run_iteration, pops[k], curmaxsize, stats)

            def result(k, fut):
                return mpx.collect(islands[k], fut) if mp_mode else fut.result()

            if det:
                for it in range(niterations):
                    futs = {k: submit(k) for k in local}
                    if dist_mode:
                        process_distributed({k: result(k, f) for k, f in futs.items()}, it)
                    else:
                        for k in local:
                            pop, best_seen = result(k, futs[k])
                            process(k, pop, best_seen)
                    if verbosity and rank == 0:
                        print(f"iteration {it + 1}/{niterations}: best loss "
                              f"{min(m.loss for m in hof.pareto_frontier()):.4g}", flush=True)
            else:
                # asynchronous like the reference: a finished population is processed and re-dispatched
                remaining = {k: niterations for k in local}
                running = {submit(k): k for k in local}
                from concurrent.futures import FIRST_COMPLETED, wait

                while running:
                    done, _ = wait(list(running), return_when=FIRST_COMPLETED)
                    for f in done:
                        k = running.pop(f)
                        pop, best_seen = result(k, f)
                        process(k, pop, best_seen)
                        remaining[k] -= 1
                        if remaining[k] > 0:
                            running[submit(k)] = k
                        elif own_scorer:
                            # one client fewer: the coalescer stops waiting for this island
                            scorer.coalescer.set_clients(sum(1 for r in remaining.values() if r > 0))
        num_evals += sum(isl.num_evals for isl in islands.values())
        if dist_mode and ws > 1:
            num_evals = float(parallel.allreduce_np(np.array([num_evals]), "sum", group)[0])
        if mp_mode:
            cstats, node_rows = mpx.cstats, mpx.node_rows
        else:
            cstats = scorer.coalescer.stats() if own_scorer else {}
            node_rows = float(getattr(scorer, "node_rows", 0))
        if dist_mode and ws > 1:
            node_rows = float(parallel.allreduce_np(np.array([node_rows]), "sum", group)[0])
        return SearchResult(hof, [pops[k] for k in local], num_evals, cstats, node_rows)
    finally:
        if xchg is not None:
            xchg.close()
        if own_scorer:
            scorer.close()
        if pool is not None:
            pool.close()
