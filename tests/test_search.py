"""The search loop — host logic on the CPU.

The product scores through the device coalescer; these CPU tests drive the same islands with a
test-only scorer built on the oracle (the checker), so mutation / selection / hall-of-fame /
migration logic runs without a GPU.  tests/test_gpu_search.py runs the real path."""
import math

import numpy as np
import pytest

import srhip
from srhip import search as S

OPS = dict(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))


class OracleScorer:
    """score_func restated through the oracle (tests only)."""

    def __init__(self, dataset, options, oracle):
        self.d, self.o, self.orc = dataset, options, oracle
        self.calls = 0

    def score(self, tree, complexity=None, idx=None):
        nodes, offs = srhip.flatten([tree], self.o, self.d.X.dtype)
        le, _, ok, _ = self.orc.eval_loss_batch(nodes, offs, self.o.binop_codes, self.o.unaop_codes, self.d.X, self.d.y)
        self.calls += 1
        L = self.d.loss_type.type
        loss = L(le[0]) if ok[0] else L(np.inf)
        return srhip.loss_to_score(loss, self.d.use_baseline, self.d.baseline_loss, tree, self.o, complexity), loss


def _data(n=100, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((2, n))
    y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
    return X, y


def _tree_ok(t, options):
    for n in t:
        if n.degree == 0:
            assert n.constant or 1 <= n.feature
        elif n.degree == 1:
            assert 1 <= n.op <= options.nuna and n.l is not None
        else:
            assert 1 <= n.op <= options.nbin and n.l is not None and n.r is not None


def test_mutations_keep_trees_valid():
    o = srhip.Options(**OPS)
    rng = np.random.default_rng(1)
    for i in range(300):
        t = S.gen_random_tree_fixed_size(int(rng.integers(1, 15)), o, 3, np.float64, rng)
        for f in (lambda t: S.swap_operands(t, rng), lambda t: S.mutate_operator(t, o, rng),
                  lambda t: S.mutate_constant(t, 0.5, o, np.float64, rng),
                  lambda t: S.append_random_op(t, o, 3, np.float64, rng),
                  lambda t: S.prepend_random_op(t, o, 3, np.float64, rng),
                  lambda t: S.insert_random_op(t, o, 3, np.float64, rng),
                  lambda t: S.delete_random_op(t, o, 3, np.float64, rng)):
            t = f(t)
            _tree_ok(t, o)


def test_insert_prepend_grow_delete_shrinks():
    """src/MutationFunctions.jl: insert / prepend add one operator node (+1 leaf if binary);
    delete removes one operator node (or replaces a leaf)."""
    o = srhip.Options(**OPS)
    rng = np.random.default_rng(2)
    for _ in range(200):
        t = S.gen_random_tree_fixed_size(9, o, 2, np.float64, rng)
        n0 = srhip.count_nodes(t)
        n1 = srhip.count_nodes(S.insert_random_op(t.copy(), o, 2, np.float64, rng))
        n2 = srhip.count_nodes(S.prepend_random_op(t.copy(), o, 2, np.float64, rng))
        n3 = srhip.count_nodes(S.delete_random_op(t.copy(), o, 2, np.float64, rng))
        assert n1 in (n0 + 1, n0 + 2) and n2 in (n0 + 1, n0 + 2) and n3 <= n0


def test_crossover_conserves_nodes():
    o = srhip.Options(**OPS)
    rng = np.random.default_rng(3)
    for _ in range(200):
        a = S.gen_random_tree_fixed_size(7, o, 2, np.float64, rng)
        b = S.gen_random_tree_fixed_size(11, o, 2, np.float64, rng)
        c, d = S.crossover_trees(a, b, rng)
        assert srhip.count_nodes(c) + srhip.count_nodes(d) == 18
        assert srhip.count_nodes(a) == 7 and srhip.count_nodes(b) == 11  # parents untouched


def test_simplify_folds_constants():
    o = srhip.Options(**OPS)
    x1 = srhip.Node("x1")
    t = (srhip.Node(val=2.0) + srhip.Node(val=3.0)) * x1
    s = S.simplify_tree(t.copy(), o, np.float64)
    assert srhip.string_tree(s, o) == "(5.0 * x1)"
    # non-finite folds are kept unfolded (1/0)
    t = srhip.Node(val=1.0) / srhip.Node(val=0.0)
    assert srhip.count_nodes(S.simplify_tree(t, o, np.float64)) == 3
    # combine_operators: 2 + (3 + x1) -> 5 + x1 ; 2 * (x1 * 4) -> 8 * x1
    t = srhip.Node(val=2.0) + (srhip.Node(val=3.0) + x1)
    assert srhip.string_tree(S.combine_operators(t, o, np.float64), o) == "(5.0 + x1)"
    t = srhip.Node(val=2.0) * (x1 * srhip.Node(val=4.0))
    assert srhip.string_tree(S.combine_operators(t, o, np.float64), o) == "(8.0 * x1)"


def test_check_constraints_size_depth():
    o = srhip.Options(maxsize=7, **OPS)
    rng = np.random.default_rng(4)
    assert S.check_constraints(S.gen_random_tree_fixed_size(7, o, 2, np.float64, rng), o, 7)
    assert not S.check_constraints(S.gen_random_tree_fixed_size(9, o, 2, np.float64, rng), o, 7)
    deep = srhip.Node("x1")
    for _ in range(8):
        deep = srhip.Node("cos", deep)
    assert not S.check_constraints(deep, srhip.Options(maxsize=30, maxdepth=5, **OPS), 30)


def test_running_statistics_window():
    """move_window! (src/AdaptiveParsimony.jl:55-88) keeps the total at window_size."""
    o = srhip.Options(maxsize=10, **OPS)
    st = S.RunningSearchStatistics(o, window_size=50)
    rng = np.random.default_rng(5)
    for _ in range(500):
        st.update_frequencies(int(rng.integers(1, 12)))
    st.move_window()
    assert abs(st.frequencies.sum() - 50) < 1e-6 and np.all(st.frequencies >= 1 - 1e-12)
    st.normalize_frequencies()
    assert abs(st.normalized_frequencies.sum() - 1) < 1e-12


def test_tournament_weights():
    w = S.tournament_selection_weights(12, 0.86)
    assert abs(w.sum() - 1) < 1e-12 and w[0] > w[1] > w[-1]


def test_migration_poisson():
    rng = np.random.default_rng(6)
    o = srhip.Options(**OPS)
    pop = [S.PopMember(srhip.Node(val=float(i)), 1.0, 1.0) for i in range(33)]
    cands = [S.PopMember(srhip.Node("x1"), 0.0, 0.0)]
    moved = []
    for _ in range(400):
        p = [m.copy() for m in pop]
        S.migrate(cands, p, o, 0.035, rng)
        moved.append(sum(1 for m in p if m.tree.degree == 0 and not m.tree.constant))
    # E[num] = 33 * 0.035 = 1.155 (clamped at len(candidates) = 1 draw per location, with replacement)
    assert 0.4 < np.mean(moved) < 1.2


def test_hall_of_fame_pareto():
    o = srhip.Options(maxsize=10, **OPS)
    h = S.HallOfFame(o)
    mk = lambda n, loss: S.PopMember(S.gen_random_tree_fixed_size(n, o, 1, np.float64, np.random.default_rng(n)),  # noqa: E731
                                     loss, loss)
    h.update([mk(1, 5.0), mk(3, 2.0), mk(5, 3.0), mk(7, 1.0)], o)
    front = h.pareto_frontier()
    assert [srhip.count_nodes(m.tree) for m in front] == [1, 3, 7]


def test_search_host_logic_deterministic(oracle):
    """A small search (4 islands x 20 members, 40 cycles, 3 iterations) with the oracle scorer:
    improves on the initial population, is reproducible with deterministic=True, and every
    hall-of-fame loss equals a fresh evaluation of its tree."""
    X, y = _data()
    o = srhip.Options(populations=4, population_size=20, ncycles_per_iteration=40, maxsize=15,
                      deterministic=True, seed=0, should_optimize_constants=False, **OPS)
    runs = []
    for _ in range(2):
        d = srhip.Dataset(X, y)
        d.baseline_loss, d.use_baseline = np.float64(np.mean((y - y.mean()) ** 2)), True
        sc = OracleScorer(d, o, oracle)
        res = S.equation_search(d, None, o, niterations=3, scorer=sc)
        runs.append(res)
        front = res.pareto_frontier()
        assert front
        for m in front:
            s2, l2 = sc.score(m.tree)
            assert l2 == m.loss or (math.isinf(l2) and math.isinf(m.loss))
    f0 = [(srhip.string_tree(m.tree, o), m.loss) for m in runs[0].pareto_frontier()]
    f1 = [(srhip.string_tree(m.tree, o), m.loss) for m in runs[1].pareto_frontier()]
    assert f0 == f1
    best = min(m.loss for m in runs[0].pareto_frontier())
    assert best < 0.5 * np.mean((y - y.mean()) ** 2)


def oracle_scorer_factory(worker, dataset, options):
    """scorer_factory of the :multiprocessing test (module level: workers import it by name)."""
    import oracle as orc

    return OracleScorer(dataset, options, orc)


def test_search_multiprocessing_equals_threads(oracle):
    """parallelism='multiprocessing' (islands in GPUWorkerPool processes, the
    dataset resident per worker, populations and RNGs shipped per iteration) returns exactly the
    threaded search's hall of fame: same seeds, same island state, same processing order."""
    X, y = _data()
    o = srhip.Options(populations=4, population_size=20, ncycles_per_iteration=30, maxsize=15,
                      deterministic=True, seed=3, should_optimize_constants=False, **OPS)
    base = np.float64(np.mean((y - y.mean()) ** 2))
    d = srhip.Dataset(X, y)
    d.baseline_loss, d.use_baseline = base, True
    threaded = S.equation_search(d, None, o, niterations=2, scorer=OracleScorer(d, o, oracle))
    d2 = srhip.Dataset(X, y)
    mp = S.equation_search(d2, None, o, niterations=2, parallelism="multiprocessing", procs=2,
                           worker_backend="host", scorer_factory=oracle_scorer_factory)
    assert d2.baseline_loss == base and d2.use_baseline
    f0 = [(srhip.string_tree(m.tree, o), m.loss, m.score) for m in threaded.pareto_frontier()]
    f1 = [(srhip.string_tree(m.tree, o), m.loss, m.score) for m in mp.pareto_frontier()]
    assert f0 == f1
    assert mp.num_evals == threaded.num_evals
    for p0, p1 in zip(threaded.populations, mp.populations):
        assert [srhip.string_tree(m.tree, o) for m in p0] == [srhip.string_tree(m.tree, o) for m in p1]
