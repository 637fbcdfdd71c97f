"""The batching-mode batch seams, each one device launch per population,
checked against the per-member reference calls bit for bit:

* s_r_cycle's fixed-batch re-score with its loss cache (src/SingleIteration.jl:46-82):
  srhip.rescore_population_batched;
* finalize_scores (src/Population.jl:162-176): srhip.finalize_scores;
* the best_seen re-score after each cycle (src/SymbolicRegression.jl:1120-1127):
  srhip.rescore_hall_of_fame.
"""
import numpy as np
import pytest

import srhip

pytestmark = pytest.mark.gpu

OPS = dict(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))


class _Member:
    def __init__(self, tree):
        self.tree, self.score, self.loss = tree, np.nan, np.nan


def _setup(dtype, n=6000, npop=200, batch_size=700):
    opts = srhip.Options(batching=True, batch_size=batch_size, **OPS)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((3, n)).astype(dtype)
    y = (2 * np.cos(X[1]) + X[0] ** 2 - 2).astype(dtype)
    d = srhip.Dataset(X, y)
    srhip.update_baseline_loss(d, opts)
    trees = srhip.random_population(npop, opts, 3, dtype, seed=4, max_size=25)
    return opts, d, [_Member(t) for t in trees]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_rescore_population_batched_equals_per_member(dtype):
    opts, d, pop = _setup(dtype)
    idx = srhip.batch_sample(d, opts, np.random.default_rng(5))
    cache = srhip.LossCache(len(pop), d.loss_type)
    scores, n_eval = srhip.rescore_population_batched(d, pop, opts, idx, cache, first_loop=True)
    assert n_eval == len(pop)
    for m, sc in zip(pop, scores):
        ref, _ = srhip.score_func_batched(d, m, opts, idx=idx)
        assert sc == ref or (np.isnan(sc) and np.isnan(ref)), (srhip.string_tree(m.tree, opts), sc, ref)
    # mutate a few members: only those are evaluated again, the rest keep their cached scores
    changed = [3, 50, 199]
    for i in changed:
        pop[i].tree = srhip.random_population(1, opts, 3, dtype, seed=100 + i, max_size=20)[0]
    pop[7].tree = pop[7].tree.copy()  # a structurally equal copy is not re-scored
    scores2, n_eval2 = srhip.rescore_population_batched(d, pop, opts, idx, cache, first_loop=False)
    assert n_eval2 == len(changed)
    for i, m in enumerate(pop):
        if i in changed:
            ref, _ = srhip.score_func_batched(d, m, opts, idx=idx)
            assert scores2[i] == ref
        else:
            assert scores2[i] == scores[i] or (np.isnan(scores2[i]) and np.isnan(scores[i]))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_finalize_scores_and_hall_of_fame_rescore(dtype):
    opts, d, pop = _setup(dtype)
    assert srhip.finalize_scores(d, pop, opts) == len(pop)
    for m in pop:
        ref_s, ref_l = srhip.score_func(d, m, opts)
        assert m.loss == ref_l or (np.isinf(m.loss) and np.isinf(ref_l))
        assert m.score == ref_s or (np.isinf(m.score) and np.isinf(ref_s))
    hof = srhip.HallOfFame(opts)
    for k in range(0, len(hof.members), 2):
        hof.members[k], hof.exists[k] = _Member(pop[k].tree), True
    assert srhip.rescore_hall_of_fame(d, hof.members, hof.exists, opts) == len(hof.members)
    for m, e in zip(hof.members, hof.exists):
        if e:
            ref_s, ref_l = srhip.score_func(d, m, opts)
            assert m.loss == ref_l or (np.isinf(m.loss) and np.isinf(ref_l))
    nob = srhip.Options(**OPS)
    assert srhip.finalize_scores(d, pop, nob) == 0.0  # batching=false: nothing to recompute
