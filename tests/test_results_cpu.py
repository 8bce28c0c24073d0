"""Host logic of Moeva2.generate's results (no GPU): the result objects that view the
engine's arrays behave like the reference's lists (result_process.py:2-23, utils.py:57-76),
and the batched per-state bounds equal the reference's per-state get_feature_min_max
(lcld_constraints.py:237-263, botnet_constraints.py:190-216)."""
import os
import pickle

import numpy as np
import pytest

from conftest import RES
from oracle.problems import PROJECTS


def _hist(P=5, O=3, G=4, w=3, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((P + (G - 1) * O, w))


def test_history_entries_match_list_form():
    from moeva2_amd.attacks.moeva2.result_process import History

    P, O, G = 5, 3, 4
    h = _hist(P, O, G)
    ref = [h[:P]] + [h[P + (g - 1) * O: P + g * O] for g in range(1, G)]
    hist = History(h, P, O, G)
    assert len(hist) == G
    for g in range(G):
        np.testing.assert_array_equal(hist[g], ref[g])
    np.testing.assert_array_equal(hist[-1], ref[-1])
    assert [a.shape for a in hist[1:3]] == [r.shape for r in ref[1:3]]
    assert [a.tolist() for a in hist] == [r.tolist() for r in ref]
    with pytest.raises(IndexError):
        hist[G]
    np.testing.assert_array_equal(hist.offspring_rows(), np.stack(ref[1:]))
    back = pickle.loads(pickle.dumps(hist))
    assert [a.tolist() for a in back] == [r.tolist() for r in ref]


def test_population_behaves_like_individual_list():
    from moeva2_amd.attacks.moeva2.result_process import Population

    rng = np.random.default_rng(1)
    X, F = rng.standard_normal((6, 4)), rng.standard_normal((6, 3))
    pop = Population(X, F)
    assert len(pop) == 6
    np.testing.assert_array_equal(np.array([ind.X for ind in pop]), X)
    np.testing.assert_array_equal(pop[2].F, F[2])
    got = pop.get("X")
    np.testing.assert_array_equal(got, X)
    assert got is not X  # pymoo's get builds a new array
    assert len(pop[1:4]) == 3
    back = pickle.loads(pickle.dumps(pop))
    np.testing.assert_array_equal(back.get("F"), F)


def test_result_conversions_match_reference_forms():
    """results_to_history / results_to_numpy_results on the view-backed results equal the
    reference's list forms (utils.py:57-76)."""
    from moeva2_amd.attacks.moeva2.result_process import (History, HistoryResult, Individual,
                                                          Population)
    from moeva2_amd.attacks.moeva2.utils import results_to_history, results_to_numpy_results

    P, O, G, V = 5, 3, 4, 4
    rng = np.random.default_rng(2)
    res_fast, res_list = [], []
    for b in range(3):
        h = _hist(P, O, G, seed=b)
        X, F = rng.standard_normal((P, V)), rng.standard_normal((P, 3))
        base = {"initial_state": np.zeros(V), "n_gen": G, "pop_size": P, "n_offsprings": O,
                "X": X[:2], "F": F[:2], "pareto": np.empty((0, V))}
        res_fast.append(HistoryResult(dict(base, pop=Population(X, F),
                                           history=History(h, P, O, G))))
        res_list.append(HistoryResult(dict(base, pop=[Individual(X[i], F[i]) for i in range(P)],
                                           history=list(History(h, P, O, G)))))
    np.testing.assert_array_equal(results_to_history(res_fast), results_to_history(res_list))

    class Ident:
        def genetic_to_ml(self, x, x0):
            return x + x0.sum()

    np.testing.assert_array_equal(results_to_numpy_results(res_fast, Ident()),
                                  results_to_numpy_results(res_list, Ident()))


@pytest.mark.parametrize("name", ["botnet", "lcld", "lcld_augmented"])
def test_batched_feature_bounds_match_per_state(name):
    from moeva2_amd.experiments.united.utils import STR_TO_CONSTRAINTS_CLASS
    from oracle.problems import Project

    feat = os.path.join(RES, PROJECTS[name][0])
    c = STR_TO_CONSTRAINTS_CLASS[name](feat, feat.replace("features", "constraints"))
    X = Project(name).x[:40]
    xl, xu = c.feature_min_max_batch(X)
    for b in range(X.shape[0]):
        lo, hi = c.get_feature_min_max(dynamic_input=X[b])
        assert np.array_equal(lo, xl[b]) and np.array_equal(hi, xu[b])
        assert lo.dtype == xl.dtype == np.float64
