"""Helpers (mirror of src/attacks/moeva2/utils.py:11-76)."""
from typing import List

import numpy as np

from .result_process import History, Population

ONE_HOT_ENCODE_KEY = "ohe"


class MinMax1D:
    """Fitted 1-feature MinMaxScaler (``get_scaler_from_norm``)."""

    def __init__(self, lo, hi):
        rng = hi - lo
        self.scale_ = np.array([1.0 / (rng if rng != 0 else 1.0)])
        self.min_ = np.array([0.0 - lo * self.scale_[0]])

    def transform(self, x):
        x = np.array(x, dtype=np.float64, copy=True)
        x *= self.scale_
        x += self.min_
        return x


def get_scaler_from_norm(norm, nb_features):
    """utils.py:11-22: f2 scaler fit on [[0],[sqrt(n)]] (L2) or [[0],[1]] (Linf)."""
    if norm in [2, "2"]:
        return MinMax1D(0.0, np.sqrt(nb_features))
    if norm in [np.inf, "inf"]:
        return MinMax1D(0.0, 1.0)
    raise NotImplementedError


def get_ohe_masks(type_mask):
    seen, masks = [], []
    for i, e_type in enumerate(type_mask):
        if str(e_type).startswith(ONE_HOT_ENCODE_KEY):
            if e_type in seen:
                masks[seen.index(e_type)].append(i)
            else:
                seen.append(e_type)
                masks.append([i])
    return [np.array(e) for e in masks]


def get_one_hot_encoding_constraints(type_mask, x):
    """utils.py:43-54: sum over groups of |1 - sum(one-hot group)|."""
    masks = get_ohe_masks(type_mask)
    if len(masks) == 0:
        return np.zeros(x.shape[0])
    vals = np.column_stack([np.sum(x[:, m], axis=1) for m in masks])
    return np.sum(np.abs(1 - vals), axis=1)


def _pop_x(pop):
    """One state's final genes (P, V) fp64: the engine's Population hands its array over,
    anything else is stacked individual by individual as utils.py:59-61 does."""
    if isinstance(pop, Population):
        return np.asarray(pop._X, dtype=np.float64)
    return np.array([ind.X.astype(np.float64) for ind in pop])


def results_to_numpy_results(results: List, encoder):
    """utils.py:57-67 -> (n_states, pop_size, n_features)."""
    initial_states = [r.initial_state for r in results]
    pops_x = [_pop_x(r.pop) for r in results]
    return np.array([encoder.genetic_to_ml(pops_x[i], initial_states[i])
                     for i in range(len(results))])


def results_to_history(results: List):
    """utils.py:70-76: drop the initial-population entry -> (n_states, n_gen - 1, O, w)."""
    if results and all(isinstance(r.history, History) for r in results):
        return np.stack([r.history.offspring_rows() for r in results])
    return np.array([[g.tolist() for i, g in enumerate(r.history) if i > 0] for r in results])
