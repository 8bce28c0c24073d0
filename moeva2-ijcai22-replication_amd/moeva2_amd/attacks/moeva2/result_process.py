"""Per-state attack results (mirror of src/attacks/moeva2/result_process.py:2-23).

The reference wraps a pymoo ``Result`` (moeva2.py:167-171); here the fields are filled from the
engine's final population.  ``pop`` is a sequence of individuals exposing ``.X`` / ``.F`` (and
``pop.get("X")`` like a pymoo Population) and ``history`` a sequence of per-evaluation ``F``
(or ``[F | G]``) arrays, one per generation.  Both are views over the arrays the engine
handed back for ALL states (one device -> host copy each), so building the B result objects
costs O(B), not O(B x P) individuals or O(B x n_gen) history arrays; an individual / a
history entry is made when it is indexed.  They pickle as their arrays.
"""
from collections.abc import Sequence

import numpy as np


class Individual:
    __slots__ = ("X", "F")

    def __init__(self, X, F):
        self.X = X
        self.F = F


class Population(Sequence):
    """pymoo Population stand-in over one state's final population: X (P, V), F (P, 3)."""

    __slots__ = ("_X", "_F")

    def __init__(self, X, F):
        self._X = X
        self._F = F

    def __len__(self):
        return self._X.shape[0]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return Population(self._X[i], self._F[i])
        return Individual(self._X[i], self._F[i])

    def get(self, key):
        """pymoo Population.get: a new array of the attribute over the individuals."""
        return np.array({"X": self._X, "F": self._F}[key])

    def __reduce__(self):
        return Population, (self._X, self._F)


class History(Sequence):
    """One state's evaluation history as DefaultProblem._evaluate appends it
    (default_problem.py:137-140): entry 0 = the initial population's P rows, entry g >= 1 =
    generation g's O offspring rows; rows (P + (n_gen - 1) O, 3 | 3 + C)."""

    __slots__ = ("_h", "_P", "_O", "_n")

    def __init__(self, rows, P, O, n_gen):
        self._h = rows
        self._P = P
        self._O = O
        self._n = n_gen

    def __len__(self):
        return self._n

    def __getitem__(self, g):
        if isinstance(g, slice):
            return [self[k] for k in range(*g.indices(self._n))]
        if g < 0:
            g += self._n
        if not 0 <= g < self._n:
            raise IndexError("history index out of range")
        if g == 0:
            return self._h[:self._P]
        lo = self._P + (g - 1) * self._O
        return self._h[lo:lo + self._O]

    def offspring_rows(self):
        """Entries 1 .. n_gen-1 as one (n_gen - 1, O, w) array view (results_to_history)."""
        return self._h[self._P:].reshape(self._n - 1, self._O, self._h.shape[1])

    def __reduce__(self):
        return History, (self._h, self._P, self._O, self._n)


class EfficientResult:
    def __init__(self, result=None):
        if result is not None:
            self.pop = result["pop"]
            self.initial_state = result["initial_state"]
            self.n_gen = result["n_gen"]
            self.pop_size = result["pop_size"]
            self.n_offsprings = result["n_offsprings"]
            self.X = result["X"]
            self.F = result["F"]
            self.pareto = result["pareto"]


class HistoryResult(EfficientResult):
    def __init__(self, result=None):
        super().__init__(result)
        if result is not None:
            self.history = result["history"]
