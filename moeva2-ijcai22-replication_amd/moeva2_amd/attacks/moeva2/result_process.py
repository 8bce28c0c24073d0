"""Per-state attack results (mirror of src/attacks/moeva2/result_process.py:2-23).

The reference wraps a pymoo ``Result``; here the fields are filled from the engine's
final population.  ``pop`` is a list of individuals exposing ``.X`` / ``.F`` (and
``pop.get("X")`` like a pymoo Population)."""
import numpy as np


class Individual:
    __slots__ = ("X", "F")

    def __init__(self, X, F):
        self.X = X
        self.F = F


class Population(list):
    def get(self, key):
        return np.array([getattr(ind, key) for ind in self])


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
