"""LCLD + augmented XOR features (mirror of src/examples/lcld/lcld_augmented_constraints.py:
10 LCLD columns, then constraints_augmented_np over the 5 important features)."""
from math import comb

import numpy as np

from ...attacks.moeva2.constraints import ConstraintProgram, TabularConstraints, _resolve
from ..utils import augmented_xor_program
from .lcld_constraints import lcld_program


class LcldAugmentedConstraints(TabularConstraints):
    def __init__(self, feature_path: str, constraints_path: str, import_features_path=None):
        super().__init__(feature_path, constraints_path)
        if import_features_path is None:
            import_features_path = _resolve(feature_path, "important_features.npy")
        self.important_features = np.load(import_features_path, allow_pickle=False)

    def device_program(self) -> ConstraintProgram:
        prog = lcld_program(ConstraintProgram())
        return augmented_xor_program(prog, self._feature_type.shape[0],
                                     self.important_features[:, 0], self.important_features[:, 1])

    def get_nb_constraints(self) -> int:
        return 10 + comb(len(self.important_features), 2)
