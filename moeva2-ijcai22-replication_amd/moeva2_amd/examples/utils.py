"""Augmented-feature consistency constraints (mirror of src/examples/utils.py:7-29) and the
XOR feature augmentation (src/experiments/botnet/features.py:6-21)."""
from itertools import combinations
from math import comb

import numpy as np

from ..attacks.moeva2.constraints import ConstraintProgram


def augmented_xor_program(prog: ConstraintProgram, n_features: int, important_features,
                          features_mean) -> ConstraintProgram:
    """One |x_aug - xor(x_i >= m_i, x_j >= m_j)| op per pair, x_aug = the trailing
    C(n_important, 2) features (constraints_augmented_np)."""
    n_imp = len(important_features)
    first_aug = n_features - comb(n_imp, 2)
    for idx, (i1, i2) in enumerate(combinations(range(n_imp), 2)):
        prog.add("XOR_AUG", (first_aug + idx, int(important_features[i1]),
                             int(important_features[i2])),
                 (float(features_mean[i1]), float(features_mean[i2])))
    return prog


def augment_data(x, important_features):
    """features.py:6-21: append the pairwise XOR indicator features."""
    original_shape = x.shape
    local_x = x.reshape(-1, original_shape[-1])
    new_features = []
    for i1, i2 in combinations(range(important_features.shape[0]), 2):
        new_features.append(np.logical_xor(
            local_x[:, int(important_features[i1, 0])] >= important_features[i1, 1],
            local_x[:, int(important_features[i2, 0])] >= important_features[i2, 1],
        ).astype(np.float64))
    new_x = np.concatenate((local_x, np.column_stack(new_features)), axis=1)
    return new_x.reshape(*original_shape[:-1], -1)
