"""Genetic <-> ML representation (mirror of src/attacks/moeva2/feature_encoder.py).

Host-side description of the genetic layout: which features mutate, how one-hot groups
collapse to one integer gene, the genetic bounds and types.  The per-candidate decode
(genetic_to_ml) of the hot path runs inside the HIP evaluation kernel; the host methods
here serve problem setup and result packaging (``results_to_numpy_results``).
"""
from typing import Tuple

import numpy as np

from .constraints import Constraints

ONEHOT_ENCODE_KEY = "ohe"


class FeatureEncoder:
    def __init__(self, mutable_mask, type_mask: np.ndarray, xl: np.ndarray, xu: np.ndarray):
        self.type_mask = type_mask
        self.mutable_mask = np.asarray(mutable_mask).astype(bool)
        self._xl = np.asarray(xl, np.float64)
        self._xu = np.asarray(xu, np.float64)
        n = self.mutable_mask.shape[0]
        if type_mask.shape[0] != n or self._xl.shape[0] != n or self._xu.shape[0] != n:
            raise ValueError("mutable_mask, type_mask, xl and xu must have same shape.")
        lo = np.minimum(self._xl, self._xu)
        rng = np.maximum(self._xl, self._xu) - lo
        rng = np.where(rng == 0, 1.0, rng)
        self._mm_scale = 1.0 / rng  # MinMaxScaler().fit([xl, xu]) (feature_encoder.py:39-40)
        self._mm_min = 0.0 - lo * self._mm_scale
        self._create_one_hot_encoders()

    def _create_one_hot_encoders(self):
        """feature_encoder.py:58-86."""
        seen, masks = [], []
        for i, e_type in enumerate(self._ml_to_mutable(self.type_mask)):
            if str(e_type).startswith(ONEHOT_ENCODE_KEY):
                if e_type in seen:
                    masks[seen.index(e_type)].append(i)
                else:
                    seen.append(e_type)
                    masks.append([i])
        self._one_hot_masks = [np.array(m) for m in masks]
        no = np.ones(int(self.mutable_mask.sum()), dtype=bool)
        for m in self._one_hot_masks:
            no[m] = False
        self._no_one_hot_mask = no

    def _ml_to_mutable(self, x: np.ndarray) -> np.ndarray:
        return x[..., self.mutable_mask]

    def _mutable_to_ml(self, x, x_initial_ml):
        out = np.zeros((x.shape[0], x_initial_ml.shape[0]))
        out[:, ~self.mutable_mask] = x_initial_ml[~self.mutable_mask]
        out[:, self.mutable_mask] = x
        return out

    def _mutable_to_cat_encode(self, x):
        n = int(self._no_one_hot_mask.sum())
        result = np.empty((x.shape[0], self.get_genetic_v_length()))
        result[:, :n] = x[:, self._no_one_hot_mask]
        for index, mask in enumerate(self._one_hot_masks):
            result[:, n + index] = np.argmax(x[:, mask], axis=1)
        return result

    def _cat_encode_to_mutable(self, x):
        n = int(self._no_one_hot_mask.sum())
        result = np.zeros((x.shape[0], int(self.mutable_mask.sum())))
        result[:, self._no_one_hot_mask] = x[:, :n]
        for index, mask in enumerate(self._one_hot_masks):
            cat = x[:, n + index]
            result[:, mask] = (cat[:, None] == np.arange(mask.shape[0])[None, :]).astype(float)
        return result

    def ml_to_genetic(self, x: np.ndarray) -> np.ndarray:
        return self._mutable_to_cat_encode(self._ml_to_mutable(x))

    def genetic_to_ml(self, x: np.ndarray, x_initial_ml) -> np.ndarray:
        return self._mutable_to_ml(self._cat_encode_to_mutable(np.atleast_2d(x)), x_initial_ml)

    def normalise(self, x: np.ndarray) -> np.ndarray:
        y = np.array(x, dtype=np.float64, copy=True)
        y *= self._mm_scale
        y += self._mm_min
        return y

    def denormalize(self, x: np.ndarray) -> np.ndarray:
        y = np.array(x, dtype=np.float64, copy=True)
        y -= self._mm_min
        y /= self._mm_scale
        return y

    def get_min_max_genetic(self) -> Tuple[np.ndarray, np.ndarray]:
        """feature_encoder.py:145-163."""
        mm = np.array([self._ml_to_mutable(self._xl), self._ml_to_mutable(self._xu)])
        n = int(self._no_one_hot_mask.sum())
        result = np.empty((2, self.get_genetic_v_length()))
        result[:, :n] = mm[:, self._no_one_hot_mask]
        for index, mask in enumerate(self._one_hot_masks):
            result[:, n + index] = [0.0, mask.shape[0] - 1]
        return result[0], result[1]

    def get_genetic_v_length(self) -> int:
        return int(self._no_one_hot_mask.sum()) + len(self._one_hot_masks)

    def get_type_mask_genetic(self) -> np.ndarray:
        """feature_encoder.py:169-181."""
        n = int(self._no_one_hot_mask.sum())
        result = np.empty(self.get_genetic_v_length(), dtype=object)
        result[:n] = self._ml_to_mutable(self.type_mask)[self._no_one_hot_mask]
        result[n:] = "int"
        return result

    # -- device layout (engine extension)
    def device_layout(self):
        """gene_kind, gene_feat, ohe_offsets, ohe_feats, mut_feats for the C ABI."""
        mut_feats = np.where(self.mutable_mask)[0].astype(np.int32)
        n = int(self._no_one_hot_mask.sum())
        V = self.get_genetic_v_length()
        types = self.get_type_mask_genetic()
        kind = np.empty(V, np.int32)
        feat = np.empty(V, np.int32)
        kind[:n] = [0 if t == "real" else 1 for t in types[:n]]
        feat[:n] = mut_feats[self._no_one_hot_mask]
        offs = [0]
        ohe_feats = []
        for k, m in enumerate(self._one_hot_masks):
            kind[n + k] = 2
            feat[n + k] = k
            ohe_feats.extend(mut_feats[m].tolist())
            offs.append(len(ohe_feats))
        return kind, feat, np.asarray(offs, np.int32), np.asarray(ohe_feats, np.int32), mut_feats


def get_encoder_from_constraints(constraints: Constraints, dynamic_input=None) -> FeatureEncoder:
    """feature_encoder.py:184-193."""
    xl, xu = constraints.get_feature_min_max(dynamic_input=dynamic_input)
    return FeatureEncoder(constraints.get_mutable_mask(), constraints.get_feature_type(), xl, xu)
