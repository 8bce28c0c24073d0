"""Project loaders for the oracle -- TEST INFRASTRUCTURE ONLY.

Reads the repo's converted copies of the reference data (resources/, written by
tools/import_reference_data.py) and builds oracle ``Problem`` objects exactly as
``Moeva2._one_generate`` builds ``DefaultProblem`` (src/attacks/moeva2/moeva2.py:141-154).
"""
import json
import os

import numpy as np
import pandas as pd

try:
    from . import moeva_oracle as mo
except ImportError:  # pragma: no cover
    import moeva_oracle as mo

RES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "moeva2-ijcai22-replication_amd", "resources")

PROJECTS = {
    # name: (features csv, model npz, scaler npz, candidates npy, important features)
    "lcld": ("data/lcld/features.csv", "models/lcld/nn.npz", "models/lcld/scaler.npz",
             "data/lcld/x_candidates_synthetic.npy", "data/lcld/important_features.npy"),
    "lcld_augmented": ("data/lcld/features_augmented.csv",
                       "models/lcld/nn_augmented_moeva_best.npz",
                       "models/lcld/scaler_augmented.npz",
                       "data/lcld/x_candidates_synthetic_augmented.npy",
                       "data/lcld/important_features.npy"),
    "botnet": ("data/botnet/features.csv", "models/botnet/nn.npz", "models/botnet/scaler.npz",
               "data/botnet/x_candidates_common.npy", "data/botnet/important_features_19.npy"),
    "botnet_augmented": ("data/botnet/features_augmented_19.csv",
                         "models/botnet/nn_augmented_19.npz",
                         "models/botnet/scaler_augmented_19.npz",
                         "data/botnet/x_candidates_common_augmented.npy",
                         "data/botnet/important_features_19.npy"),
}


def read_features(path):
    """pandas.read_csv exactly like lcld_constraints.py:268-273 (its C float parser is not
    always correctly rounded; the reference's bounds are whatever it returns)."""
    df = pd.read_csv(path, low_memory=False)
    return (df["type"].to_numpy(), df["mutable"].to_numpy().astype(bool),
            df["min"].to_numpy(), df["max"].to_numpy())


class Project:
    def __init__(self, name):
        feat, model, scaler, cand, imp = PROJECTS[name]
        self.name = name
        self.types, self.mutable, self.fmin, self.fmax = read_features(os.path.join(RES, feat))
        m = np.load(os.path.join(RES, model))
        self.weights = [m[f"W{i}"] for i in range(4)]
        self.biases = [m[f"b{i}"] for i in range(4)]
        s = np.load(os.path.join(RES, scaler))
        self.ml = (s["scale_"], s["min_"])
        self.x = np.load(os.path.join(RES, cand))
        self.important = np.load(os.path.join(RES, imp))
        self.lay = mo.make_layout(self.mutable, self.types)
        if name.startswith("botnet"):
            with open(os.path.join(RES, "data/botnet/feat_idx.json")) as f:
                self.feat_idx = json.load(f)
        if name == "lcld":
            self.constraints = mo.lcld_constraints
        elif name == "lcld_augmented":
            self.constraints = lambda x: mo.lcld_augmented_constraints(x, self.important)
        elif name == "botnet":
            self.constraints = lambda x: mo.botnet_constraints(x, self.feat_idx)
        else:
            self.constraints = lambda x: mo.botnet_augmented_constraints(x, self.feat_idx,
                                                                         self.important)

    def problem(self, x_init, norm=2, minimize_class=1):
        return mo.make_problem(self.lay, x_init, self.fmin, self.fmax, self.ml, self.weights,
                               self.biases, self.constraints, minimize_class, norm, True)
