"""CTU-13 botnet constraints (mirror of src/examples/botnet/botnet_constraints.py).

The numpy path (botnet_constraints.py:117-173, 271-309) becomes 360 device ops:
  g1, g2   |sum(icmp,udp,tcp) - sum(bytes_in, bytes_out)| per direction (:127-148)
  34       bytes_out/pkts_out - 1500 over 17 ports per direction -- the reference loops
           ``range(len(bytes_out[i]) - 2)``, i.e. the key string's length minus 2 (:299)
  324      x[lower] - x[upper] for (sum,max), (sum,min), (max,min) over 6 key triples x 18
           ports, in feat_idx key order (:123-125, :271-288)
``feat_idx`` is read from the JSON conversion of ``data/botnet/feat_idx.pickle`` (no
unpickling of shipped files).
"""
import json
from math import comb

import numpy as np

from ...attacks.moeva2.constraints import ConstraintProgram, TabularConstraints, _resolve
from ..utils import augmented_xor_program

SUM_IDX = [0, 3, 6, 12, 15, 18]
MAX_IDX = [1, 4, 7, 13, 16, 19]
MIN_IDX = [2, 5, 8, 14, 17, 20]


def botnet_program(prog: ConstraintProgram, feat_idx: dict) -> ConstraintProgram:
    fi = feat_idx
    for d in ("s", "d"):
        prog.add_sumdiff(fi[f"icmp_sum_{d}_idx"] + fi[f"udp_sum_{d}_idx"] + fi[f"tcp_sum_{d}_idx"],
                         fi[f"bytes_in_sum_{d}_idx"] + fi[f"bytes_out_sum_{d}_idx"])
    for bo, po in (("bytes_out_sum_s_idx", "pkts_out_sum_s_idx"),
                   ("bytes_out_sum_d_idx", "pkts_out_sum_d_idx")):
        for j in range(len(bo) - 2):
            prog.add("RATIO_SAFE", (fi[bo][j], fi[po][j]), (1500.0,))
    keys = list(fi.keys())
    for upper, lower in ((SUM_IDX, MAX_IDX), (SUM_IDX, MIN_IDX), (MAX_IDX, MIN_IDX)):
        for i in range(len(upper)):
            up_k, lo_k = keys[upper[i]], keys[lower[i]]
            for j in range(len(fi[keys[upper[i]]])):
                prog.add("DIFF", (fi[lo_k][j], fi[up_k][j]))
    return prog


def load_feat_idx(feature_path: str) -> dict:
    with open(_resolve(feature_path, "feat_idx.json")) as f:
        return json.load(f)


class BotnetConstraints(TabularConstraints):
    def __init__(self, feature_path: str, constraints_path: str):
        super().__init__(feature_path, constraints_path)
        self.feat_idx = load_feat_idx(feature_path)
        self.important_features = np.load(_resolve(feature_path, "important_features_19.npy"),
                                          allow_pickle=False)

    def fix_features_types(self, x):
        return x  # botnet_constraints.py:14-15

    def device_program(self) -> ConstraintProgram:
        return botnet_program(ConstraintProgram(), self.feat_idx)

    def get_nb_constraints(self) -> int:
        return 360


class BotnetAugmentedConstraints(TabularConstraints):
    """botnet_augmented_constraints.py: the 360 botnet columns + C(19,2) XOR columns."""

    def __init__(self, feature_path: str, constraints_path: str, import_features_path=None):
        super().__init__(feature_path, constraints_path)
        self.feat_idx = load_feat_idx(feature_path)
        if import_features_path is None:
            import_features_path = _resolve(feature_path, "important_features_19.npy")
        self.important_features = np.load(import_features_path, allow_pickle=False)

    def device_program(self) -> ConstraintProgram:
        prog = botnet_program(ConstraintProgram(), self.feat_idx)
        return augmented_xor_program(prog, self._feature_type.shape[0],
                                     self.important_features[:, 0], self.important_features[:, 1])

    def get_nb_constraints(self) -> int:
        return 360 + comb(len(self.important_features), 2)
