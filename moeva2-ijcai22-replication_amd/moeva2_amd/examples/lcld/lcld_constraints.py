"""LCLD domain constraints (mirror of src/examples/lcld/lcld_constraints.py).

The numpy path (``evaluate_numpy``, lcld_constraints.py:168-223) becomes a 10-op device
program; feature indices are the ones the reference hard-codes.
"""
import numpy as np

from ...attacks.moeva2.constraints import ConstraintProgram, TabularConstraints, _resolve


def lcld_program(prog: ConstraintProgram) -> ConstraintProgram:
    prog.add("LCLD_INSTALL", (0, 1, 2, 3), (0.099999,))  # g41 :174-177
    prog.add("DIFF", (10, 14))  # g42 open_acc <= total_acc :180
    prog.add("DIFF", (16, 11))  # g43 pub_rec_bankruptcies <= pub_rec :183
    prog.add("LCLD_TERM", (1,))  # g44 term in {36, 60} :186
    prog.add("ABS_RATIO", (20, 0, 6))  # g45 ratio_loan_amnt_annual_inc :189
    prog.add("ABS_RATIO", (21, 10, 14))  # g46 ratio_open_acc_total_acc :192
    prog.add("MONTHDIFF", (22, 7, 9))  # g47 diff_issue_d_earliest_cr_line :195-201
    prog.add("ABS_RATIO", (23, 11, 22))  # g48 :204
    prog.add("ABS_RATIO", (24, 16, 22))  # g49 :207
    prog.add("RATIO_MASKED", (25, 16, 11))  # g410 :210-216
    return prog


class LcldConstraints(TabularConstraints):
    def __init__(self, feature_path: str, constraints_path: str):
        super().__init__(feature_path, constraints_path)
        self.important_features = np.load(_resolve(feature_path, "important_features.npy"),
                                          allow_pickle=False)

    @staticmethod
    def _date_feature_to_month(feature):
        return np.floor(feature / 100) * 12 + (feature % 100)

    def device_program(self) -> ConstraintProgram:
        return lcld_program(ConstraintProgram())

    def get_nb_constraints(self) -> int:
        return 10
