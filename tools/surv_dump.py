"""Checks build only: run the botnet rq1 attack (387 states x 1000 generations, seed 1000 --
the first device seed of tests/test_gpu_e2e.py) until a survival picks duplicate survivors
(device check 26), then save that state's survival inputs (mv_debug_survival_dump) and the
check record to gpurun_out/fault/surv_dump.npz for a CPU replay against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "moeva2-ijcai22-replication_amd")]

import torch  # noqa: E402

from moeva2_amd import _native  # noqa: E402
from test_gpu_e2e import NpScaler  # noqa: E402
from conftest import RES  # noqa: E402
from oracle.problems import PROJECTS, Project  # noqa: E402


def main():
    from moeva2_amd.attacks.moeva2.classifier import Classifier, load_model
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs
    from moeva2_amd.experiments.united.utils import STR_TO_CONSTRAINTS_CLASS
    from moeva2_amd.problem import get_engine

    name, B, G = "botnet", 387, int(os.environ.get("DUMP_GENS", "1000"))
    seeds = [int(s) for s in os.environ.get("DUMP_SEEDS", "1000").split(",")]
    p = Project(name)
    X = p.x[:B]
    feat = os.path.join(RES, PROJECTS[name][0])
    c = STR_TO_CONSTRAINTS_CLASS[name](feat, feat.replace("features", "constraints"))
    eng = get_engine(c, Classifier(load_model(os.path.join(RES, PROJECTS[name][1]))),
                     NpScaler(os.path.join(RES, PROJECTS[name][2])), 2)
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    ref = energy_ref_dirs(3, 200, seed=1)
    out = os.path.join(ROOT, "gpurun_out", "fault")
    os.makedirs(out, exist_ok=True)
    for s in seeds:
        eng.attack_run(G, 203, 100, s, ref, 0.05, 0)
        on, rec = _native.debug_checks()
        dump = _native.debug_survival_dump()
        print("seed", s, "checks", on, rec, "dump valid", dump[0], flush=True)
        if rec[0] or dump[0]:
            groups = max(1, min(4, B // 64))
            np.savez(os.path.join(out, f"surv_dump_s{s}.npz"), record=np.array(rec), dump=dump,
                     ref=ref, seed=s, groups=groups, group_b0=np.array(
                         [B * q // groups for q in range(groups + 1)]))


if __name__ == "__main__":
    main()
