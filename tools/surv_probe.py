"""Development probe: per-kernel device times per generation (one state group) and the
survival phase split, on the first n botnet states, for several n.

    MV_SURV_PHASES=1 python tools/surv_probe.py 64 128 256 387
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "moeva2-ijcai22-replication_amd"))
os.environ.setdefault("MV_GROUPS", "1")

import torch  # noqa: E402

import bench  # noqa: E402
from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs  # noqa: E402


def main():
    w = dict(bench.WORKLOADS[os.environ.get("WORKLOAD", "rq1.botnet.static")])
    G = int(os.environ.get("GENS", "50"))
    eng, c = bench.build_engine(w, 0)
    X_all = bench.load_states(w)
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O = w["n_pop"] + 3, w["n_off"]
    for n in [int(a) for a in sys.argv[1:]] or [387]:
        X = np.resize(X_all, (n, X_all.shape[1]))
        bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
        eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
        eng.attack_run(G, P, O, 42, ref, 0.05, 1)  # warm
        torch.cuda.synchronize()
        eng.set_profiling(True)
        eng.attack_run(G, P, O, 42, ref, 0.05, 1)
        torch.cuda.synchronize()
        kt = eng.kernel_times()
        eng.set_profiling(False)
        g = max(kt["generations"], 1)
        print(f"n={n}: us/gen k_gen {1e3 * kt['gen_ms'] / g:.1f} k_cons {1e3 * kt['cons_ms'] / g:.1f} "
              f"k_mlp {1e3 * kt['mlp_ms'] / g:.1f} k_survive {1e3 * kt['survive_ms'] / g:.1f}",
              flush=True)


if __name__ == "__main__":
    main()
