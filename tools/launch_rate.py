"""Host enqueue time vs device time of one attack (development tool): is the chain
launch-bound?  python tools/launch_rate.py [--n-gen 200] [--groups G]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="rq1.botnet.static")
    ap.add_argument("--n-gen", type=int, default=200)
    args = ap.parse_args()
    import torch

    w = dict(bench.WORKLOADS[args.workload])
    w["n_gen"] = args.n_gen
    from moeva2_amd.attacks.moeva2.moeva2 import history_mode
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    eng, c = bench.build_engine(w, 0)
    X = bench.load_states(w)
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O, G = w["n_pop"] + 3, w["n_off"], w["n_gen"]
    hm = history_mode(w["history"])
    for groups in ("1", "2", "3", "4"):
        os.environ["MV_GROUPS"] = groups
        eng.attack_run(G, P, O, 42, ref, 0.05, hm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.attack_run(G, P, O, 42, ref, 0.05, hm)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"groups={groups} enqueue {1e3 * (t1 - t0):.1f} ms, total {1e3 * (t2 - t0):.1f} ms,"
              f" per generation {1e6 * (t2 - t0) / G:.1f} us", flush=True)


if __name__ == "__main__":
    main()
