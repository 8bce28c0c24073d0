"""A/B timing of the attack modes on one GPU (development tool).

    python tools/attack_ab.py [--workload rq1.botnet.static] [--n-gen 1000] [--reps 3]

Times mv_attack_run in the whole-attack mode (one k_attack launch) and in the per-phase
chain mode on the bench workload, checks that both give identical final populations, and
prints one JSON line per mode.
"""
import argparse
import json
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
    ap.add_argument("--n-gen", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="whole,chain")
    args = ap.parse_args()
    import torch

    w = dict(bench.WORKLOADS[args.workload])
    if args.n_gen:
        w["n_gen"] = args.n_gen
    from moeva2_amd.attacks.moeva2.moeva2 import history_mode
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    eng, c = bench.build_engine(w, 0)
    X = bench.load_states(w)
    B = X.shape[0]
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O, G = w["n_pop"] + 3, w["n_off"], w["n_gen"]
    hm = history_mode(w["history"])
    V = eng.prog.V
    outs = {}
    for mode in args.modes.split(","):
        eng.set_attack_mode(mode)
        genes = torch.empty((B, P, V), dtype=torch.float64, device="cuda")
        F = torch.empty((B, P, 3), dtype=torch.float64, device="cuda")
        eng.attack_run(G, P, O, 42, ref, 0.05, hm)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.attack_run(G, P, O, 42, ref, 0.05, hm)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        eng.attack_population(genes, F)
        torch.cuda.synchronize()
        eng.set_profiling(True)
        eng.attack_run(G, P, O, 42, ref, 0.05, hm)
        torch.cuda.synchronize()
        ms, whole = eng.attack_time()
        eng.set_profiling(False)
        outs[mode] = (genes.cpu().numpy(), F.cpu().numpy())
        print(json.dumps({"mode": mode, "whole_kernel": whole, "workload": args.workload,
                          "states": B, "n_gen": G, "s_per_attack": dt,
                          "evals_per_s": B * (P + (G - 1) * O) / dt,
                          "k_attack_ms": ms}), flush=True)
    ms = list(outs)
    if len(ms) == 2:
        same = all(np.array_equal(a, b) for a, b in zip(outs[ms[0]], outs[ms[1]]))
        print(json.dumps({"identical_populations": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
