"""Run-to-run determinism of the device attack (development tool).

    python tools/determinism.py [--workload rq1.botnet.static] [--n-gen 1000] [--reps 3]

Runs the same attack (same states, seed, budget) several times, with the default state
groups and with MV_GROUPS=1, and reports whether the final populations are bit-identical.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="rq1.botnet.static")
    ap.add_argument("--n-gen", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    w = dict(bench.WORKLOADS[args.workload])
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
    runs = []
    for r in range(args.reps):
        for grp in ("", "1"):
            if grp:
                os.environ["MV_GROUPS"] = grp
            else:
                os.environ.pop("MV_GROUPS", None)
            eng.attack_run(G, P, O, 42, ref, 0.05, hm)
            genes = torch.empty((B, P, V), dtype=torch.float64, device="cuda")
            F = torch.empty((B, P, 3), dtype=torch.float64, device="cuda")
            eng.attack_population(genes, F)
            torch.cuda.synchronize()
            runs.append((f"rep{r}/groups={grp or 'default'}", genes.cpu().numpy(),
                         F.cpu().numpy()))
    import hashlib

    out = os.environ.get("DET_OUT")
    if out:
        np.save(out, np.stack([[int(hashlib.md5(runs[0][1][b].tobytes()).hexdigest()[:8], 16)
                                for b in range(B)]]))
    print(json.dumps({"digest": hashlib.md5(runs[0][1].tobytes()).hexdigest(),
                      "poison": os.environ.get("MV_POISON")}), flush=True)
    g0, f0 = runs[0][1], runs[0][2]
    for name, g, f in runs:
        diff = [b for b in range(B) if not (np.array_equal(g[b], g0[b])
                                            and np.array_equal(f[b], f0[b]))]
        print(json.dumps({"run": name, "states_differing_from_run0": len(diff),
                          "first": diff[:8]}), flush=True)


if __name__ == "__main__":
    main()
