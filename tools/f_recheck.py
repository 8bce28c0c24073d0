"""Development check: the device attack's final populations re-evaluated by the oracle's
numpy-order DefaultProblem._evaluate restatement; reports how far the device F is from it
(beyond ulps = a semantic difference on evolved individuals the golden vectors miss).

    python tools/f_recheck.py [seed] [n_gen] [n_states]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_parity as T  # noqa: E402
from oracle import moeva_oracle as mo  # noqa: E402
from oracle.problems import Project  # noqa: E402


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 387
    p = Project("botnet")
    X = p.x[:B]
    _, g, F, _, _ = T._attack("botnet", X, G, seed, P=203, O=100)
    g, F = g.cpu().numpy(), F.cpu().numpy()
    worst = np.zeros(3)
    bad = [0, 0, 0]
    rel = []
    for b in range(B):
        ref = mo.evaluate(p.problem(X[b]), g[b])
        d = np.abs(F[b] - ref)
        r = d / np.maximum(np.abs(ref), 1e-30)
        rel.append(r.max(axis=0))
        worst = np.maximum(worst, d.max(axis=0))
        tol = [1e-5, 1e-12, 1e-12]
        for k in range(3):
            m = d[:, k] > tol[k] * np.maximum(np.abs(ref[:, k]), 1.0)
            bad[k] += int(m.sum())
            if m.any() and bad[k] <= 5:
                i = int(np.argmax(m))
                print(f"state {b} row {i} obj {k}: device {F[b][i, k]!r} oracle {ref[i, k]!r}")
    rel = np.array(rel)
    print("max abs diff per objective", worst, "rows beyond tol", bad)
    print("max rel diff per objective", rel.max(axis=0))
    print("f1 == 1.0 rows device", int((F[:, :, 0] == 1.0).sum()), "f1 == 0 rows", int((F[:, :, 0] == 0).sum()))


if __name__ == "__main__":
    main()
