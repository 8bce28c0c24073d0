"""Development check: first generation at which the device attack and the engine-order
oracle attack (oracle/device_order.py) part, per state, and what differs there.

    python tools/traj_diff.py lcld 16 20
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    from conftest import RES  # noqa: F401  (sys.path of the package)
    from oracle import device_order as do
    from oracle import moeva_oracle as mo
    from oracle.problems import Project
    from test_gpu_parity import _attack, make_constraints
    from moeva2_amd.problem import build_device_program

    name = sys.argv[1] if len(sys.argv) > 1 else "lcld"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    Gmax = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    P, O, seed = 43, 20, 9
    p = Project(name)
    X = p.x[:B]
    codes = build_device_program(make_constraints(name)).op_code

    def ev(prob, gg, return_g=False):
        return do.evaluate_device_order(prob, gg, codes, return_g)

    first = [None] * B
    for G in range(1, Gmax + 1):
        _, g, F, _, ref = _attack(name, X, G, seed, P=P, O=O)
        genes, Fd = g.cpu().numpy(), F.cpu().numpy()
        for b in range(B):
            if first[b] is not None:
                continue
            r = mo.run_attack(p.problem(X[b]), ref, G, P, O, seed, evaluate_fn=ev)
            if not (np.array_equal(r.pop_X, genes[b]) and np.array_equal(r.pop_F, Fd[b])):
                first[b] = G
                sd = set(map(tuple, genes[b]))
                so = set(map(tuple, r.pop_X))
                print(f"state {b}: parts at G={G}; rows only on device {len(sd - so)}, only "
                      f"in oracle {len(so - sd)}; same row set {sd == so}", flush=True)
                if sd == so:
                    print("   order differs only")
                else:
                    # F of a shared row that differs
                    for i in range(P):
                        k = np.where((r.pop_X == genes[b][i]).all(1))[0]
                        if k.size and not np.array_equal(r.pop_F[k[0]], Fd[b][i]):
                            print("   same genes, F device", Fd[b][i], "oracle", r.pop_F[k[0]],
                                  "diff", Fd[b][i] - r.pop_F[k[0]])
                            break
                    # the oracle's generation G-1 step from the agreed population
                    prob = p.problem(X[b])
                    r0 = mo.run_attack(prob, ref, G - 1, P, O, seed, evaluate_fn=ev)
                    types = mo.genetic_types(p.lay)
                    gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
                    masks = [np.array([t == "real" for t in types]),
                             np.array([t == "int" for t in types])]
                    gg = G - 1
                    par = mo.tournament_parents(P, O, seed, gg)
                    pX = np.stack([r0.pop_X[par[:, 0]], r0.pop_X[par[:, 1]]])
                    off = mo.crossover(pX, masks, seed, gg)[:O]
                    offm = mo.mutation(off, gl, gu, types, seed, gg)
                    so_off = set(map(tuple, offm))
                    donly = [x for x in genes[b] if tuple(x) not in so]
                    print("   device-only rows among the oracle's offspring:",
                          [tuple(x) in so_off for x in donly])
                    for x in donly[:1]:
                        # nearest oracle offspring (genes differing)
                        dd = np.abs(offm - x).sum(1)
                        k = int(dd.argmin())
                        diff = np.where(offm[k] != x)[0]
                        print("   nearest oracle child", k, "differs at genes", diff,
                              "device", x[diff], "oracle", offm[k][diff], "crossed",
                              off[k][diff], "parents", pX[0][k % ((O + 1) // 2)][diff] if False else "")
                    # an evaluation of the device-only rows by the oracle
                    only = np.array([x for x in genes[b] if tuple(x) not in so])[:2]
                    if only.size:
                        Fo = ev(p.problem(X[b]), only)
                        idx = [int(np.where((genes[b] == x).all(1))[0][0]) for x in only]
                        print("   device-only rows F device", Fd[b][idx], "oracle eval", Fo)
        if all(f is not None for f in first):
            break
    print("first parting generation per state:", first)


if __name__ == "__main__":
    main()
