"""Debug: replay the oracle attack with the device's objective values; first mismatch."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
from test_gpu_parity import _attack
from oracle import moeva_oracle as mo
from oracle.problems import Project

p = Project("lcld")
B, P, O, seed, GM = 4, 43, 20, 7, 6
X = p.x[:B]
_, _, _, H, ref = _attack("lcld", X, GM, seed, hist=1, P=P, O=O)
H = H.cpu().numpy()
dev = {}
for G in range(1, GM + 1):
    _, g, F, _, _ = _attack("lcld", X, G, seed, P=P, O=O)
    dev[G] = (g.cpu().numpy(), F.cpu().numpy())
for b in range(B):
    prob = p.problem(X[b])
    asp = np.full((1, 3), 1.0 / 3.0)
    gl, gu = mo.genetic_bounds(prob.lay, prob.xl, prob.xu)
    types = mo.genetic_types(prob.lay)
    masks = [np.array([t == "real" for t in types]), np.array([t == "int" for t in types])]
    Xp = mo.initial_population(prob, P)
    Fp = H[b, :P].copy()
    st = mo.SurvivalState()
    r = mo.survive(Fp, P, st, ref, asp, 0.05, seed, 0)
    Xp, Fp = Xp[r.survivors], Fp[r.survivors]
    print(f"b={b} G=1 genes_eq={np.array_equal(Xp, dev[1][0][b])} F_eq={np.array_equal(Fp, dev[1][1][b])}")
    for gg in range(1, GM):
        par = mo.tournament_parents(P, O, seed, gg)
        pX = np.stack([Xp[par[:, 0]], Xp[par[:, 1]]])
        off = mo.crossover(pX, masks, seed, gg)[:O]
        off = mo.mutation(off, gl, gu, types, seed, gg)
        Fh = H[b, P + (gg - 1) * O: P + gg * O]
        mX = np.concatenate([Xp, off])
        mF = np.concatenate([Fp, Fh])
        r = mo.survive(mF, P, st, ref, asp, 0.05, seed, gg)
        Xp, Fp = mX[r.survivors], mF[r.survivors]
        dg, dF = dev[gg + 1][0][b], dev[gg + 1][1][b]
        ge, fe = np.array_equal(Xp, dg), np.array_equal(Fp, dF)
        print(f"b={b} G={gg+1} genes_eq={ge} F_eq={fe}", flush=True)
        if not (ge and fe):
            rows = [int(np.nonzero(np.all(dg == x, axis=1))[0][0]) if np.any(np.all(dg == x, axis=1)) else -1 for x in Xp]
            print("  oracle survivor -> device position:", rows)
            print("  F rows equal where genes found:", all(np.array_equal(Fp[i], dF[j]) for i, j in enumerate(rows) if j >= 0))
            for i, j in enumerate(rows):
                if j < 0:
                    d = dg[i]
                    x = Xp[i]
                    bad = np.nonzero(~((d == x) | (np.isnan(d) & np.isnan(x))))[0]
                    print("  row", i, "nan_dev", np.isnan(d).sum(), "nan_or", np.isnan(x).sum(),
                          "diff cols", bad, "dev", d[bad], "oracle", x[bad])
            break
