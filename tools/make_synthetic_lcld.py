"""Generate synthetic LCLD initial states (the reference's LCLD candidate files are missing:
``/root/reference/.MISSING_LARGE_BLOBS:1-6``).

Each state satisfies all 10 LCLD constraints exactly as the reference evaluates them
(``src/examples/lcld/lcld_constraints.py:168-223``), lies inside the ML scaler's fitted
range (so ``ObjectiveCalculator``'s [0,1] asserts hold, objective_calculator.py:72-76),
and is classified as class 1 with probability >= the rq1 threshold 0.25
(``config/rq1.lcld.static.yaml``) by the shipped model, so the attack has work to do.
The augmented variant applies ``augment_data`` (``src/experiments/botnet/features.py:6-21``)
and is filtered with the augmented model (``config/rq4.lcld.moeva_augmented.yaml``).

    python tools/make_synthetic_lcld.py   -> resources/data/lcld/x_candidates_synthetic*.npy
"""
import os
from itertools import combinations

import numpy as np

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "moeva2-ijcai22-replication_amd", "resources")


def _month(f):
    return np.floor(f / 100) * 12 + (f % 100)


def raw_states(rng, n):
    x = np.zeros((n, 47))
    x[:, 0] = rng.integers(40, 1600, n) * 25.0  # loan_amnt 1000..40000
    x[:, 1] = rng.choice([36.0, 60.0], n, p=[0.7, 0.3])
    x[:, 2] = np.round(rng.uniform(5.31, 30.99, n), 2)
    r = x[:, 2] / 1200
    x[:, 3] = (x[:, 0] * r * (1 + r) ** x[:, 1]) / ((1 + r) ** x[:, 1] - 1)  # exact identity
    x[:, 4] = rng.integers(1, 8, n)
    x[:, 5] = rng.integers(0, 11, n)
    x[:, 6] = np.round(rng.uniform(15000, 250000, n), 0)
    year = rng.integers(2012, 2019, n)
    month = rng.integers(1, 13, n)
    month = np.where(year == 2012, np.maximum(month, 3), month)
    x[:, 7] = year * 100 + month
    x[:, 8] = np.round(rng.uniform(0, 40, n), 2)
    cy = rng.integers(1965, 2009, n)
    cm = rng.integers(1, 13, n)
    x[:, 9] = cy * 100 + cm
    x[:, 10] = rng.integers(1, 35, n)
    x[:, 11] = rng.choice([0.0, 0.0, 0.0, 1.0, 2.0], n)
    x[:, 12] = np.round(rng.uniform(0, 60000, n), 0)
    x[:, 13] = np.round(rng.uniform(0, 100, n), 1)
    x[:, 14] = x[:, 10] + rng.integers(0, 40, n)
    x[:, 15] = rng.integers(0, 6, n)
    x[:, 16] = np.minimum(x[:, 11], rng.integers(0, 2, n))
    x[:, 17] = rng.choice(np.arange(662.0, 848.0, 5.0), n)
    x[:, 18] = rng.integers(0, 2, n)
    x[:, 19] = (rng.uniform(size=n) < 0.05).astype(float)
    x[:, 20] = x[:, 0] / x[:, 6]
    x[:, 21] = x[:, 10] / x[:, 14]
    x[:, 22] = _month(x[:, 7]) - _month(x[:, 9])
    x[:, 23] = x[:, 11] / x[:, 22]
    x[:, 24] = x[:, 16] / x[:, 22]
    x[:, 25] = np.where(x[:, 11] != 0, x[:, 16] / np.where(x[:, 11] != 0, x[:, 11], 1), -1.0)
    x[np.arange(n), 26 + rng.integers(0, 4, n)] = 1.0
    x[np.arange(n), 30 + rng.integers(0, 3, n)] = 1.0
    x[np.arange(n), 33 + rng.integers(0, 14, n)] = 1.0
    return x


def augment(x, imp):
    nf = [np.logical_xor(x[:, int(imp[a, 0])] >= imp[a, 1], x[:, int(imp[b, 0])] >= imp[b, 1])
          .astype(np.float64) for a, b in combinations(range(imp.shape[0]), 2)]
    return np.concatenate([x, np.column_stack(nf)], axis=1)


def proba1(x, model, scaler):
    m = np.load(model)
    s = np.load(scaler)
    h = (x * s["scale_"] + s["min_"]).astype(np.float32)
    for i in range(4):
        h = h @ m[f"W{i}"] + m[f"b{i}"]
        if i < 3:
            h = np.maximum(h, 0)
    h = h - h.max(1, keepdims=True)
    e = np.exp(h)
    return (e / e.sum(1, keepdims=True))[:, 1]


def in_range(x, scaler):
    s = np.load(scaler)
    z = x * s["scale_"] + s["min_"]
    return np.all((z >= 0) & (z <= 1), axis=1)


def main(n_target=4000, seed=20221):
    rng = np.random.default_rng(seed)
    imp = np.load(os.path.join(PKG, "data/lcld/important_features.npy"))
    mdl = os.path.join(PKG, "models/lcld")
    keep, keep_aug = [], []
    while min(sum(len(k) for k in keep), sum(len(k) for k in keep_aug)) < n_target:
        x = raw_states(rng, 20000)
        ok = in_range(x, f"{mdl}/scaler.npz")
        p = proba1(x, f"{mdl}/nn.npz", f"{mdl}/scaler.npz")
        keep.append(x[ok & (p >= 0.25)])
        xa = augment(x, imp)
        oka = in_range(xa, f"{mdl}/scaler_augmented.npz")
        pa = proba1(xa, f"{mdl}/nn_augmented_moeva_best.npz", f"{mdl}/scaler_augmented.npz")
        keep_aug.append(xa[oka & (pa >= 0.25)])
    x = np.concatenate(keep)[:n_target]
    xa = np.concatenate(keep_aug)[:n_target]
    np.save(os.path.join(PKG, "data/lcld/x_candidates_synthetic.npy"), x)
    np.save(os.path.join(PKG, "data/lcld/x_candidates_synthetic_augmented.npy"), xa)
    print("lcld", x.shape, "aug", xa.shape)


if __name__ == "__main__":
    main()
