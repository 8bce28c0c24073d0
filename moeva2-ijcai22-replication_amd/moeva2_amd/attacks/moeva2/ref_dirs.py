"""Riesz s-energy reference directions on the unit simplex.

Replaces ``get_reference_directions("energy", n_obj, n_pop, seed=1)``
(``src/attacks/moeva2/moeva2.py:113``), pymoo 0.4.2.2's ``RieszEnergyReferenceDirectionFactory``
(pymoo is a dependency that is not vendored in the reference).  This module implements that
published method (Blank et al. 2020, "Generating well-spaced points on a unit simplex"):

* start: the ``n_dim`` corners, then farthest-point selection over ``n_samples`` uniform
  points on the simplex, refined by k-means with the corners held (pymoo's
  ``ReductionBasedReferenceDirectionFactory(kmeans=True)``, 10 000 samples);
* objective: the Riesz energy ``E = sum_{i<j} ||x_i - x_j||^-d`` with ``d = 2 n_dim``,
  optimised as ``log E``; each point's gradient row is normalised to unit length and
  projected onto the plane ``sum(x) = 0``;
* Adam steps (alpha 0.005), every iterate projected back onto the unit simplex; the
  optimiser restarts when the energy rises; stop when the mean point movement falls below
  ``precision`` (1e-5) or after ``n_max_iter`` (1000) steps.

pymoo's own iterate sequence (its RNG stream and k-means details) cannot be reproduced
offline, so the point SET is parity-unpinned against pymoo; the method is the same.  The
arrays the engine uses are this generator's output, shipped under ``resources/ref_dirs/`` so
every run (CPU oracle or GPU) reads identical points; ``tests/test_ref_dirs_cpu.py`` checks
that regenerating them reproduces the shipped files exactly.
"""
import os

import numpy as np

_RES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))), "resources", "ref_dirs")


def simplex_projection(Y: np.ndarray) -> np.ndarray:
    """Row-wise Euclidean projection onto {x >= 0, sum(x) = 1} (sorted-threshold form)."""
    n, k = Y.shape
    desc = np.sort(Y, axis=1)[:, ::-1]
    excess = np.cumsum(desc, axis=1) - 1.0
    ks = np.arange(1, k + 1, dtype=np.float64)
    active = desc * ks > excess  # desc_j - excess_j / j > 0
    rho = k - np.argmax(active[:, ::-1], axis=1)  # number of active coordinates
    tau = excess[np.arange(n), rho - 1] / rho
    return np.maximum(Y - tau[:, None], 0.0)


def _farthest_points(S: np.ndarray, n: int, fixed: int) -> np.ndarray:
    """Indices of n rows of S: rows [0, fixed) first, then repeatedly the row farthest from
    every row chosen so far."""
    chosen = list(range(fixed))
    near = np.full(S.shape[0], np.inf)
    for c in chosen:
        near = np.minimum(near, ((S - S[c]) ** 2).sum(axis=1))
    while len(chosen) < n:
        c = int(np.argmax(near))
        chosen.append(c)
        near = np.minimum(near, ((S - S[c]) ** 2).sum(axis=1))
    return np.asarray(chosen)


def _kmeans_held(S: np.ndarray, C: np.ndarray, held: int, max_iter: int, tol: float):
    """Lloyd iterations over the samples S; centroids [0, held) stay where they are."""
    C = C.copy()
    lab = np.empty(S.shape[0], np.int64)
    for _ in range(max_iter):
        for a in range(0, S.shape[0], 2048):
            blk = S[a:a + 2048]
            lab[a:a + 2048] = ((blk[:, None, :] - C[None, :, :]) ** 2).sum(axis=2).argmin(1)
        moved = 0.0
        for j in range(held, C.shape[0]):
            m = lab == j
            if m.any():
                c = S[m].mean(axis=0)
                moved = max(moved, float(np.abs(c - C[j]).max()))
                C[j] = c
        if moved < tol:
            break
    return C


def reduction_start(n_dim: int, n_points: int, seed: int = 1, n_samples: int = 10000,
                    kmeans_max_iter: int = 1000, kmeans_tol: float = 1e-4) -> np.ndarray:
    rng = np.random.default_rng(seed)
    S = np.vstack([np.eye(n_dim), rng.dirichlet(np.ones(n_dim), size=n_samples)])
    C = S[_farthest_points(S, n_points, n_dim)]
    return _kmeans_held(S, C, n_dim, kmeans_max_iter, kmeans_tol)


def log_energy_and_grad(X: np.ndarray, d: float):
    """log(E) - log(#pairs) and the gradient of log E w.r.t. X."""
    n = X.shape[0]
    diff = X[:, None, :] - X[None, :, :]
    r = np.sqrt((diff * diff).sum(axis=2))
    np.fill_diagonal(r, np.inf)
    r = np.maximum(r, 10.0 ** (-320.0 / (d + 2.0)))  # keep r^-(d+2) finite
    inv = r ** -d
    E = inv[np.triu_indices(n, 1)].sum()
    g = (-d * (inv / (r * r))[:, :, None] * diff).sum(axis=1) / E
    return float(np.log(E) - np.log(n * (n - 1) / 2)), g


class _Adam:
    def __init__(self, alpha=0.005, b1=0.9, b2=0.999, eps=1e-16):
        self.alpha, self.b1, self.b2, self.eps = alpha, b1, b2, eps
        self.t, self.m, self.v = 0, 0.0, 0.0

    def step(self, X, g):
        self.t += 1
        self.m = self.b1 * self.m + (1.0 - self.b1) * g
        self.v = self.b2 * self.v + (1.0 - self.b2) * g * g
        mh = self.m / (1.0 - self.b1 ** self.t)
        vh = self.v / (1.0 - self.b2 ** self.t)
        return X - self.alpha * mh / (np.sqrt(vh) + self.eps)


def riesz_energy_dirs(n_dim: int, n_points: int, seed: int = 1, n_max_iter: int = 1000,
                      precision: float = 1e-5, X=None) -> np.ndarray:
    """The energy method above; ``X`` overrides the reduction start."""
    d = 2.0 * n_dim
    X = reduction_start(n_dim, n_points, seed) if X is None else np.array(X, np.float64)
    opt = _Adam()
    prev = np.inf
    for _ in range(n_max_iter):
        e, g = log_energy_and_grad(X, d)
        g = g / np.linalg.norm(g, axis=1)[:, None]
        g = g - g.mean(axis=1, keepdims=True)  # onto the plane sum(x) = 0
        Xn = simplex_projection(opt.step(X, g))
        Xn = Xn / Xn.sum(axis=1)[:, None]
        moved = np.sqrt((Xn - X) ** 2).mean(axis=1).mean()
        if moved < precision:
            break
        if e > prev:  # the energy rose: restart the optimiser
            opt = _Adam()
        prev = e
        X = Xn
    return X


def energy_ref_dirs(n_dim: int, n_points: int, seed: int = 1) -> np.ndarray:
    """Shipped array if present, else computed (and not written)."""
    path = os.path.join(_RES, f"energy_{n_dim}_{n_points}_seed{seed}.npy")
    if os.path.exists(path):
        return np.load(path, allow_pickle=False)
    return riesz_energy_dirs(n_dim, n_points, seed)


if __name__ == "__main__":  # regenerate the shipped arrays
    import time

    os.makedirs(_RES, exist_ok=True)
    for n in (200, 640):
        t = time.time()
        X = riesz_energy_dirs(3, n, seed=1)
        np.save(os.path.join(_RES, f"energy_3_{n}_seed1.npy"), X)
        print(n, "log energy", log_energy_and_grad(X, 6.0)[0], f"{time.time() - t:.1f} s")
