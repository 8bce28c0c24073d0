"""Riesz s-energy reference directions on the unit simplex.

Replaces ``get_reference_directions("energy", n_obj, n_pop, seed=1)``
(``src/attacks/moeva2/moeva2.py:113``; pymoo 0.4.2.2's energy factory, not vendored
in the reference).  pymoo's exact iterate sequence cannot be reproduced offline, so
parity with pymoo's point set is UNPINNED; what is kept is the method: start from
random points on the simplex, minimise the Riesz s-energy
``sum_{i<j} ||x_i - x_j||^-s`` with projected Adam steps, project back onto the
simplex.  The arrays used by the engine are generated once and shipped under
``resources/ref_dirs/`` so every run (CPU oracle or GPU) sees identical points.
"""
import os

import numpy as np

_RES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))), "resources", "ref_dirs")


def _project_simplex(X):
    X = np.maximum(X, 0.0)
    return X / X.sum(axis=1, keepdims=True)


def riesz_energy_dirs(n_dim: int, n_points: int, seed: int = 1, n_iter: int = 1500,
                      s: float = None, lr: float = 5e-3) -> np.ndarray:
    s = float(2 * n_dim - 1) if s is None else s
    rng = np.random.default_rng(seed)
    X = rng.dirichlet(np.ones(n_dim), size=n_points)
    X[:n_dim] = np.eye(n_dim)  # keep the corners: the extreme directions
    m = np.zeros_like(X)
    v = np.zeros_like(X)
    b1, b2 = 0.9, 0.999
    for t in range(1, n_iter + 1):
        diff = X[:, None, :] - X[None, :, :]
        d2 = (diff ** 2).sum(-1)
        np.fill_diagonal(d2, np.inf)
        w = d2 ** (-(s + 2) / 2)
        grad = -s * (w[:, :, None] * diff).sum(1)
        grad /= np.abs(grad).max() + 1e-300
        grad -= grad.mean(axis=1, keepdims=True)  # stay on the plane sum(x)=1
        grad[:n_dim] = 0.0
        m = b1 * m + (1 - b1) * grad
        v = b2 * v + (1 - b2) * grad ** 2
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        X = _project_simplex(X - lr * mh / (np.sqrt(vh) + 1e-8))
    return X


def energy_ref_dirs(n_dim: int, n_points: int, seed: int = 1) -> np.ndarray:
    """Shipped array if present, else computed (and not written)."""
    path = os.path.join(_RES, f"energy_{n_dim}_{n_points}_seed{seed}.npy")
    if os.path.exists(path):
        return np.load(path, allow_pickle=False)
    return riesz_energy_dirs(n_dim, n_points, seed)


if __name__ == "__main__":
    os.makedirs(_RES, exist_ok=True)
    for n in (200, 640):
        X = riesz_energy_dirs(3, n, seed=1)
        np.save(os.path.join(_RES, f"energy_3_{n}_seed1.npy"), X)
        d = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1))
        np.fill_diagonal(d, np.inf)
        print(n, "min pairwise distance", d.min(), "sum", X.sum(1).min(), X.sum(1).max())
