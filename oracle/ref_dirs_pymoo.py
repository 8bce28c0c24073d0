"""TEST INFRASTRUCTURE ONLY -- a CPU restatement of pymoo 0.4.2.2's "energy" reference
directions (Riesz s-energy, Blank et al. 2020), the method behind
``get_reference_directions("energy", n_obj, n_pop, seed=1)`` at
/root/reference/src/attacks/moeva2/moeva2.py:113.  pymoo is a third-party dependency that is
NOT vendored in the reference (and not installed here), so this follows the published
algorithm, not pymoo's source; its output is a checker for the engine's shipped directions
(tests/test_ref_dirs_cpu.py), never a product input.  Parity with pymoo's point set is
UNPINNED: its k-means initialisation and RNG stream cannot be reproduced offline.

The method, as published in pymoo's ``RieszEnergyReferenceDirectionFactory``:
  * initial points: a reduction of many uniform simplex samples -- the n_dim corners first,
    then the sample farthest from the points chosen so far, repeatedly, then k-means
    refinement with the corners held;
  * energy: E = sum_{i<j} ||x_i - x_j||^-d with d = 2 n_dim, reported as
    log(E) - log(#pairs); the gradient of log E, each row normalised to unit length and
    projected onto the plane sum(x) = 0 (so a step stays on the simplex's plane);
  * Adam steps (pymoo's util.ref_dirs.optimizer.Adam), every iterate projected back onto the
    unit simplex; stop when the mean point movement drops below ``precision``; restart the
    optimiser when the energy increases.
"""
import numpy as np


def riesz_log_energy(X: np.ndarray, d: float) -> float:
    """log( sum_{i<j} ||x_i - x_j||^-d ) - log(#pairs)."""
    diff = X[:, None, :] - X[None, :, :]
    dist = np.sqrt((diff ** 2).sum(-1))
    iu = np.triu_indices(len(X), 1)
    m = dist[iu]
    return float(np.log((1.0 / m ** d).sum()) - np.log(len(m)))


def _energy_grad(X, d):
    diff = X[:, None, :] - X[None, :, :]
    dist = np.sqrt((diff ** 2).sum(-1))
    np.fill_diagonal(dist, np.inf)
    eps = 10.0 ** (-320.0 / (d + 2))
    dist = np.maximum(dist, eps)
    iu = np.triu_indices(len(X), 1)
    energy = (1.0 / dist[iu] ** d).sum()
    grad = ((-d * diff) / (dist ** (d + 2))[..., None]).sum(1) / energy
    return float(np.log(energy) - np.log(len(iu[0]))), grad


def _project_simplex_rows(Y):
    """Euclidean projection of each row onto {x >= 0, sum x = 1} (sort-based)."""
    n, k = Y.shape
    U = -np.sort(-Y, axis=1)
    css = np.cumsum(U, axis=1) - 1.0
    idx = np.arange(1, k + 1)
    cond = U - css / idx > 0
    rho = k - 1 - np.argmax(cond[:, ::-1], axis=1)
    theta = css[np.arange(n), rho] / (rho + 1)
    return np.maximum(Y - theta[:, None], 0.0)


class _Adam:
    def __init__(self, alpha=0.005, beta_1=0.9, beta_2=0.999, epsilon=1e-16):
        self.alpha, self.b1, self.b2, self.eps = alpha, beta_1, beta_2, epsilon
        self.t, self.m, self.v = 0, 0.0, 0.0

    def next(self, X, dX):
        self.t += 1
        self.m = self.b1 * self.m + (1 - self.b1) * dX
        self.v = self.b2 * self.v + (1 - self.b2) * dX * dX
        mh = self.m / (1 - self.b1 ** self.t)
        vh = self.v / (1 - self.b2 ** self.t)
        return X - self.alpha * mh / (np.sqrt(vh) + self.eps)


def reduction_init(n_dim: int, n_points: int, rng, n_samples_per_point: int = 25,
                   kmeans_iter: int = 8) -> np.ndarray:
    """Corners + farthest-point selection over uniform simplex samples, then k-means with the
    corners held (pymoo ReductionBasedReferenceDirectionFactory(kmeans=True); fewer samples
    and k-means rounds than pymoo's defaults keep the checker fast -- it is only the start
    of the energy descent)."""
    S = rng.dirichlet(np.ones(n_dim), size=n_points * n_samples_per_point)
    S = np.vstack([np.eye(n_dim), S])
    chosen = list(range(n_dim))
    dmin = np.full(len(S), np.inf)
    for c in chosen:
        dmin = np.minimum(dmin, ((S - S[c]) ** 2).sum(1))
    while len(chosen) < n_points:
        c = int(np.argmax(dmin))
        chosen.append(c)
        dmin = np.minimum(dmin, ((S - S[c]) ** 2).sum(1))
    C = S[chosen].copy()
    for _ in range(kmeans_iter):
        lab = np.empty(len(S), np.int64)
        for s0 in range(0, len(S), 4096):  # nearest centroid, in blocks
            blk = S[s0:s0 + 4096]
            lab[s0:s0 + 4096] = ((blk[:, None, :] - C[None]) ** 2).sum(-1).argmin(1)
        for j in range(n_dim, n_points):
            m = lab == j
            if m.any():
                C[j] = S[m].mean(0)
    return C


def energy_dirs(n_dim: int, n_points: int, seed: int = 1, n_max_iter: int = 1000,
                precision: float = 1e-5, restarts: bool = True, X=None) -> np.ndarray:
    rng = np.random.default_rng(seed)
    d = 2.0 * n_dim
    X = reduction_init(n_dim, n_points, rng) if X is None else np.array(X, np.float64)
    opt = _Adam()
    obj = np.inf
    for _ in range(n_max_iter):
        _obj, grad = _energy_grad(X, d)
        grad = grad / np.linalg.norm(grad, axis=1)[:, None]
        grad = grad - grad.mean(axis=1, keepdims=True)  # onto sum(x) = 0
        _X = _project_simplex_rows(opt.next(X, grad))
        _X = _X / _X.sum(1)[:, None]
        delta = np.sqrt((_X - X) ** 2).mean(axis=1).mean()
        if delta < precision:
            break
        if restarts and _obj > obj:
            opt = _Adam()
        obj = _obj
        X = _X
    return X
