"""CPU restatement of the MoEvA2 hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for the HIP engine in
``moeva2-ijcai22-replication_amd/csrc``.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path never does.

Every function cites the reference file:line it restates (paths relative to the
reference repository root).  Items marked [pymoo-recall] restate pymoo 0.4.2.2
(``requirements.txt:5``), which is NOT vendored in the reference: their parity
against pymoo itself is UNPINNED.  The only pymoo code the
reference carries in-repo -- the dominance relation (``pareto_operation.py:148-164``
numbering of the file as shipped: ``calc_domination_matrix``), two-point crossover
(``softmax_crossover.py:17-38``) and polynomial mutation (``softmax_mutation.py:20-67``)
-- is pinned by golden vectors generated from those files (tests/golden).

Random draws: the reference uses numpy's MT19937; this oracle (and the kernels)
use Philox4x32-10 with the counter layout in ``oracle/philox.py``.  Functions that
consume randomness take the draws (or a Philox stream) explicitly so the same code
path can be pinned against the reference's np.random order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from itertools import combinations
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

try:  # allow both `import oracle.moeva_oracle` and a flat sys.path
    from . import philox as px
except ImportError:  # pragma: no cover
    import philox as px

TOL = 1e-3  # lcld_constraints.py:171, botnet_constraints.py:120


# --------------------------------------------------------------------------------------
# A. sklearn MinMaxScaler semantics (sklearn 0.24.1, requirements.txt:7)
# --------------------------------------------------------------------------------------
def minmax_fit(data_min: np.ndarray, data_max: np.ndarray):
    """``MinMaxScaler().fit([xl, xu])``: scale_ = 1/range (range 0 -> 1), min_ = -xl*scale_.

    Used by FeatureEncoder (feature_encoder.py:39-40) and get_scaler_from_norm (utils.py:11-22).
    """
    data_min = np.asarray(data_min, dtype=np.float64)
    data_max = np.asarray(data_max, dtype=np.float64)
    lo = np.minimum(data_min, data_max)
    hi = np.maximum(data_min, data_max)
    rng = hi - lo
    rng = np.where(rng == 0.0, 1.0, rng)
    scale = 1.0 / rng
    mn = 0.0 - lo * scale
    return scale, mn


def minmax_transform(x, scale, mn):
    x = np.array(x, dtype=np.float64, copy=True)
    x *= scale
    x += mn
    return x


# --------------------------------------------------------------------------------------
# B. FeatureEncoder (src/attacks/moeva2/feature_encoder.py)
# --------------------------------------------------------------------------------------
@dataclass
class GeneticLayout:
    mutable_mask: np.ndarray  # (D,) bool
    type_mask: np.ndarray  # (D,) object: 'real' | 'int' | 'ohe<k>'
    ohe_masks: List[np.ndarray]  # indices into the MUTABLE sub-vector
    no_ohe_mask: np.ndarray  # over the mutable sub-vector

    @property
    def V(self) -> int:
        return int(self.no_ohe_mask.sum()) + len(self.ohe_masks)

    @property
    def D(self) -> int:
        return self.mutable_mask.shape[0]


def make_layout(mutable_mask, type_mask) -> GeneticLayout:
    """feature_encoder.py:58-86 ``_create_one_hot_encoders``."""
    mutable_mask = np.asarray(mutable_mask, dtype=bool)
    type_mask = np.asarray(type_mask, dtype=object)
    mt = type_mask[mutable_mask]
    seen: List[str] = []
    masks: List[List[int]] = []
    for i, t in enumerate(mt):
        if str(t).startswith("ohe"):
            if t in seen:
                masks[seen.index(t)].append(i)
            else:
                seen.append(t)
                masks.append([i])
    ohe = [np.array(m) for m in masks]
    no = np.ones(mt.shape[0], dtype=bool)
    for m in ohe:
        no[m] = False
    return GeneticLayout(mutable_mask, type_mask, ohe, no)


def genetic_bounds(lay: GeneticLayout, xl, xu):
    """feature_encoder.py:145-163 ``get_min_max_genetic``."""
    mxl = np.asarray(xl, np.float64)[lay.mutable_mask]
    mxu = np.asarray(xu, np.float64)[lay.mutable_mask]
    n = int(lay.no_ohe_mask.sum())
    gl = np.empty(lay.V)
    gu = np.empty(lay.V)
    gl[:n] = mxl[lay.no_ohe_mask]
    gu[:n] = mxu[lay.no_ohe_mask]
    for k, m in enumerate(lay.ohe_masks):
        gl[n + k] = 0.0
        gu[n + k] = m.shape[0] - 1
    return gl, gu


def genetic_types(lay: GeneticLayout) -> np.ndarray:
    """feature_encoder.py:169-181 ``get_type_mask_genetic``."""
    mt = lay.type_mask[lay.mutable_mask]
    n = int(lay.no_ohe_mask.sum())
    out = np.empty(lay.V, dtype=object)
    out[:n] = mt[lay.no_ohe_mask]
    out[n:] = "int"
    return out


def ml_to_genetic(lay: GeneticLayout, x: np.ndarray) -> np.ndarray:
    """feature_encoder.py:97-110,126-127 (OHE group -> argmax category)."""
    x = np.atleast_2d(np.asarray(x, np.float64))
    xm = x[:, lay.mutable_mask]
    n = int(lay.no_ohe_mask.sum())
    out = np.empty((x.shape[0], lay.V))
    out[:, :n] = xm[:, lay.no_ohe_mask]
    for k, m in enumerate(lay.ohe_masks):
        out[:, n + k] = np.argmax(xm[:, m], axis=1)  # OneHotEncoder.inverse_transform
    return out


def genetic_to_ml(lay: GeneticLayout, genes: np.ndarray, x_init: np.ndarray) -> np.ndarray:
    """feature_encoder.py:91-95,112-124,129-130."""
    genes = np.atleast_2d(np.asarray(genes, np.float64))
    n = int(lay.no_ohe_mask.sum())
    nm = int(lay.mutable_mask.sum())
    mut = np.zeros((genes.shape[0], nm))
    mut[:, lay.no_ohe_mask] = genes[:, :n]
    for k, m in enumerate(lay.ohe_masks):
        cat = genes[:, n + k]
        oh = (cat[:, None] == np.arange(m.shape[0])[None, :]).astype(np.float64)
        mut[:, m] = oh
    out = np.zeros((genes.shape[0], lay.D))
    out[:, ~lay.mutable_mask] = np.asarray(x_init, np.float64)[~lay.mutable_mask]
    out[:, lay.mutable_mask] = mut
    return out


def feature_min_max(fmin_raw, fmax_raw, dynamic_input=None):
    """lcld_constraints.py:237-263 / botnet_constraints.py:190-216 ``get_feature_min_max``."""
    fmin_raw = np.asarray(fmin_raw, dtype=object)
    fmax_raw = np.asarray(fmax_raw, dtype=object)
    dmin = fmin_raw.astype(str) == "dynamic"
    dmax = fmax_raw.astype(str) == "dynamic"
    xl = np.zeros(fmin_raw.shape[0])
    xu = np.zeros(fmax_raw.shape[0])
    xl[~dmin] = fmin_raw[~dmin].astype(np.float64)
    xu[~dmax] = fmax_raw[~dmax].astype(np.float64)
    if dynamic_input is not None:
        xl[dmin] = dynamic_input[dmin]
        xu[dmax] = dynamic_input[dmax]
    return xl, xu


# --------------------------------------------------------------------------------------
# C. Domain constraints (numpy path)
# --------------------------------------------------------------------------------------
def _month(f):
    """lcld_constraints.py:32-34."""
    return np.floor(f / 100) * 12 + (f % 100)


def lcld_constraints(x: np.ndarray) -> np.ndarray:
    """lcld_constraints.py:168-223 ``LcldConstraints.evaluate_numpy`` (10 columns)."""
    x = np.asarray(x, np.float64)
    calc = (x[:, 0] * (x[:, 2] / 1200) * (1 + x[:, 2] / 1200) ** x[:, 1]) / (
        (1 + x[:, 2] / 1200) ** x[:, 1] - 1
    )
    g41 = np.absolute(x[:, 3] - calc) - 0.099999
    g42 = x[:, 10] - x[:, 14]
    g43 = x[:, 16] - x[:, 11]
    g44 = np.absolute((36 - x[:, 1]) * (60 - x[:, 1]))
    g45 = np.absolute(x[:, 20] - x[:, 0] / x[:, 6])
    g46 = np.absolute(x[:, 21] - x[:, 10] / x[:, 14])
    g47 = np.absolute(x[:, 22] - (_month(x[:, 7]) - _month(x[:, 9])))
    g48 = np.absolute(x[:, 23] - x[:, 11] / x[:, 22])
    g49 = np.absolute(x[:, 24] - x[:, 16] / x[:, 22])
    mask = x[:, 11] == 0
    ratio = np.full(x.shape[0], -1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio[~mask] = x[~mask, 16] / x[~mask, 11]
    ratio[ratio == np.inf] = -1
    ratio[np.isnan(ratio)] = -1
    g410 = np.absolute(x[:, 25] - ratio)
    c = np.column_stack([g41, g42, g43, g44, g45, g46, g47, g48, g49, g410])
    c[c <= TOL] = 0.0
    return c


def augmented_xor_constraints(x, important_features, features_mean) -> List[np.ndarray]:
    """src/examples/utils.py:7-29 ``constraints_augmented_np``."""
    n_imp = len(important_features)
    x_aug = x[:, -math.comb(n_imp, 2):]
    out = []
    for idx, (i1, i2) in enumerate(combinations(range(n_imp), 2)):
        g = np.abs(
            x_aug[:, idx]
            - np.logical_xor(
                x[:, int(important_features[i1])] >= features_mean[i1],
                x[:, int(important_features[i2])] >= features_mean[i2],
            ).astype(np.float64)
        )
        out.append(g)
    return out


def lcld_augmented_constraints(x: np.ndarray, important: np.ndarray) -> np.ndarray:
    """lcld_augmented_constraints.py:176-234 (10 LCLD + 10 XOR columns)."""
    x = np.asarray(x, np.float64)
    base = lcld_constraints_raw(x)
    aug = augmented_xor_constraints(x, important[:, 0], important[:, 1])
    c = np.column_stack(base + aug)
    c[c <= TOL] = 0.0
    return c


def lcld_constraints_raw(x) -> List[np.ndarray]:
    x = np.asarray(x, np.float64)
    calc = (x[:, 0] * (x[:, 2] / 1200) * (1 + x[:, 2] / 1200) ** x[:, 1]) / (
        (1 + x[:, 2] / 1200) ** x[:, 1] - 1
    )
    mask = x[:, 11] == 0
    ratio = np.full(x.shape[0], -1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio[~mask] = x[~mask, 16] / x[~mask, 11]
    ratio[ratio == np.inf] = -1
    ratio[np.isnan(ratio)] = -1
    return [
        np.absolute(x[:, 3] - calc) - 0.099999,
        x[:, 10] - x[:, 14],
        x[:, 16] - x[:, 11],
        np.absolute((36 - x[:, 1]) * (60 - x[:, 1])),
        np.absolute(x[:, 20] - x[:, 0] / x[:, 6]),
        np.absolute(x[:, 21] - x[:, 10] / x[:, 14]),
        np.absolute(x[:, 22] - (_month(x[:, 7]) - _month(x[:, 9]))),
        np.absolute(x[:, 23] - x[:, 11] / x[:, 22]),
        np.absolute(x[:, 24] - x[:, 16] / x[:, 22]),
        np.absolute(x[:, 25] - ratio),
    ]


BOTNET_SUM_IDX = [0, 3, 6, 12, 15, 18]  # botnet_constraints.py:123-125
BOTNET_MAX_IDX = [1, 4, 7, 13, 16, 19]
BOTNET_MIN_IDX = [2, 5, 8, 14, 17, 20]


def _botnet_pairs(feat_idx: Dict[str, list], upper_idx, lower_idx):
    """botnet_constraints.py:271-288 ``define_individual_constraints`` (column x[lower]-x[upper])."""
    keys = list(feat_idx.keys())
    pairs = []
    for i in range(len(upper_idx)):
        key = keys[upper_idx[i]]
        lo_k, up_k = keys[lower_idx[i]], keys[upper_idx[i]]
        for j in range(len(feat_idx[key])):
            pairs.append((feat_idx[lo_k][j], feat_idx[up_k][j]))
    return pairs


def botnet_constraints_raw(x: np.ndarray, feat_idx: Dict[str, list]) -> List[np.ndarray]:
    """botnet_constraints.py:117-168 (before the tol clamp)."""
    x = np.asarray(x, np.float64)
    fi = feat_idx

    def s(k):
        return x[:, fi[k]].sum(axis=1)

    g1 = np.absolute((s("icmp_sum_s_idx") + s("udp_sum_s_idx") + s("tcp_sum_s_idx"))
                     - (s("bytes_in_sum_s_idx") + s("bytes_out_sum_s_idx")))
    g2 = np.absolute((s("icmp_sum_d_idx") + s("udp_sum_d_idx") + s("tcp_sum_d_idx"))
                     - (s("bytes_in_sum_d_idx") + s("bytes_out_sum_d_idx")))
    cons = [g1, g2]
    # botnet_constraints.py:290-309: NOTE range(len(key string) - 2) = 17 ports
    for bo, po in (("bytes_out_sum_s_idx", "pkts_out_sum_s_idx"),
                   ("bytes_out_sum_d_idx", "pkts_out_sum_d_idx")):
        for j in range(len(bo) - 2):
            a = x[:, fi[bo][j]]
            b = x[:, fi[po][j]]
            cons.append(np.divide(a, b, out=np.zeros_like(a), where=b != 0) - 1500)
    for up, lo in ((BOTNET_SUM_IDX, BOTNET_MAX_IDX), (BOTNET_SUM_IDX, BOTNET_MIN_IDX),
                   (BOTNET_MAX_IDX, BOTNET_MIN_IDX)):
        for a, b in _botnet_pairs(fi, up, lo):
            cons.append(x[:, a] - x[:, b])
    return cons


def botnet_constraints(x, feat_idx) -> np.ndarray:
    c = np.column_stack(botnet_constraints_raw(x, feat_idx))
    c[c <= TOL] = 0.0
    return c


def botnet_augmented_constraints(x, feat_idx, important) -> np.ndarray:
    """botnet_augmented_constraints.py (A10 + constraints_augmented_np)."""
    x = np.asarray(x, np.float64)
    c = np.column_stack(botnet_constraints_raw(x, feat_idx)
                        + augmented_xor_constraints(x, important[:, 0], important[:, 1]))
    c[c <= TOL] = 0.0
    return c


def augment_data(x, important_features):
    """src/experiments/botnet/features.py:6-21."""
    shape = x.shape
    lx = x.reshape(-1, shape[-1])
    nf = []
    for i1, i2 in combinations(range(important_features.shape[0]), 2):
        nf.append(np.logical_xor(
            lx[:, int(important_features[i1, 0])] >= important_features[i1, 1],
            lx[:, int(important_features[i2, 0])] >= important_features[i2, 1],
        ).astype(np.float64))
    out = np.concatenate((lx, np.column_stack(nf)), axis=1)
    return out.reshape(*shape[:-1], -1)


# --------------------------------------------------------------------------------------
# D. Classifier + objectives (default_problem.py:76-140, classifier.py:23-29)
# --------------------------------------------------------------------------------------
def mlp_predict_proba(x_ml: np.ndarray, weights, biases) -> np.ndarray:
    """Keras Sequential(Dense relu x3, Dense softmax) forward in fp32.

    The reference model is a TF SavedModel (src/experiments/{lcld,botnet}/model.py:9-20);
    Keras casts the fp64 input to float32.  Summation order differs from Eigen: parity
    is within fp32 rounding (tolerance 1e-5 relative in tests).
    """
    h = np.asarray(x_ml, np.float64).astype(np.float32)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = h @ w.astype(np.float32) + b.astype(np.float32)
        if i < len(weights) - 1:
            h = np.maximum(h, np.float32(0))
    h = h - h.max(axis=1, keepdims=True)
    e = np.exp(h)
    p = e / e.sum(axis=1, keepdims=True)
    if p.shape[1] == 1:  # classifier.py:27-28
        p = np.concatenate((1 - p, p), axis=1)
    return p


@dataclass
class Problem:
    """Everything `DefaultProblem._evaluate` needs for one initial state."""

    lay: GeneticLayout
    x_init: np.ndarray  # (D,)
    xl: np.ndarray  # feature bounds for this state (dynamic ones = x_init)
    xu: np.ndarray
    enc_scale: np.ndarray  # encoder MinMax on [xl, xu] (state-dependent bounds)
    enc_min: np.ndarray
    ml_scale: Optional[np.ndarray]  # ML scaler (models/*/scaler.joblib)
    ml_min: Optional[np.ndarray]
    weights: list
    biases: list
    constraints_fn: object  # x_f -> (n, C)
    minimize_class: int = 1
    norm: object = 2
    scale_objectives: bool = True

    @property
    def x_init_mm(self):
        return minmax_transform(self.x_init[None, :], self.enc_scale, self.enc_min)[0]


def make_problem(lay, x_init, fmin_raw, fmax_raw, ml_scaler, weights, biases, constraints_fn,
                 minimize_class=1, norm=2, scale_objectives=True) -> Problem:
    """moeva2.py:141-154 per-state problem: encoder bounds are dynamic in x_init."""
    xl, xu = feature_min_max(fmin_raw, fmax_raw, x_init)
    sc, mn = minmax_fit(xl, xu)
    ml_s = ml_m = None
    if ml_scaler is not None:
        ml_s, ml_m = ml_scaler
    return Problem(lay, np.asarray(x_init, np.float64), xl, xu, sc, mn, ml_s, ml_m, weights, biases,
                   constraints_fn, minimize_class, norm, scale_objectives)


def evaluate(prob: Problem, genes: np.ndarray, return_g=False):
    """default_problem.py:99-140 ``DefaultProblem._evaluate`` -> F (n,3) [, G_all (n,C)]."""
    x_f = genetic_to_ml(prob.lay, genes, prob.x_init)
    x_f_mm = minmax_transform(x_f, prob.enc_scale, prob.enc_min)
    x_ml = x_f if prob.ml_scale is None else minmax_transform(x_f, prob.ml_scale, prob.ml_min)
    f1 = mlp_predict_proba(x_ml, prob.weights, prob.biases)[:, prob.minimize_class]
    d = x_f_mm - prob.x_init_mm
    if prob.norm in ("inf", np.inf):
        f2 = np.linalg.norm(d, ord=np.inf, axis=1)
        f2_scale = 1.0  # utils.py:18-19 MinMaxScaler fit [[0],[1]]
    elif prob.norm in ("2", 2):
        f2 = np.linalg.norm(d, ord=2, axis=1)
        f2_scale = 1.0 / np.sqrt(prob.x_init.shape[0])  # utils.py:16-17
    else:
        raise NotImplementedError
    if prob.scale_objectives:
        f2 = f2 * f2_scale + 0.0
    g = prob.constraints_fn(x_f)
    g = g * (g > 0).astype(np.float64)  # default_problem.py:93-97
    f3 = g.sum(axis=1)
    F = np.column_stack([f1.astype(np.float64), f2, f3])
    return (F, g) if return_g else F


# --------------------------------------------------------------------------------------
# E. R-NSGA-III survival  [pymoo-recall except the dominance relation]
# --------------------------------------------------------------------------------------
def domination_matrix(F: np.ndarray) -> np.ndarray:
    """pareto_operation.py ``calc_domination_matrix`` (copy of pymoo Dominator), epsilon 0.
    The reference builds L = repeat(F), R = tile(F) and compares row pairs; the broadcast
    below compares the same pairs (i, j) -> (F[i], F[j])."""
    smaller = np.zeros((F.shape[0], F.shape[0]), dtype=bool)
    larger = np.zeros_like(smaller)
    for k in range(F.shape[1]):
        a, b = F[:, k, None], F[None, :, k]
        smaller |= a < b
        larger |= a > b
    return (np.logical_and(smaller, ~larger) * 1 + np.logical_and(larger, ~smaller) * -1)


def fast_non_dominated_sort(F: np.ndarray, n_stop_if_ranked: int):
    """[pymoo-recall] NonDominatedSorting().do(F, return_rank=True, n_stop_if_ranked)
    with the fast-non-dominated-sort discovery order.

    pymoo's loop (for i, for j > i: append the dominated index to ``is_dom[dominator]``)
    leaves ``is_dom[i]`` = the indices i dominates in increasing order, and front 0 = the
    undominated indices in increasing order.  Each later front lists j in the order its
    counter reaches zero while the previous front is walked in order: by the position of
    j's last dominator in that front, then by j.  That order is computed here array-wise
    (tests/test_oracle_survival_cpu.py pins it to the literal loop)."""
    M = domination_matrix(F)
    n = M.shape[0]
    D = M == 1  # D[i, j]: i dominates j
    n_dom = D.sum(axis=0)
    cur = np.flatnonzero(n_dom == 0)
    fronts = [cur]
    ranked = len(cur)
    while ranked < n:
        Dc = D[cur]
        dec = Dc.sum(axis=0)
        n_dom = n_dom - dec
        newly = np.flatnonzero((n_dom == 0) & (dec > 0))
        last = (len(cur) - 1) - np.argmax(Dc[::-1][:, newly], axis=0)
        cur = newly[np.lexsort((newly, last))]
        fronts.append(cur)
        ranked += len(cur)
    out = []
    nr = 0
    for f in fronts:
        out.append(np.asarray(f, dtype=np.int64))
        nr += len(f)
        if nr >= n_stop_if_ranked:
            break
    rank = np.full(n, int(1e16), dtype=np.int64)
    for i, f in enumerate(out):
        rank[f] = i
    return out, rank


def extreme_points(F, ideal, prev_extreme):
    """[pymoo-recall] nsga3.get_extreme_points_c (ASF, weights eye / 1e6 off-diagonal)."""
    w = np.eye(F.shape[1])
    w[w == 0] = 1e6
    _F = F if prev_extreme is None else np.concatenate([prev_extreme, F], axis=0)
    __F = _F - ideal
    __F[__F < 1e-3] = 0
    asf = np.max(__F * w[:, None, :], axis=2)
    I = np.argmin(asf, axis=1)
    return _F[I, :]


def lu_solve3(M, b):
    """Gaussian elimination with partial pivoting in the LAPACK dgetf2/dgetrs operation
    order (column scaling by the reciprocal pivot, column-oriented triangular solves).
    Restates the np.linalg.solve call of nsga3.get_nadir_point [pymoo-recall]; returns
    None when a pivot is exactly zero (LinAlgError)."""
    A = np.array(M, dtype=np.float64, copy=True)
    x = np.array(b, dtype=np.float64, copy=True)
    n = A.shape[0]
    piv = list(range(n))
    for k in range(n):
        p = k
        for i in range(k + 1, n):
            if abs(A[i, k]) > abs(A[p, k]):
                p = i
        if A[p, k] == 0.0:
            return None
        if p != k:
            A[[k, p], :] = A[[p, k], :]
            piv[k], piv[p] = piv[p], piv[k]
            x[k], x[p] = x[p], x[k]
        r = 1.0 / A[k, k]
        for i in range(k + 1, n):
            A[i, k] = A[i, k] * r
        for j in range(k + 1, n):
            for i in range(k + 1, n):
                A[i, j] = A[i, j] - A[i, k] * A[k, j]
    for j in range(n):  # forward, unit lower
        for i in range(j + 1, n):
            x[i] = x[i] - x[j] * A[i, j]
    for j in range(n - 1, -1, -1):  # backward
        x[j] = x[j] / A[j, j]
        for i in range(j):
            x[i] = x[i] - x[j] * A[i, j]
    return x


def nadir_point(extreme, ideal, worst, worst_of_front_arg, worst_of_population_arg):
    """[pymoo-recall] nsga3.get_nadir_point. NOTE the reference call site
    (AspirationPointSurvival) passes (worst_of_population, worst_of_front) into the
    (worst_of_front, worst_of_population) parameters -- the swap is kept."""
    M = extreme - ideal
    b = np.ones(extreme.shape[1])
    plane = lu_solve3(M, b)
    ok = plane is not None
    if ok:
        with np.errstate(divide="ignore", invalid="ignore"):
            intercepts = 1.0 / plane
        nadir = ideal + intercepts
        Mp = np.array([(M[i, 0] * plane[0] + M[i, 1] * plane[1]) + M[i, 2] * plane[2]
                       for i in range(3)])
        close = np.all(np.abs(Mp - b) <= 1e-8 + 1e-5 * np.abs(b))
        if not close or np.any(intercepts <= 1e-6):
            ok = False
        else:
            m = nadir > worst
            nadir[m] = worst[m]
    if not ok:
        nadir = np.array(worst_of_front_arg, dtype=np.float64, copy=True)
    m = nadir - ideal <= 1e-6
    nadir[m] = worst_of_population_arg[m]
    return nadir


def ref_dirs_from_points(ref_point, asp_dirs, mu):
    """[pymoo-recall] rnsga3.get_ref_dirs_from_points + line_plane_intersection.
    With one aspiration direction (MoEvA2's, ``moeva2.py``'s 1x3 (1/3, 1/3, 1/3)) the
    per-point loop is evaluated for all points at once with the same operations."""
    n_obj = ref_point.shape[1]
    nvec = np.ones(n_obj) / np.sqrt(n_obj)
    p0 = np.eye(n_obj)[0]
    asp = np.asarray(asp_dirs, dtype=np.float64)
    if asp.shape[0] == 1 and n_obj == 3:
        P = np.asarray(ref_point, dtype=np.float64)
        r0 = mu * asp[0]
        cent = r0 / 1.0  # np.mean over one row
        l = P - 0.0
        dot = (l[:, 0] * nvec[0] + l[:, 1] * nvec[1]) + l[:, 2] * nvec[2]
        w = p0 - 0.0
        wn = (w[0] * nvec[0] + w[1] * nvec[1]) + w[2] * nvec[2]
        big = np.abs(dot) > 1e-6
        with np.errstate(divide="ignore", invalid="ignore"):
            d = wn / dot
            inter_a = 0.0 + l * d[:, None]
        q = P - p0
        t = (q[:, 0] * nvec[0] + q[:, 1] * nvec[1]) + q[:, 2] * nvec[2]
        inter_b = P - t[:, None] * nvec
        inter = np.where(big[:, None], inter_a, inter_b)
        r = r0[None, :] + (inter - cent[None, :])
        fix = ~(r > 0).min(axis=1)
        if fix.any():
            rf = r[fix]
            rf[rf < 0] = 0
            s = (rf[:, 0] + rf[:, 1]) + rf[:, 2]
            r[fix] = rf / s[:, None]
        return np.concatenate([r, np.eye(n_obj)])
    return _ref_dirs_from_points_loop(ref_point, asp_dirs, mu)


def _ref_dirs_from_points_loop(ref_point, asp_dirs, mu):
    """The per-point loop of get_ref_dirs_from_points as pymoo writes it (any number of
    aspiration directions); tests/test_oracle_survival_cpu.py pins the vectorised one-direction
    path above to it."""
    n_obj = ref_point.shape[1]
    nvec = np.ones(n_obj) / np.sqrt(n_obj)
    p0 = np.eye(n_obj)[0]
    val = []
    for point in ref_point:
        r = mu * np.array(asp_dirs, dtype=np.float64, copy=True)
        cent = np.mean(r, axis=0)
        l = point - 0.0
        dot = (l[0] * nvec[0] + l[1] * nvec[1]) + l[2] * nvec[2]
        if abs(dot) > 1e-6:
            w = p0 - 0.0
            d = ((w[0] * nvec[0] + w[1] * nvec[1]) + w[2] * nvec[2]) / dot
            inter = 0.0 + l * d
        else:
            q = point - p0
            t = (q[0] * nvec[0] + q[1] * nvec[1]) + q[2] * nvec[2]
            inter = point - t * nvec
        r = r + (inter - cent)
        if not (r > 0).min():
            r[r < 0] = 0
            r = r / np.sum(r, axis=1)[:, None]
        val.extend(r)
    val.extend(np.eye(n_obj))
    return np.array(val)


def normalized_dirs(ref_dirs):
    """Cython calc_perpendicular_distance line normalisation [pymoo-recall]."""
    nrm = np.sqrt((ref_dirs[:, 0] * ref_dirs[:, 0] + ref_dirs[:, 1] * ref_dirs[:, 1])
                  + ref_dirs[:, 2] * ref_dirs[:, 2])
    return ref_dirs / nrm[:, None]


def associate(F, ref_dirs, ideal, nadir):
    """[pymoo-recall] nsga3.associate_to_niches with the Cython perpendicular distance:
    s = N.u_hat ; d = sqrt(sum((s*u_hat - N)^2)); niche = first argmin."""
    denom = nadir - ideal
    denom = np.where(denom == 0, 1e-12, denom)
    N = (F - ideal) / denom
    U = normalized_dirs(ref_dirs)
    s = (N[:, None, 0] * U[None, :, 0] + N[:, None, 1] * U[None, :, 1]) + N[:, None, 2] * U[None, :, 2]
    e0 = s * U[None, :, 0] - N[:, None, 0]
    e1 = s * U[None, :, 1] - N[:, None, 1]
    e2 = s * U[None, :, 2] - N[:, None, 2]
    dist = np.sqrt((e0 * e0 + e1 * e1) + e2 * e2)
    niche = np.argmin(dist, axis=1)
    return niche, dist[np.arange(F.shape[0]), niche]


NICHE_KEY_BLOCK = 8  # rounds of niche-order keys drawn per Philox batch in niching()


def niching(n_remaining, niche_count, niche_of, dist, seed, gen, stream_key=0):
    """[pymoo-recall] nsga3.niching with Philox draws replacing np.random:
    * ``np.random.permutation(next_niches)[:n_select]`` in loop iteration ``round`` ->
      niches ordered by (key(TAG_NICHE_PERM, round*n_niches + niche), niche);
    * ``np.random.shuffle(members)`` then argmin/first -> among the eligible members the
      smallest (key(TAG_NICHE_MEMBER, position), position), the member keys being drawn once
      per generation.  Successive uniform picks without replacement (the reference's fresh
      shuffle per round) and picks in the order of one random permutation have the same
      distribution; fixing the keys makes each niche's pick order a single sort."""
    niche_count = np.array(niche_count, dtype=np.int64, copy=True)
    niche_of = np.asarray(niche_of)
    L = len(niche_of)
    n_niches = len(niche_count)
    mask = np.ones(L, dtype=bool)
    survivors = []
    rnd = 0
    sp = px.Stream(seed, gen, px.TAG_NICHE_PERM, stream_key)
    sm = px.Stream(seed, gen, px.TAG_NICHE_MEMBER, stream_key)
    km = sm.words(np.arange(L))[0].astype(np.int64)
    # members of each niche in increasing position (np.where order)
    by_niche = np.argsort(niche_of, kind="stable")
    starts = np.searchsorted(niche_of[by_niche], np.arange(n_niches + 1))
    # niche-order keys are drawn for blocks of rounds at once (same counters; the block
    # size changes nothing: tests/test_oracle_survival_cpu.py)
    kblk, k0, KB = None, -1, NICHE_KEY_BLOCK
    while len(survivors) < n_remaining:
        n_select = n_remaining - len(survivors)
        nl = np.unique(niche_of[mask])
        cnt = niche_count[nl]
        cand = nl[cnt == cnt.min()]
        if kblk is None or rnd >= k0 + KB:
            k0 = rnd
            kblk = sp.words(np.arange(k0 * n_niches, (k0 + KB) * n_niches))[0].astype(np.int64)
        kn = kblk[(rnd - k0) * n_niches + cand]
        order = np.lexsort((cand, kn))
        cand = cand[order][:n_select]
        for nn in cand:
            members = by_niche[starts[nn]:starts[nn + 1]]
            members = members[mask[members]]
            if niche_count[nn] == 0:
                dmin = dist[members].min()
                members = members[dist[members] == dmin]
            pick = members[np.lexsort((members, km[members]))[0]]
            mask[pick] = False
            survivors.append(int(pick))
            niche_count[nn] += 1
        rnd += 1
    return np.array(survivors, dtype=np.int64)


@dataclass
class SurvivalState:
    ideal: np.ndarray = field(default_factory=lambda: np.full(3, np.inf))
    worst: np.ndarray = field(default_factory=lambda: np.full(3, -np.inf))
    extreme: Optional[np.ndarray] = None


@dataclass
class SurvivalResult:
    survivors: np.ndarray  # indices into the merged population, new population order
    fronts: list
    rank: np.ndarray
    niche: np.ndarray  # for the I-ordered (ranked) individuals
    dist: np.ndarray
    nadir: np.ndarray
    ref_dirs: np.ndarray


def survive(F, n_survive, st: SurvivalState, ref_points, asp_dirs, mu, seed, gen, stream_key=0):
    """[pymoo-recall] rnsga3.AspirationPointSurvival._do (mutates ``st``)."""
    F = np.asarray(F, np.float64)
    st.ideal = np.min(np.vstack((st.ideal, F, ref_points)), axis=0)
    st.worst = np.max(np.vstack((st.worst, F, ref_points)), axis=0)
    fronts, rank = fast_non_dominated_sort(F, n_survive)
    nd = fronts[0]
    st.extreme = extreme_points(np.vstack([F[nd], ref_points]), st.ideal, st.extreme)
    worst_pop = np.max(F, axis=0)
    worst_front = np.max(F[nd, :], axis=0)
    nadir = nadir_point(st.extreme, st.ideal, st.worst, worst_pop, worst_front)
    I = np.concatenate(fronts)
    FI = F[I]
    lens = [len(f) for f in fronts]
    starts = np.cumsum([0] + lens)
    with np.errstate(divide="ignore", invalid="ignore"):
        unit = (ref_points - st.ideal) / (nadir - st.ideal)
    rd = ref_dirs_from_points(unit, asp_dirs, mu)
    niche, dist = associate(FI, rd, st.ideal, nadir)
    if len(I) > n_survive:
        last = np.arange(starts[-2], starts[-1])
        if len(fronts) == 1:
            until = np.array([], dtype=np.int64)
            count = np.zeros(len(rd), dtype=np.int64)
            n_rem = n_survive
        else:
            until = np.arange(0, starts[-2])
            count = np.bincount(niche[until], minlength=len(rd)).astype(np.int64)
            n_rem = n_survive - len(until)
        S = niching(n_rem, count, niche[last], dist[last], seed, gen, stream_key)
        surv_pos = np.concatenate((until, last[S]))
    else:
        surv_pos = np.arange(len(I))
    return SurvivalResult(I[surv_pos], fronts, rank, niche, dist, nadir, rd)


# --------------------------------------------------------------------------------------
# F. Mating: tournament selection, two-point crossover, polynomial mutation
# --------------------------------------------------------------------------------------
def tournament_parents(pop_size, n_offsprings, seed, gen, stream_key=0):
    """[pymoo-recall] TournamentSelection(comp_by_cv_then_random), pressure 2, all CV = 0
    (n_constr=0, default_problem.py:262-268): random permutations (Philox-keyed ranks),
    then ``np.random.choice([a, b])`` -> Philox bit.  Returns (n_matings, 2) positions."""
    n_matings = (n_offsprings + 1) // 2
    n_random = n_matings * 2 * 2
    n_perms = -(-n_random // pop_size)
    sp = px.Stream(seed, gen, px.TAG_SEL_PERM, stream_key)
    perm = []
    for q in range(n_perms):
        keys = sp.words(q * pop_size + np.arange(pop_size))[0].astype(np.int64)
        perm.append(np.lexsort((np.arange(pop_size), keys)))
    P = np.concatenate(perm)[:n_random].reshape(-1, 2)
    sc = px.Stream(seed, gen, px.TAG_SEL_CHOICE, stream_key)
    bit = sc.words(np.arange(P.shape[0]))[0] & 1
    S = np.where(bit == 0, P[:, 0], P[:, 1])
    return S.reshape(n_matings, 2)


def two_point_mask(n_var, n_matings, cuts):
    """softmax_crossover.py:17-36 (pymoo PointCrossover, n_points=2) given cut points
    ``cuts`` (n_matings, min(2, n_var-1)) drawn from 1..n_var-1 without replacement."""
    r = np.sort(np.asarray(cuts, dtype=np.int64).reshape(n_matings, -1), axis=1)
    r = np.column_stack([r, np.full(n_matings, n_var)])
    M = np.zeros((n_matings, n_var), dtype=bool)
    for i in range(n_matings):
        j = 0
        while j < r.shape[1] - 1:
            a, b = r[i, j], r[i, j + 1]
            M[i, a:b] = True
            j += 2
    return M


def crossover_draws(n_sub, n_matings, subset, seed, gen, stream_key=0, prob=0.9):
    """Philox statement of the crossover draws for one variable-type subset:
    do_crossover = u53 < prob; cut a = 1 + floor(w2*(n-1)/2^32); cut b from the
    remaining n-2 points (skip a)."""
    st = px.Stream(seed, gen, px.TAG_CX, stream_key)
    w0, w1, w2, w3 = st.words(np.arange(n_matings) * 2 + subset)
    do = px.u53(w0, w1) < prob
    if n_sub - 1 <= 0:
        return do, np.zeros((n_matings, 0), dtype=np.int64)
    a = 1 + ((w2.astype(np.uint64) * np.uint64(n_sub - 1)) >> np.uint64(32)).astype(np.int64)
    if n_sub - 1 == 1:
        return do, a[:, None]
    b = 1 + ((w3.astype(np.uint64) * np.uint64(n_sub - 2)) >> np.uint64(32)).astype(np.int64)
    b = np.where(b >= a, b + 1, b)
    return do, np.column_stack([a, b])


def crossover(parents_X, masks_by_type, seed, gen, stream_key=0):
    """MixedVariableCrossover (moeva2.py:90-101) of real_two_point / int_two_point
    [pymoo-recall: each type subset is crossed independently, empty subsets skipped,
    Crossover.do applies prob 0.9 per mating].  parents_X: (2, n_matings, V).
    Offspring order = X.reshape(-1, V) of (2, n_matings, V): all first children, then
    all second children."""
    X = np.array(parents_X, dtype=np.float64, copy=True)
    _, n_m, V = X.shape
    out = X.copy()
    for subset, mask in enumerate(masks_by_type):
        idx = np.where(mask)[0]
        if idx.size == 0:
            continue
        do, cuts = crossover_draws(idx.size, n_m, subset, seed, gen, stream_key)
        M = two_point_mask(idx.size, n_m, cuts)
        M &= do[:, None]
        sub0 = X[0][:, idx]
        sub1 = X[1][:, idx]
        c0 = np.where(M, sub1, sub0)
        c1 = np.where(M, sub0, sub1)
        out[0][:, idx] = c0
        out[1][:, idx] = c1
    return out.reshape(-1, V)


def sbx_draws(n_matings, V, seed, gen, stream_key=0):
    """Philox statement of SimulatedBinaryCrossover's per-variable draws [pymoo-recall]:
    one word per (mating m, gene g) at index m*MUT_J + g, TAG_SBX: bit 0 == 0 -> the
    variable crosses (``random > prob_per_variable`` with prob 0.5), bit 1 -> swap c1/c2
    (``random <= 0.5``), words 1, 2 -> calc_betaq's uniform ``rand``."""
    st = px.Stream(seed, gen, px.TAG_SBX, stream_key)
    idx = (np.arange(n_matings, dtype=np.int64)[:, None] * MUT_J +
           np.arange(V, dtype=np.int64)[None, :])
    w0, w1, w2, _ = st.words(idx)
    return (w0 & 1) == 0, (w0 & 2) != 0, px.u53(w1, w2)


def sbx_pair(p0, p1, xl, xu, rand, swap, eta, pow_fn=np.power):
    """pymoo 0.4.2.2 SimulatedBinaryCrossover._do [pymoo-recall] on aligned arrays: the two
    children (c[0], c[1]) where every variable crosses (the caller masks), clipped to the
    bounds (set_to_bounds_if_outside_by_problem).  ``pow_fn``: np.power (the reference) or
    oracle.device_order.det_pow (the engine's)."""
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        y1 = np.minimum(p0, p1)
        y2 = np.maximum(p0, p1)
        delta = y2 - y1
        delta = np.where(delta < 1.0e-10, 1.0e-10, delta)

        def calc_betaq(beta):
            alpha = 2.0 - pow_fn(beta, -(eta + 1.0))
            mask = rand <= (1.0 / alpha)
            return np.where(mask, pow_fn((rand * alpha), (1.0 / (eta + 1.0))),
                            pow_fn((1.0 / (2.0 - rand * alpha)), (1.0 / (eta + 1.0))))

        beta = 1.0 + (2.0 * (y1 - xl) / delta)
        c1 = 0.5 * ((y1 + y2) - calc_betaq(beta) * delta)
        beta = 1.0 + (2.0 * (xu - y2) / delta)
        c2 = 0.5 * ((y1 + y2) + calc_betaq(beta) * delta)
    a, b = np.where(swap, c2, c1), np.where(swap, c1, c2)
    a = np.minimum(np.maximum(a, xl), xu)
    b = np.minimum(np.maximum(b, xl), xu)
    return a, b


def sbx_crossover(parents_X, masks_by_type, xl, xu, seed, gen, eta=30.0, prob=0.9,
                  stream_key=0, pow_fn=np.power):
    """MixedVariableCrossover with real_sbx / int_sbx (north_star's SBX option; the
    reference's stale comment moeva2.py:87 names prob 0.9, eta 30): per subset the
    mating-level draw of crossover_draws (prob), then SBX per variable; int_sbx =
    IntegerFromFloatCrossover [pymoo-recall]: bounds widened by 0.5-1e-16, np.round, and
    the build's clamp to [xl, xu] (as for the mutation).  parents_X: (2, n_matings, V)."""
    X = np.array(parents_X, dtype=np.float64, copy=True)
    _, n_m, V = X.shape
    out = X.copy()
    var_on, swap, rand = sbx_draws(n_m, V, seed, gen, stream_key)
    xl = np.asarray(xl, np.float64)
    xu = np.asarray(xu, np.float64)
    for subset, mask in enumerate(masks_by_type):
        idx = np.where(mask)[0]
        if idx.size == 0:
            continue
        do, _ = crossover_draws(idx.size, n_m, subset, seed, gen, stream_key, prob)
        p0, p1 = X[0][:, idx], X[1][:, idx]
        lo, hi = xl[idx][None, :], xu[idx][None, :]
        wl, wu = (lo, hi) if subset == 0 else (lo - INT_WIDEN, hi + INT_WIDEN)
        c0, c1 = sbx_pair(p0, p1, wl, wu, rand[:, idx], swap[:, idx], eta, pow_fn)
        cross = var_on[:, idx] & (np.abs(p0 - p1) > 1.0e-14) & do[:, None]
        c0 = np.where(cross, c0, p0)
        c1 = np.where(cross, c1, p1)
        if subset == 1:
            c0 = np.minimum(np.maximum(np.round(c0), lo), hi)
            c1 = np.minimum(np.maximum(np.round(c1), lo), hi)
        out[0][:, idx] = c0
        out[1][:, idx] = c1
    return out.reshape(-1, V)


def polynomial_mutation(X, xl, xu, eta, do_mutation, rand, pow_fn=np.power):
    """softmax_mutation.py:60-108 (pymoo PolynomialMutation._do) without the softmax.
    ``do_mutation`` (n, V) bool and ``rand`` (n_mutated,) are the two np.random draws.
    ``pow_fn``: np.power (the reference) or oracle.device_order.det_pow (the engine's)."""
    X = np.asarray(X, np.float64)
    Y = np.full(X.shape, np.inf)
    Y[:, :] = X
    xl_ = np.repeat(np.asarray(xl, np.float64)[None, :], X.shape[0], axis=0)[do_mutation]
    xu_ = np.repeat(np.asarray(xu, np.float64)[None, :], X.shape[0], axis=0)[do_mutation]
    Xm = X[do_mutation]
    with np.errstate(divide="ignore", invalid="ignore"):
        delta1 = (Xm - xl_) / (xu_ - xl_)
        delta2 = (xu_ - Xm) / (xu_ - xl_)
        mut_pow = 1.0 / (eta + 1.0)
        mask = rand <= 0.5
        deltaq = np.zeros(Xm.shape)
        xy = 1.0 - delta1
        val = 2.0 * rand + (1.0 - 2.0 * rand) * (pow_fn(xy, (eta + 1.0)))
        d = pow_fn(val, mut_pow) - 1.0
        deltaq[mask] = d[mask]
        xy = 1.0 - delta2
        val = 2.0 * (1.0 - rand) + 2.0 * (rand - 0.5) * (pow_fn(xy, (eta + 1.0)))
        d = 1.0 - (pow_fn(val, mut_pow))
        deltaq[~mask] = d[~mask]
        _Y = Xm + deltaq * (xu_ - xl_)
    _Y[_Y < xl_] = xl_[_Y < xl_]
    _Y[_Y > xu_] = xu_[_Y > xu_]
    Y[do_mutation] = _Y
    xlb = np.asarray(xl, np.float64)[None, :]
    xub = np.asarray(xu, np.float64)[None, :]
    Y = np.where(Y < xlb, xlb, Y)  # set_to_bounds_if_outside_by_problem
    Y = np.where(Y > xub, xub, Y)
    return Y


INT_WIDEN = 0.5 - 1e-16


MUT_J = 1024  # Philox indices per offspring row of the mutation stream (csrc MUT_J)


def geometric_table(V):
    """T[k] = floor((1 - 1/V)^k * 2^32), k = 0..V, with the C library pow (math.pow) so
    the table is bit-identical to the engine's (csrc/api.cpp)."""
    q = 1.0 - 1.0 / V
    T = [math.floor(math.pow(q, float(k)) * 4294967296.0) for k in range(V + 1)]
    return np.minimum(np.array(T, dtype=np.float64), 4294967295.0).astype(np.uint64)


def mutation_draws(n_off, V, seed, gen, stream_key=0):
    """Philox statement of ``np.random.random((n, n_var)) < 1/n_var`` (softmax_mutation.py
    :60-64; prob = 1/n_var, n_var = V) as a Bernoulli process with geometric gaps: the
    j-th draw of offspring o (counter index o*MUT_J + j, TAG_MUT_MASK) gives the gap
    = #{k in 1..V : word_x < T[k]} to the next mutated gene; words y, z give its PM
    uniform u53.  Returns the (n_off, V) mask and the uniforms in row-major mask order."""
    T = geometric_table(V)[1:]
    sm = px.Stream(seed, gen, px.TAG_MUT_MASK, stream_key)
    do = np.zeros((n_off, V), dtype=bool)
    u = np.zeros((n_off, V))
    pos = np.full(n_off, -1, dtype=np.int64)
    live = np.arange(n_off)
    j = 0
    while live.size:
        w0, w1, w2, _ = sm.words(live * MUT_J + j)
        gap = (w0.astype(np.uint64)[:, None] < T[None, :]).sum(axis=1)
        pos[live] += 1 + gap.astype(np.int64)
        ok = pos[live] < V
        rows = live[ok]
        do[rows, pos[rows]] = True
        u[rows, pos[rows]] = px.u53(w1[ok], w2[ok])
        live = rows
        j += 1
    return do, u[do]


def mutation(X, xl, xu, types, seed, gen, eta=20.0, stream_key=0, pow_fn=np.power):
    """MixedVariableMutation (moeva2.py:104-111): real_pm / int_pm, eta=20.
    int_pm = IntegerFromFloatMutation [pymoo-recall]: bounds widened by 0.5-1e-16,
    np.round (half to even) afterwards.  Build choice: the rounded value is clamped to
    [xl, xu] (differs from the reference only on an exact widened-bound hit)."""
    X = np.asarray(X, np.float64)
    n, V = X.shape
    do, u = mutation_draws(n, V, seed, gen, stream_key)
    is_int = np.asarray([t != "real" for t in types])
    xl = np.asarray(xl, np.float64)
    xu = np.asarray(xu, np.float64)
    wl = np.where(is_int, xl - INT_WIDEN, xl)
    wu = np.where(is_int, xu + INT_WIDEN, xu)
    Y = polynomial_mutation(X, wl, wu, eta, do, u, pow_fn)
    Yi = np.round(Y)
    Yi = np.minimum(np.maximum(Yi, xl[None, :]), xu[None, :])
    return np.where(is_int[None, :], Yi, Y)


# --------------------------------------------------------------------------------------
# G. The per-state GA loop (moeva2.py:128-171 + pymoo.minimize [pymoo-recall])
# --------------------------------------------------------------------------------------
@dataclass
class AttackResult:
    pop_X: np.ndarray  # (P, V) genetic
    pop_F: np.ndarray  # (P, 3)
    history: list


def initial_population(prob: Problem, pop_size: int) -> np.ndarray:
    """sampling.py:64-78 ``InitialStateSampling._do``."""
    g = ml_to_genetic(prob.lay, prob.x_init[None, :])[0]
    X = np.tile(g, (pop_size, 1))
    types = genetic_types(prob.lay)
    m = np.asarray([t != "real" for t in types])
    X[:, m] = np.rint(X[:, m]).astype(int)
    return X


def run_attack(prob: Problem, ref_points, n_gen, pop_size, n_offsprings, seed, mu=0.05,
               save_history=None, stream_key=0, crossover_kind="two_point", sbx_eta=30.0,
               evaluate_fn=None, pow_fn=np.power):
    """evaluate_fn(prob, genes, return_g=True) -> (F, G): default ``evaluate`` (numpy's
    summation orders); oracle.device_order.evaluate_device_order gives the engine's.
    pow_fn: the variation operators' pow -- np.power (the reference) or
    oracle.device_order.det_pow (the engine's)."""
    evaluate_fn = evaluate_fn or evaluate
    asp = np.full((1, 3), 1.0 / 3.0)
    gl, gu = genetic_bounds(prob.lay, prob.xl, prob.xu)
    types = genetic_types(prob.lay)
    masks = [np.array([t == "real" for t in types]), np.array([t == "int" for t in types])]
    X = initial_population(prob, pop_size)
    F, G = evaluate_fn(prob, X, return_g=True)
    hist = []
    _hist_add(hist, save_history, F, G)
    st = SurvivalState()
    r = survive(F, pop_size, st, ref_points, asp, mu, seed, 0, stream_key)
    X, F = X[r.survivors], F[r.survivors]
    for g in range(1, n_gen):
        par = tournament_parents(X.shape[0], n_offsprings, seed, g, stream_key)
        pX = np.stack([X[par[:, 0]], X[par[:, 1]]])
        if crossover_kind == "sbx":
            off = sbx_crossover(pX, masks, gl, gu, seed, g, sbx_eta, 0.9, stream_key, pow_fn)
        else:
            off = crossover(pX, masks, seed, g, stream_key)
        off = off[:n_offsprings]
        off = mutation(off, gl, gu, types, seed, g, stream_key=stream_key, pow_fn=pow_fn)
        Fo, Go = evaluate_fn(prob, off, return_g=True)
        _hist_add(hist, save_history, Fo, Go)
        mX = np.concatenate([X, off])
        mF = np.concatenate([F, Fo])
        r = survive(mF, pop_size, st, ref_points, asp, mu, seed, g, stream_key)
        X, F = mX[r.survivors], mF[r.survivors]
    return AttackResult(X, F, hist)


def _hist_add(hist, mode, F, G):
    if not mode:
        return
    if "reduced" in str(mode):
        hist.append(F)
    elif "full" in str(mode):
        hist.append(np.concatenate((F, G), axis=1))


# --------------------------------------------------------------------------------------
# H. Success rate (objective_calculator.py:44-119, utils.py:43-54)
# --------------------------------------------------------------------------------------
def ohe_distance(type_mask, x):
    """utils.py:43-54 ``get_one_hot_encoding_constraints``."""
    masks = make_layout(np.ones(len(type_mask), bool), type_mask).ohe_masks
    if len(masks) == 0:
        return np.zeros(x.shape[0])
    vals = np.column_stack([np.sum(x[:, m], axis=1) for m in masks])
    return np.sum(np.abs(1 - vals), axis=1)


def objectives_calc(x_init, x_f, constraints_fn, type_mask, ml_scale, ml_min, weights, biases,
                    minimize_class, mm_scale, mm_min, norm):
    """objective_calculator.py:44-84 ``_calculate_objective`` -> [CV, f1, f2]."""
    G = np.concatenate((constraints_fn(x_f), ohe_distance(type_mask, x_f).reshape(-1, 1)), axis=1)
    cv = (G * (G > 0)).sum(axis=1)  # Problem.calc_constraint_violation
    x_ml = x_f if ml_scale is None else minmax_transform(x_f, ml_scale, ml_min)
    f1 = mlp_predict_proba(x_ml, weights, biases)[:, minimize_class]
    xi = minmax_transform(np.asarray(x_init)[None, :], mm_scale, mm_min)
    xs = minmax_transform(x_f, mm_scale, mm_min)
    ordv = np.inf if norm in ("inf", np.inf) else 2
    f2 = np.linalg.norm(xi - xs, ord=ordv, axis=1)
    return np.column_stack([cv, f1.astype(np.float64), f2])


def objectives_respected(obj, thr_f1, thr_f2):
    """objective_calculator.py:86-100 -> o1..o7 columns."""
    c = obj[:, 0] <= 0
    m = obj[:, 1] < thr_f1
    d = obj[:, 2] <= thr_f2
    return np.column_stack([c, m, d, c * m, c * d, m * d, c * m * d])


def success_rate_3d(x_inits, x_attacks, obj_fn, thr_f1, thr_f2):
    """objective_calculator.py:106-119."""
    rows = []
    for i, xs in enumerate(x_attacks):
        rows.append(objectives_respected(obj_fn(x_inits[i], xs), thr_f1, thr_f2).mean(axis=0) > 0)
    return np.array(rows).mean(axis=0)
