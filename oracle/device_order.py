"""The oracle's objectives in the engine's floating-point evaluation order -- TEST
INFRASTRUCTURE ONLY (tests/, tests/golden/make_e2e.py).

``moeva_oracle.evaluate`` restates DefaultProblem._evaluate (default_problem.py:99-140) with
numpy's summation orders (BLAS sgemm for the fp32 classifier, pairwise sums for the
distance and the constraint row sum).  The engine sums the same terms in other orders, so f1
/ f2 / f3 agree to the last few bits only -- and over hundreds of generations one flipped
comparison between two near-equal objective values sends a state's attack down another,
equally valid path (tests/test_gpu_e2e.py measured 0/387 identical botnet trajectories
after 1000 generations with numpy's order).  This module restates the SAME arithmetic
(same operands, same roundings, same order as csrc/eval.hip) so that the oracle's attack
and the device attack can be compared trajectory for trajectory:

* f1: the classifier exactly as k_mlp2 runs it -- the immutable features folded into the
  first layer's bias by an fmaf chain in feature order (k_setup_states); the Dense layers
  as v_mfma_f32_16x16x4f32 accumulations (each output an fmaf chain over k in the order
  16 kg + 4 ka + s for kg, then s = 0..3, then ka = 0..3); the last Dense layer as four
  sequential quarters combined ((q0 + q1) + q2) + q3; the 2-way softmax in fp64 rounded
  to fp32.  One fp32 fmaf is restated as round32(a * b + c) evaluated in fp64, where a * b
  is exact; the fp64 rounding of the sum can differ from the fused single rounding only if
  it lands exactly on an fp32 midpoint (probability ~2^-29 per operation).
* f2: each of 64 lanes sums the squared distances of features lane + 64 t in order, the 64
  partial sums are combined by the wave's butterfly (a balanced pairwise tree in lane
  order), then sqrt and the scale (default_problem.py:80-91).
* f3: the constraint columns in the engine's op order (stable-sorted by op code, the
  ABS_SUMDIFF columns last), the lane-parallel ops summed per lane then by the butterfly,
  plus the ABS_SUMDIFF values in order (constraints_regs in csrc/rowops.h).

Every element value (each constraint column, each scaled feature) is the oracle's own; only
the order of the sums is the engine's.
"""
import numpy as np

from . import moeva_oracle as mo

MV_OP_ABS_SUMDIFF = 3


def _fma32(a, b, c):
    """round32(a * b + c) for fp32 arrays (a * b exact in fp64)."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(
        np.float32)


def mfma_k_order(K):
    """The k sequence of one output element of mlp2_layer: kg, then s, then ka."""
    return [16 * kg + 4 * ka + s for kg in range(K // 16) for s in range(4) for ka in range(4)]


def _dense_mfma(h, W, K):
    """h (n, K) fp32 [zero padded to K], W (K, N) fp32 -> acc (n, N) fp32, k in MFMA order."""
    acc = np.zeros((h.shape[0], W.shape[1]), np.float32)
    for k in mfma_k_order(K):
        acc = _fma32(h[:, k:k + 1], W[k][None, :], acc)
    return acc


def layer0_bias(prob: "mo.Problem"):
    """k_setup_states: b1 + fmaf chain over the immutable features (ascending) of the
    ML-scaled initial state."""
    W0 = prob.weights[0].astype(np.float32)
    x = prob.x_init
    if prob.ml_scale is not None:
        x = mo.minmax_transform(x[None, :], prob.ml_scale, prob.ml_min)[0]
    x32 = x.astype(np.float32)
    s = np.zeros(W0.shape[1], np.float32)
    for f in np.where(~prob.lay.mutable_mask)[0]:
        s = _fma32(x32[f], W0[f], s)
    return (prob.biases[0].astype(np.float32) + s).astype(np.float32)


def f1_device_order(prob: "mo.Problem", x_f: np.ndarray) -> np.ndarray:
    mut = np.where(prob.lay.mutable_mask)[0]
    x_ml = x_f if prob.ml_scale is None else mo.minmax_transform(x_f, prob.ml_scale, prob.ml_min)
    Dm = mut.size
    K0 = (Dm + 15) // 16 * 16
    h = np.zeros((x_f.shape[0], K0), np.float32)
    h[:, :Dm] = x_ml[:, mut].astype(np.float32)
    W0 = np.zeros((K0, prob.weights[0].shape[1]), np.float32)
    W0[:Dm] = prob.weights[0][mut].astype(np.float32)
    nl = len(prob.weights)
    h = np.maximum(_dense_mfma(h, W0, K0) + layer0_bias(prob), np.float32(0))
    for l in range(1, nl - 1):
        W = prob.weights[l].astype(np.float32)
        h = np.maximum(_dense_mfma(h, W, W.shape[0]) + prob.biases[l].astype(np.float32),
                       np.float32(0))
    W = prob.weights[nl - 1].astype(np.float32)
    Kl = W.shape[0]
    kq = Kl // 4
    q = []
    for w in range(4):
        ps = np.zeros((h.shape[0], W.shape[1]), np.float32)
        for k in range(w * kq, (w + 1) * kq):
            ps = _fma32(h[:, k:k + 1], W[k][None, :], ps)
        q.append(ps)
    z = ((((q[0] + q[1]) + q[2]) + q[3]) + prob.biases[nl - 1].astype(np.float32))
    z = z.astype(np.float64)
    e = np.exp(z - z.max(axis=1, keepdims=True))
    den = np.zeros(z.shape[0])
    for c in range(z.shape[1]):
        den = den + e[:, c]
    return (e[:, prob.minimize_class] / den).astype(np.float32).astype(np.float64)


def wave_tree(v):
    """The wave64 butterfly (csrc/wave.h wave_sum): v (n, 64) -> (n,) as a balanced pairwise
    tree in lane order."""
    while v.shape[1] > 1:
        v = v[:, 0::2] + v[:, 1::2]
    return v[:, 0]


def lane_partials(terms):
    """terms (n, m): lane l accumulates terms l, l + 64, ... in order (from +0.0)."""
    n, m = terms.shape
    T = -(-m // 64)
    pad = np.zeros((n, T * 64))
    pad[:, :m] = terms
    acc = np.zeros((n, 64))
    for t in range(T):
        acc = acc + pad[:, 64 * t:64 * (t + 1)]
    return acc


def f2_device_order(prob: "mo.Problem", x_f: np.ndarray) -> np.ndarray:
    mut = np.where(prob.lay.mutable_mask)[0]
    d = mo.minmax_transform(x_f, prob.enc_scale, prob.enc_min)[:, mut] - prob.x_init_mm[mut]
    if prob.norm in ("inf", np.inf):
        f2 = np.abs(d).max(axis=1)
        scale = 1.0
    else:
        f2 = np.sqrt(wave_tree(lane_partials(d * d)))
        scale = 1.0 / (np.sqrt(x_f.shape[1]) - 0.0)
    return f2 * scale + 0.0 if prob.scale_objectives else f2


def engine_op_order(op_codes):
    """Column order of the engine's constraint program (api.cpp: stable sort by op code,
    ABS_SUMDIFF last) and the number of lane-parallel ops."""
    codes = np.asarray(op_codes)
    key = np.where(codes == MV_OP_ABS_SUMDIFF, 1 << 20, codes)
    order = np.argsort(key, kind="stable")
    return order, int((codes != MV_OP_ABS_SUMDIFF).sum())


def f3_device_order(G: np.ndarray, op_codes) -> np.ndarray:
    """G (n, C) after the tol clamp and G * (G > 0) -> the engine's row sum."""
    order, n_lane = engine_op_order(op_codes)
    Gs = G[:, order]
    f3 = wave_tree(lane_partials(Gs[:, :n_lane]))
    sd = np.zeros(G.shape[0])
    for c in range(n_lane, G.shape[1]):
        sd = sd + Gs[:, c]
    return f3 + sd


def evaluate_device_order(prob: "mo.Problem", genes: np.ndarray, op_codes, return_g=False):
    """``moeva_oracle.evaluate`` with the engine's summation orders (module docstring)."""
    x_f = mo.genetic_to_ml(prob.lay, genes, prob.x_init)
    g = prob.constraints_fn(x_f)
    g = g * (g > 0).astype(np.float64)
    F = np.column_stack([f1_device_order(prob, x_f), f2_device_order(prob, x_f),
                         f3_device_order(g, op_codes)])
    return (F, g) if return_g else F
