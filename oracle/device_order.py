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
  sequential quarters combined ((q0 + q1) + q2) + q3; Keras's fp32 softmax (h = z - max,
  exp correctly rounded to fp32, fp32 class-order sum and division: softmax_keras32).
  One fp32 fmaf is restated as round32(a * b + c) evaluated in fp64, where a * b
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

* ``fixed`` (bool [D], optional): the attack's compact gene layout (mv_get_stored_genes,
  csrc/api.cpp stored_genes): mutable features whose gene never changes on the bound state
  set.  The attack evaluates them as immutable features -- folded into the layer-1 bias in
  feature order, left out of the classifier's k sequence and of f2's lanes -- so its f1 /
  f2 are these functions with ``fixed`` set.

* pow in the variation operators: ``det_pow`` restates csrc/detmath.h operation for
  operation (np.power and the device library's pow each round within about an ulp but
  not identically; run_attack(..., pow_fn=det_pow) gives the engine's mutated genes).
"""
import numpy as np

from . import moeva_oracle as mo

MV_OP_ABS_SUMDIFF = 3

# fdlibm e_log.c / e_exp.c constants (csrc/detmath.h)
_LN2_HI, _LN2_LO = 6.93147180369123816490e-01, 1.90821492927058770002e-10
_LG = (6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01,
       2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01,
       1.479819860511658591e-01)
_INVLN2 = 1.44269504088896338700e+00
_P = (1.66666666666666019037e-01, -2.77777777770155933842e-03, 6.61375632143793436117e-05,
      -1.65339022054652515390e-06, 4.13813679705723846039e-08)


def _split(a):
    t = 134217729.0 * a
    hi = t - (t - a)
    return hi, a - hi


def _two_prod(a, b):
    ah, al = _split(a)
    bh, bl = _split(b)
    p = a * b
    return p, ((ah * bh - p) + ah * bl + al * bh) + al * bl


def _two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def _fast_two_sum(a, b):
    s = a + b
    return s, b - (s - a)


def _dd_mul(ah, al, bh, bl):
    p, e = _two_prod(ah, bh)
    e = e + (ah * bl + al * bh)
    return _fast_two_sum(p, e)


def det_log2(x):
    """csrc/detmath.h det_log2: ln x as (hi, lo) for x > 0 finite."""
    m, e = np.frexp(np.asarray(x, np.float64))
    sm = m < 0.7071067811865476
    m = np.where(sm, m * 2.0, m)
    k = (e - sm.astype(e.dtype)).astype(np.float64)
    f = m - 1.0
    s = f / (2.0 + f)
    z = s * s
    w = z * z
    L1, L2, L3, L4, L5, L6, L7 = _LG
    t1 = w * (L2 + w * (L4 + w * L6))
    t2 = z * (L1 + w * (L3 + w * (L5 + w * L7)))
    R = t2 + t1
    hfsq = 0.5 * f * f
    hi, e1 = _two_sum(k * _LN2_HI, f)
    lo = ((k * _LN2_LO - hfsq) + s * (hfsq + R)) + e1
    return hi, lo


def det_exp2(th, tl):
    """csrc/detmath.h det_exp2: exp(th + tl), elementwise."""
    with np.errstate(over="ignore", invalid="ignore"):
        kd = np.floor(_INVLN2 * th + 0.5)
        hi = th - kd * _LN2_HI
        lo = kd * _LN2_LO - tl
        r = hi - lo
        q = r * r
        P1, P2, P3, P4, P5 = _P
        c = r - q * (P1 + q * (P2 + q * (P3 + q * (P4 + q * P5))))
        y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi)
        kk = np.where(np.isfinite(kd), kd, 0.0).astype(np.int64)
        out = np.ldexp(y, kk)
    out = np.where(th > 7.09782712893383973096e+02, np.inf, out)
    out = np.where(th < -7.45133219101941108420e+02, 0.0, out)
    return np.where(np.isnan(th), th, out)


def _int_pow(x, n, neg):
    """det_pow's integer branch (n = |y| <= 64) for positive finite x."""
    _, ex = np.frexp(x)
    big = np.abs(ex) * n > 900
    r = np.ones_like(x)
    b = x.copy()
    rh, rl, bh, bl = np.ones_like(x), np.zeros_like(x), x.copy(), np.zeros_like(x)
    m = n
    while m:
        if m & 1:
            r = r * b
            rh, rl = _dd_mul(rh, rl, bh, bl)
        m >>= 1
        if m:
            b = b * b
            bh, bl = _dd_mul(bh, bl, bh, bl)
    if not neg:
        return np.where(big, r, rh)
    q = 1.0 / rh
    p, pe = _two_prod(q, rh)
    rem = ((1.0 - p) - pe) - q * rl
    return np.where(big, 1.0 / r, q + rem / rh)


def det_pow(x, y):
    """csrc/detmath.h det_pow, elementwise (y broadcast against x)."""
    x, y = np.broadcast_arrays(np.asarray(x, np.float64), np.asarray(y, np.float64))
    with np.errstate(all="ignore"):
        xs = np.where((x > 0) & np.isfinite(x), x, 1.0)
        lh, ll = det_log2(xs)
        th, tl0 = _two_prod(y, lh)
        tl = tl0 + y * ll
        th, tl = _fast_two_sum(th, tl)
        out = det_exp2(th, tl)
        yi = (y == np.floor(y)) & (np.abs(y) <= 64.0)
        if yi.any():
            ay = np.where(yi, np.abs(y), 0.0).astype(np.int64)
            for n in np.unique(ay[yi]):
                for neg in (False, True):
                    sel = yi & (ay == n) & ((y < 0) == neg)
                    if sel.any():
                        out[sel] = _int_pow(xs[sel], int(n), neg)
        out = np.where(x == np.inf, np.where(y > 0, np.inf, 0.0), out)
        out = np.where(x == 0.0, np.where(y > 0, 0.0, np.inf), out)
        out = np.where(x < 0.0, np.nan, out)
        out = np.where((y == 0.0) | (x == 1.0), 1.0, out)
        out = np.where(np.isnan(x) | np.isnan(y), x + y, out)
    return out


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


def _mutable(prob, fixed):
    """The engine's mutable features: the layout's, less the compact layout's fixed ones."""
    m = np.asarray(prob.lay.mutable_mask, bool)
    return m if fixed is None else m & ~np.asarray(fixed, bool)


def compact_fixed(lay, probs):
    """The attack's compact layout for a state set (csrc/api.cpp stored_genes): the feature
    mask of the mutable features whose gene is an integer gene with xl == xu == its initial
    value in every state (``probs``: the states' problems).  One-hot layouts are never
    compacted; nor is a layout whose genes would all be fixed."""
    fixed = np.zeros(lay.D, bool)
    if lay.ohe_masks:
        return fixed
    g_fixed = mo.genetic_types(lay) == "int"
    for prob in probs:
        gl, gu = mo.genetic_bounds(lay, prob.xl, prob.xu)
        g0 = mo.ml_to_genetic(lay, prob.x_init[None, :])[0]
        g_fixed &= (gl == gu) & (g0 == gl) & (np.rint(g0) == g0)
    if not g_fixed.all():
        fixed[np.where(lay.mutable_mask)[0][g_fixed]] = True
    return fixed


def layer0_bias(prob: "mo.Problem", fixed=None):
    """k_setup_states: b1 + fmaf chain over the immutable features (ascending) of the
    ML-scaled initial state."""
    W0 = prob.weights[0].astype(np.float32)
    x = prob.x_init
    if prob.ml_scale is not None:
        x = mo.minmax_transform(x[None, :], prob.ml_scale, prob.ml_min)[0]
    x32 = x.astype(np.float32)
    s = np.zeros(W0.shape[1], np.float32)
    for f in np.where(~_mutable(prob, fixed))[0]:
        s = _fma32(x32[f], W0[f], s)
    return (prob.biases[0].astype(np.float32) + s).astype(np.float32)


def f1_device_order(prob: "mo.Problem", x_f: np.ndarray, fixed=None) -> np.ndarray:
    mut = np.where(_mutable(prob, fixed))[0]
    x_ml = x_f if prob.ml_scale is None else mo.minmax_transform(x_f, prob.ml_scale, prob.ml_min)
    Dm = mut.size
    K0 = (Dm + 15) // 16 * 16
    h = np.zeros((x_f.shape[0], K0), np.float32)
    h[:, :Dm] = x_ml[:, mut].astype(np.float32)
    W0 = np.zeros((K0, prob.weights[0].shape[1]), np.float32)
    W0[:Dm] = prob.weights[0][mut].astype(np.float32)
    nl = len(prob.weights)
    h = np.maximum(_dense_mfma(h, W0, K0) + layer0_bias(prob, fixed), np.float32(0))
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
    return softmax_keras32(z)[:, prob.minimize_class].astype(np.float64)


def softmax_keras32(z):
    """csrc/rowops.h softmax_e: Keras's fp32 softmax of fp32 logits z (n, n_out) -- h = z - max
    in fp32, e = exp(h) correctly rounded to fp32 (fp64 exp, one rounding), the class-order
    fp32 sum, e / sum in fp32."""
    z = np.asarray(z, np.float32)
    h = (z - z.max(axis=1, keepdims=True)).astype(np.float32)
    e = np.exp(h.astype(np.float64)).astype(np.float32)
    den = np.zeros(z.shape[0], np.float32)
    for c in range(z.shape[1]):
        den = (den + e[:, c]).astype(np.float32)
    return (e / den[:, None]).astype(np.float32)


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


def f2_device_order(prob: "mo.Problem", x_f: np.ndarray, fixed=None) -> np.ndarray:
    mut = np.where(_mutable(prob, fixed))[0]
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


def evaluate_device_order(prob: "mo.Problem", genes: np.ndarray, op_codes, return_g=False,
                          fixed=None):
    """``moeva_oracle.evaluate`` with the engine's summation orders (module docstring);
    ``fixed``: the attack's compact layout (features evaluated as immutable)."""
    x_f = mo.genetic_to_ml(prob.lay, genes, prob.x_init)
    g = prob.constraints_fn(x_f)
    g = g * (g > 0).astype(np.float64)
    F = np.column_stack([f1_device_order(prob, x_f, fixed), f2_device_order(prob, x_f, fixed),
                         f3_device_order(g, op_codes)])
    return (F, g) if return_g else F
