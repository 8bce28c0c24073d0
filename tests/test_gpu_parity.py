"""GPU parity: every HIP kernel, called through the C ABI, against the oracle / the
reference's golden vectors.  Tolerances (from BASELINE.json north_star):
  * objectives: 1e-5 relative on f1 (fp32 classifier), 1e-12 on f2/f3 (fp64);
  * constraint-satisfied masks, dominance ranks, niche counts and survivor indices:
    bit-exact on identical objective arrays;
  * variation: integer genes exact, real genes within 1e-12 relative (device pow vs libm).
"""
import os

import numpy as np
import pytest

from conftest import RES
from oracle import moeva_oracle as mo
from oracle import philox as px
from oracle.problems import PROJECTS, Project

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make_constraints(name):
    from moeva2_amd.experiments.united.utils import STR_TO_CONSTRAINTS_CLASS

    feat = os.path.join(RES, PROJECTS[name][0])
    return STR_TO_CONSTRAINTS_CLASS[name](feat, feat.replace("features", "constraints"))


def make_classifier(name):
    from moeva2_amd.attacks.moeva2.classifier import Classifier, load_model

    return Classifier(load_model(os.path.join(RES, PROJECTS[name][1])))


class NpScaler:
    def __init__(self, path):
        d = np.load(path)
        self.scale_, self.min_ = d["scale_"], d["min_"]


def make_scaler(name):
    return NpScaler(os.path.join(RES, PROJECTS[name][2]))


# ------------------------------------------------------------------ constraints / evaluate
@pytest.mark.parametrize("name,fixture", [
    ("botnet", "botnet_constraints.npz"), ("botnet_augmented", "botnet_aug_constraints.npz"),
    ("lcld", "lcld_constraints.npz"), ("lcld_augmented", "lcld_aug_constraints.npz")])
def test_constraints_kernel_matches_reference(golden, name, fixture):
    d = golden(fixture)
    g = make_constraints(name).evaluate(d["x"])
    np.testing.assert_array_equal(g > 0, d["g"] > 0)
    np.testing.assert_allclose(g, d["g"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("name,fixture", [("botnet", "problem_botnet.npz"),
                                          ("lcld", "problem_lcld.npz"),
                                          ("lcld_augmented", "problem_lcld_aug.npz")])
@pytest.mark.parametrize("norm,tag", [(2, "l2"), (np.inf, "linf")])
def test_evaluate_matches_reference_default_problem(golden, name, fixture, norm, tag):
    from moeva2_amd.attacks.moeva2.default_problem import DefaultProblem
    from moeva2_amd.attacks.moeva2.feature_encoder import get_encoder_from_constraints

    d = golden(fixture)
    c, clf, sc = make_constraints(name), make_classifier(name), make_scaler(name)
    for s, x in enumerate(d["x_init"]):
        enc = get_encoder_from_constraints(c, x)
        prob = DefaultProblem(x, clf, 1, enc, c, True, save_history="full", ml_scaler=sc,
                              norm=norm)
        out = {}
        prob._evaluate(d[f"s{s}_genes"], out)
        ref = d[f"s{s}_F_{tag}"]
        np.testing.assert_allclose(out["F"][:, 0], ref[:, 0], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(out["F"][:, 1], ref[:, 1], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(out["F"][:, 2], ref[:, 2], rtol=1e-12, atol=0)
        hist = prob.get_history()[0]
        ref_h = d[f"s{s}_hist_{tag}"]
        np.testing.assert_array_equal(hist[:, 3:] > 0, ref_h[:, 3:] > 0)
        np.testing.assert_allclose(hist[:, 3:], ref_h[:, 3:], rtol=1e-12, atol=0)


@pytest.mark.parametrize("name", ["botnet", "lcld", "lcld_augmented"])
def test_predict_proba_matches_fp32_reference(name):
    p = Project(name)
    x = p.x[:50]
    xm = x * p.ml[0] + p.ml[1]
    ref = mo.mlp_predict_proba(xm, p.weights, p.biases)
    got = make_classifier(name).predict_proba(xm)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("name", ["botnet", "lcld", "lcld_augmented"])
def test_evaluate_bit_exact_in_engine_order(name):
    """mv_evaluate's F is bit-identical to the oracle's objectives restated in the engine's
    summation orders (oracle/device_order.py): same element values, MFMA fmaf-chain order
    for the classifier, wave-butterfly sums for f2 / f3.  (Against numpy's orders F agrees
    to 1e-5 / 1e-12: test_evaluate_matches_reference_default_problem.)"""
    from oracle import device_order as do
    from moeva2_amd.problem import build_device_program, get_engine

    p = Project(name)
    c, clf, sc = make_constraints(name), make_classifier(name), make_scaler(name)
    codes = build_device_program(c).op_code
    eng = get_engine(c, clf, sc, 2)
    X = p.x[:4]
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    rng = np.random.default_rng(11)
    n = 150
    genes = np.empty((X.shape[0], n, p.lay.V))
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        isr = np.array([t == "real" for t in mo.genetic_types(p.lay)])
        g = np.repeat(mo.initial_population(prob, 1), n, axis=0)
        for r in range(n):
            k = rng.integers(0, p.lay.V, size=1 + r % 6)
            v = rng.uniform(gl[k], gu[k])
            g[r, k] = np.where(isr[k], v, np.round(v))
        genes[b] = g
    F = torch.empty((X.shape[0], n, 3), dtype=torch.float64, device="cuda")
    eng.evaluate(torch.as_tensor(genes, device="cuda"), F)
    F = F.cpu().numpy()
    for b in range(X.shape[0]):
        ref = do.evaluate_device_order(p.problem(X[b]), genes[b], codes)
        np.testing.assert_array_equal(F[b, :, :2], ref[:, :2])
        if name == "botnet":  # integer / ratio constraint values: identical element values
            np.testing.assert_array_equal(F[b, :, 2], ref[:, 2])
        else:  # LCLD's installment identity calls pow(): device pow vs numpy may differ by
            # an ulp in a violated column (a few rows in 150)
            np.testing.assert_allclose(F[b, :, 2], ref[:, 2], rtol=1e-14, atol=0)


@pytest.mark.parametrize("dims", [(756, 48, 32, 16, 3), (756, 64, 2), (756, 32, 64, 48, 2)])
def test_row_classifier_shapes_bit_exact(dims):
    """k_mlpr (the gene-reading fp32 classifier: each wave on its own 32 rows, the Dense layers
    transposed on MFMA, hidden layers in registers) on shapes other than the shipped botnet
    net -- widths below 64 (column blocks past a layer's width zeroed), one hidden layer,
    three classes: mv_evaluate's F (full gene layout, mode 0) and a short attack's final F
    (compact layout, offspring rows through out_map) bit-identical to oracle/device_order,
    i.e. to k_mlp2's summation order."""
    import dataclasses

    from oracle import device_order as do
    from moeva2_amd.attacks.moeva2.classifier import Classifier, DenseMLPModel
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs
    from moeva2_amd.io.tf_bundle import DenseMLP
    from moeva2_amd.problem import build_device_program, get_engine

    p = Project("botnet")
    W, _ = _wide_mlp(dims, seed=3)
    rng = np.random.default_rng(4)
    bs = [(0.1 * rng.standard_normal(b)).astype(np.float32) for b in dims[1:]]
    clf = Classifier(DenseMLPModel(DenseMLP(W, bs, ["relu"] * (len(dims) - 2) + ["softmax"])))
    c, sc = make_constraints("botnet"), make_scaler("botnet")
    codes = build_device_program(c).op_code
    eng = get_engine(c, clf, sc, 2)
    X = p.x[:3]
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    assert eng.kernel_times()["mlp_kernel"] == "k_mlpr(genes)"
    probs = [dataclasses.replace(p.problem(X[b]), weights=W, biases=bs) for b in range(3)]
    n = 45
    genes = np.empty((3, n, p.lay.V))
    for b in range(3):
        gl, gu = mo.genetic_bounds(p.lay, probs[b].xl, probs[b].xu)
        g = np.repeat(mo.initial_population(probs[b], 1), n, axis=0)
        for r in range(n):
            k = rng.integers(0, p.lay.V, size=1 + r % 5)
            g[r, k] = np.round(rng.uniform(gl[k], gu[k]))
        genes[b] = g
    F = torch.empty((3, n, 3), dtype=torch.float64, device="cuda")
    eng.evaluate(torch.as_tensor(genes, device="cuda"), F)
    F = F.cpu().numpy()
    for b in range(3):
        ref = do.evaluate_device_order(probs[b], genes[b], codes)
        np.testing.assert_array_equal(F[b], ref)
    eng.attack_run(4, 23, 10, 5, energy_ref_dirs(3, 20, 1), 0.05, 0)
    ga = torch.empty((3, 23, p.lay.V), dtype=torch.float64, device="cuda")
    Fa = torch.empty((3, 23, 3), dtype=torch.float64, device="cuda")
    eng.attack_population(ga, Fa)
    torch.cuda.synchronize()
    fixed = np.zeros(p.lay.mutable_mask.shape[0], bool)
    fixed[np.where(p.lay.mutable_mask)[0][~eng.stored_genes()]] = True
    ga, Fa = ga.cpu().numpy(), Fa.cpu().numpy()
    for b in range(3):
        ref = do.evaluate_device_order(probs[b], ga[b], codes, fixed=fixed)
        np.testing.assert_array_equal(Fa[b], ref)


def _wide_mlp(dims=(756, 512, 512, 256, 2), seed=7):
    """bench.py's configs[4] classifier: Dense relu x3 + softmax, weights ~ N(0, 1/fan_in)."""
    rng = np.random.default_rng(seed)
    W = [(rng.standard_normal((a, b)) / np.sqrt(a)).astype(np.float32)
         for a, b in zip(dims[:-1], dims[1:])]
    return W, [np.zeros(b, np.float32) for b in dims[1:]]


def test_wide_mlp_config_matches_fp32_reference():
    """BASELINE configs[4] (synthetic.botnet.wide: 756-512-512-256-2) runs the 64-row-tile
    k_mlpw32 path (fp32 hidden widths > 128) in the attack and k_predict in predict_proba: f1
    of mv_evaluate and of Classifier.predict_proba against the fp32 numpy forward (1e-5 rel),
    f2/f3 unchanged, then a short attack keeps its invariants and is deterministic."""
    from moeva2_amd.attacks.moeva2.classifier import Classifier, DenseMLPModel
    from moeva2_amd.io.tf_bundle import DenseMLP
    from moeva2_amd.problem import get_engine

    p = Project("botnet")
    W, bs = _wide_mlp()
    clf = Classifier(DenseMLPModel(DenseMLP(W, bs, ["relu"] * 3 + ["softmax"])))
    c, sc = make_constraints("botnet"), make_scaler("botnet")
    X = p.x[:6]
    xm = X * p.ml[0] + p.ml[1]
    ref_p = mo.mlp_predict_proba(xm, W, bs)
    np.testing.assert_allclose(clf.predict_proba(xm), ref_p, rtol=1e-5, atol=1e-7)
    eng = get_engine(c, clf, sc, 2)
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    assert eng.kernel_times()["mlp_kernel"] == "k_mlpw32"
    rng = np.random.default_rng(5)
    n = 37
    genes = np.empty((X.shape[0], n, p.lay.V))
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        g = np.repeat(mo.initial_population(prob, 1), n, axis=0)
        k = rng.integers(0, p.lay.V, size=(n, 3))
        for r in range(n):
            g[r, k[r]] = np.round(rng.uniform(gl[k[r]], gu[k[r]]))
        genes[b] = g
    gd = torch.as_tensor(genes, device="cuda")
    F = torch.empty((X.shape[0], n, 3), dtype=torch.float64, device="cuda")
    eng.evaluate(gd, F)
    F = F.cpu().numpy()
    for b in range(X.shape[0]):
        x_f = mo.genetic_to_ml(p.lay, genes[b], X[b])
        f1 = mo.mlp_predict_proba(x_f * p.ml[0] + p.ml[1], W, bs)[:, 1]
        np.testing.assert_allclose(F[b, :, 0], f1, rtol=1e-5, atol=1e-7)
        ref = mo.evaluate(p.problem(X[b]), genes[b])
        np.testing.assert_allclose(F[b, :, 1:], ref[:, 1:], rtol=1e-12, atol=1e-15)
    from moeva2_amd.attacks.moeva2.ref_dirs import riesz_energy_dirs

    ref_dirs = riesz_energy_dirs(3, 20, seed=1, n_max_iter=200)
    outs = []
    for _ in range(2):
        eng.attack_run(4, 23, 10, 3, ref_dirs, 0.05, 0)
        g = torch.empty((X.shape[0], 23, p.lay.V), dtype=torch.float64, device="cuda")
        Fa = torch.empty((X.shape[0], 23, 3), dtype=torch.float64, device="cuda")
        eng.attack_population(g, Fa)
        torch.cuda.synchronize()
        outs.append((g.cpu().numpy(), Fa.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    # the attack ran the compact gene layout (120 fixed botnet genes evaluated as immutable
    # features), mv_evaluate the full one: same values, f1 / f2 summed in another order
    assert (~eng.stored_genes()).sum() == 120
    Fe = torch.empty((X.shape[0], 23, 3), dtype=torch.float64, device="cuda")
    eng.evaluate(torch.as_tensor(outs[0][0], device="cuda"), Fe)
    Fe = Fe.cpu().numpy()
    np.testing.assert_allclose(Fe[..., 0], outs[0][1][..., 0], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(Fe[..., 1], outs[0][1][..., 1], rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(Fe[..., 2], outs[0][1][..., 2])


# ------------------------------------------------------------------ bf16 perf mode
def _bf16(a):
    """fp32 -> bf16 -> fp32, round to nearest even (v_cvt_pk_bf16_f32 on finite values)."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def _bf16_forward(x_ml, mut, W, bs):
    """The engine's bf16 perf-mode classifier restated in numpy: layer 1 over the mutable
    features with bf16 weights/activations and the immutable features folded into an fp32
    per-row bias (k_setup_states), hidden layers bf16 x bf16 with fp32 accumulation, final
    Dense + softmax in fp32 (test infrastructure, not an oracle of the reference)."""
    x = np.asarray(x_ml, np.float64).astype(np.float32)
    imm = np.setdiff1d(np.arange(x.shape[1]), mut)
    bias1 = bs[0].astype(np.float32) + x[:, imm].astype(np.float64) @ W[0][imm].astype(np.float64)
    h = _bf16(x[:, mut]).astype(np.float64) @ _bf16(W[0][mut]).astype(np.float64) + bias1
    h = np.maximum(h.astype(np.float32), 0)
    for w, b in zip(W[1:-1], bs[1:-1]):
        h = _bf16(h).astype(np.float64) @ _bf16(w).astype(np.float64) + b
        h = np.maximum(h.astype(np.float32), 0)
    z = h.astype(np.float64) @ W[-1].astype(np.float64) + bs[-1]
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


@pytest.mark.parametrize("wide", [False, True])
def test_bf16_mode_classifier(wide):
    """mv_set_mlp_precision(bf16): k_mlp2 (shipped botnet net) / k_mlp (configs[4] wide net)
    on bf16 MFMA.  f1 matches the numpy restatement of the bf16 arithmetic (accumulation order
    aside: 2e-3 absolute), stays close to the fp32 parity value (0.05 absolute on these rows),
    f2/f3 are unchanged, and an attack in bf16 mode reports the bf16 f1 of its final genes."""
    from moeva2_amd.attacks.moeva2.classifier import Classifier, DenseMLPModel
    from moeva2_amd.io.tf_bundle import DenseMLP
    from moeva2_amd.problem import get_engine

    p = Project("botnet")
    if wide:
        W, bs = _wide_mlp()
        clf = Classifier(DenseMLPModel(DenseMLP(W, bs, ["relu"] * 3 + ["softmax"])))
    else:
        clf = make_classifier("botnet")
        dw = clf.dense_weights()
        W, bs = [np.asarray(w, np.float32) for w in dw.weights], [np.asarray(b, np.float32) for b in dw.biases]
    c, sc = make_constraints("botnet"), make_scaler("botnet")
    X = p.x[:5]
    eng = get_engine(c, clf, sc, 2)
    mut = np.asarray(eng.prog.mut_feats)
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    rng = np.random.default_rng(11)
    n = 70
    genes = np.empty((X.shape[0], n, p.lay.V))
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        g = np.repeat(mo.initial_population(prob, 1), n, axis=0)
        k = rng.integers(0, p.lay.V, size=(n, 4))
        for r in range(n):
            g[r, k[r]] = np.round(rng.uniform(gl[k[r]], gu[k[r]]))
        genes[b] = g
    gd = torch.as_tensor(genes, device="cuda")
    F32 = torch.empty((X.shape[0], n, 3), dtype=torch.float64, device="cuda")
    F16 = torch.empty_like(F32)
    try:
        eng.set_mlp_precision("fp32")
        eng.evaluate(gd, F32)
        eng.set_mlp_precision("bf16")
        eng.evaluate(gd, F16)
        torch.cuda.synchronize()
        F32, F16 = F32.cpu().numpy(), F16.cpu().numpy()
        np.testing.assert_array_equal(F16[:, :, 1:], F32[:, :, 1:])
        worst = 0.0
        for b in range(X.shape[0]):
            x_ml = mo.genetic_to_ml(p.lay, genes[b], X[b]) * p.ml[0] + p.ml[1]
            emu = _bf16_forward(x_ml, mut, W, bs)[:, 1]
            np.testing.assert_allclose(F16[b, :, 0], emu, rtol=0, atol=2e-3)
            worst = max(worst, float(np.abs(F16[b, :, 0] - F32[b, :, 0]).max()))
        print(f"bf16 vs fp32 f1: max |diff| {worst:.2e}")
        assert worst < 0.05
        from moeva2_amd.attacks.moeva2.ref_dirs import riesz_energy_dirs

        ref_dirs = riesz_energy_dirs(3, 20, seed=1, n_max_iter=200)
        eng.attack_run(5, 23, 10, 3, ref_dirs, 0.05, 0)
        g = torch.empty((X.shape[0], 23, p.lay.V), dtype=torch.float64, device="cuda")
        Fa = torch.empty((X.shape[0], 23, 3), dtype=torch.float64, device="cuda")
        eng.attack_population(g, Fa)
        torch.cuda.synchronize()
        g, Fa = g.cpu().numpy(), Fa.cpu().numpy()
        assert np.isfinite(Fa).all()
        for b in range(X.shape[0]):
            x_ml = mo.genetic_to_ml(p.lay, g[b], X[b]) * p.ml[0] + p.ml[1]
            np.testing.assert_allclose(Fa[b, :, 0], _bf16_forward(x_ml, mut, W, bs)[:, 1],
                                       rtol=0, atol=2e-3)
    finally:
        eng.set_mlp_precision("fp32")


# ------------------------------------------------------------------ survival
def _random_F(rng, B, N):
    F = np.empty((B, N, 3))
    for b in range(B):
        f = rng.uniform(size=(N, 3))
        f[:, 0] = np.round(f[:, 0], 2)  # ties in f1
        f[: N // 10] = f[N // 10: 2 * (N // 10)]  # duplicates
        f[-5:, 2] = 0.0
        F[b] = f
    return F


def _run_survive(F, ref, n_survive, seed, gen, state):
    from moeva2_amd import _native

    B, N, _ = F.shape
    dev = torch.device("cuda")
    t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
    Fd, refd = t(F), t(ref)
    ideal, worst, ext, has = (t(state["ideal"]), t(state["worst"]), t(state["extreme"]),
                              t(state["has"], torch.int32))
    surv = torch.empty((B, n_survive), dtype=torch.int32, device=dev)
    rank = torch.empty((B, N), dtype=torch.int32, device=dev)
    order = torch.empty((B, N), dtype=torch.int32, device=dev)
    nr = torch.empty((B,), dtype=torch.int32, device=dev)
    niche = torch.empty((B, N), dtype=torch.int32, device=dev)
    dist = torch.empty((B, N), dtype=torch.float64, device=dev)
    nadir = torch.empty((B, 3), dtype=torch.float64, device=dev)
    _native.survive(Fd, refd, n_survive, 0.05, seed, gen, ideal, worst, ext, has, surv, rank,
                    order, nr, niche, dist, nadir)
    torch.cuda.synchronize()
    state.update(ideal=ideal.cpu().numpy(), worst=worst.cpu().numpy(),
                 extreme=ext.cpu().numpy(), has=has.cpu().numpy())
    return dict(surv=surv.cpu().numpy(), rank=rank.cpu().numpy(), order=order.cpu().numpy(),
                nr=nr.cpu().numpy(), niche=niche.cpu().numpy(), dist=dist.cpu().numpy(),
                nadir=nadir.cpu().numpy())


@pytest.mark.parametrize("N,n_survive", [(303, 203), (203, 203), (120, 100), (963, 643),
                                         (643, 643), (64, 40), (96, 64), (33, 20)])
def test_survival_bit_exact_vs_oracle(N, n_survive):
    """N > 512 (Moeva2's default n_pop 640: P + O = 963) keeps the dominance bitsets in HBM.
    N = 64, 96, 33 hit the dominance block-pair edges (a full last block, a last block of
    exactly one 32-row half, a one-row second half)."""
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    rng = np.random.default_rng(N)
    B = 5
    ref = energy_ref_dirs(3, 640 if N > 512 else 200, seed=1)
    asp = np.full((1, 3), 1.0 / 3.0)
    state = dict(ideal=np.full((B, 3), np.inf), worst=np.full((B, 3), -np.inf),
                 extreme=np.zeros((B, 9)), has=np.zeros(B, np.int32))
    ost = [mo.SurvivalState() for _ in range(B)]
    for gen in range(3):  # carries ideal/worst/extreme across generations
        F = _random_F(rng, B, N)
        if N == n_survive and gen == 0:
            F[:] = F[:, :1]  # the initial population: identical copies
        got = _run_survive(F, ref, n_survive, 42, gen, state)
        for b in range(B):
            r = mo.survive(F[b], n_survive, ost[b], ref, asp, 0.05, 42, gen)
            nr = len(np.concatenate(r.fronts))
            assert got["nr"][b] == nr
            np.testing.assert_array_equal(got["order"][b, :nr], np.concatenate(r.fronts))
            rk = np.where(r.rank > 10 ** 15, -1, r.rank)
            np.testing.assert_array_equal(got["rank"][b], rk)
            np.testing.assert_array_equal(got["nadir"][b], r.nadir)
            np.testing.assert_array_equal(got["niche"][b, :nr], r.niche)
            np.testing.assert_array_equal(got["dist"][b, :nr], r.dist)
            np.testing.assert_array_equal(got["surv"][b], r.survivors)
            np.testing.assert_array_equal(state["ideal"][b], ost[b].ideal)
            np.testing.assert_array_equal(state["worst"][b], ost[b].worst)
            np.testing.assert_array_equal(state["extreme"][b].reshape(3, 3), ost[b].extreme)


@pytest.mark.parametrize("N,n_survive,crowd", [(963, 643, 0), (963, 643, 1), (700, 400, 1),
                                               (963, 643, 2)])
def test_survival_bit_exact_one_long_front(N, n_survive, crowd):
    """Every merged individual non-dominated (points on the plane f0 + f1 + f2 = 1, with
    exact duplicates), so the last front is the whole population.  crowd 1: the points
    bunched near one corner, so one niche holds ~300 members (N = 963: more than
    NICHE_SORT_MIN = 256, so niching ranks the members by one bitonic sort of the keys;
    N = 700: ~230, counted); crowd 2: every row identical (the first generations' copies of
    one initial state), one niche holds all 963."""
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    rng = np.random.default_rng(N + crowd)
    B = 4
    ref = energy_ref_dirs(3, 640, seed=1)
    asp = np.full((1, 3), 1.0 / 3.0)
    state = dict(ideal=np.full((B, 3), np.inf), worst=np.full((B, 3), -np.inf),
                 extreme=np.zeros((B, 9)), has=np.zeros(B, np.int32))
    ost = [mo.SurvivalState() for _ in range(B)]
    for gen in range(2):
        w = rng.dirichlet([0.3, 0.3, 8.0] if crowd else [1.0, 1.0, 1.0], size=(B, N))
        F = np.round(w, 3)  # ties and duplicates
        F[..., 2] = 1.0 - F[..., 0] - F[..., 1]
        F[:, N // 2:N // 2 + 20] = F[:, :20]
        if crowd == 2:
            F[:] = F[:, :1]
        got = _run_survive(F, ref, n_survive, 7, gen, state)
        for b in range(B):
            r = mo.survive(F[b], n_survive, ost[b], ref, asp, 0.05, 7, gen)
            nr = len(np.concatenate(r.fronts))
            assert got["nr"][b] == nr
            assert len(r.fronts[-1]) > 512 or N < 900
            np.testing.assert_array_equal(got["order"][b, :nr], np.concatenate(r.fronts))
            np.testing.assert_array_equal(got["niche"][b, :nr], r.niche)
            np.testing.assert_array_equal(got["dist"][b, :nr], r.dist)
            np.testing.assert_array_equal(got["surv"][b], r.survivors)


def test_survival_bit_exact_on_clone_heavy_botnet_states(golden):
    """Survival inputs of real botnet attack generations where the merged population is
    mostly clones (41-93 distinct objective rows of 303, one front of ~275 individuals, so
    niching picks 203 of them): recorded from the device by tools/surv_dump.py when the
    survivors were not distinct (round 4).  The survivors must be distinct and bit-exact vs
    the oracle, with every intermediate (ranks, order, niches, distances, nadir)."""
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    d = golden("survival_botnet_clones.npz")
    F = d["F"]
    B, N, _ = F.shape
    n_survive = int(d["n_survive"])
    ref = energy_ref_dirs(3, int(d["n_pop"]), seed=1)
    asp = np.full((1, 3), 1.0 / 3.0)
    for b in range(B):
        state = dict(ideal=d["ideal"][b:b + 1], worst=d["worst"][b:b + 1],
                     extreme=d["extreme"][b:b + 1], has=d["has_extreme"][b:b + 1])
        seed, gen = int(d["seed"][b]), int(d["gen"][b])
        got = _run_survive(F[b:b + 1], ref, n_survive, seed, gen, state)
        ost = mo.SurvivalState(ideal=d["ideal"][b].copy(), worst=d["worst"][b].copy(),
                               extreme=d["extreme"][b].reshape(3, 3).copy()
                               if d["has_extreme"][b] else None)
        r = mo.survive(F[b], n_survive, ost, ref, asp, 0.05, seed, gen)
        nr = len(np.concatenate(r.fronts))
        assert got["nr"][0] == nr
        np.testing.assert_array_equal(got["order"][0, :nr], np.concatenate(r.fronts))
        np.testing.assert_array_equal(got["nadir"][0], r.nadir)
        np.testing.assert_array_equal(got["niche"][0, :nr], r.niche)
        np.testing.assert_array_equal(got["dist"][0, :nr], r.dist)
        assert len(set(got["surv"][0].tolist())) == n_survive, f"state {b}: duplicate survivors"
        np.testing.assert_array_equal(got["surv"][0], r.survivors)


def _oracle_attack_merges(prob, ref, G, P, O, seed):
    """The merged objective arrays the oracle's attack hands to survival, per generation."""
    asp = np.full((1, 3), 1.0 / 3.0)
    gl, gu = mo.genetic_bounds(prob.lay, prob.xl, prob.xu)
    types = mo.genetic_types(prob.lay)
    masks = [np.array([t == "real" for t in types]), np.array([t == "int" for t in types])]
    X = mo.initial_population(prob, P)
    F = mo.evaluate(prob, X)
    st, out = mo.SurvivalState(), [F]
    r = mo.survive(F, P, st, ref, asp, 0.05, seed, 0)
    X, F = X[r.survivors], F[r.survivors]
    for g in range(1, G):
        par = mo.tournament_parents(P, O, seed, g)
        off = mo.crossover(np.stack([X[par[:, 0]], X[par[:, 1]]]), masks, seed, g)[:O]
        off = mo.mutation(off, gl, gu, types, seed, g)
        mX, mF = np.concatenate([X, off]), np.concatenate([F, mo.evaluate(prob, off)])
        out.append(mF)
        r = mo.survive(mF, P, st, ref, asp, 0.05, seed, g)
        X, F = mX[r.survivors], mF[r.survivors]
    return out


def test_survival_bit_exact_on_attack_objectives():
    """Survival on the objective arrays a real attack produces (clones of x_init, feasible
    rows with f3 == 0, near-equal f1): the tie-breaking cases random arrays rarely hit."""
    p = Project("lcld")
    B, G, P, O, seed = 6, 10, 43, 20, 7
    ref = mo_ref_dirs(P - 3)
    asp = np.full((1, 3), 1.0 / 3.0)
    seqs = [_oracle_attack_merges(p.problem(p.x[b]), ref, G, P, O, seed) for b in range(B)]
    state = dict(ideal=np.full((B, 3), np.inf), worst=np.full((B, 3), -np.inf),
                 extreme=np.zeros((B, 9)), has=np.zeros(B, np.int32))
    ost = [mo.SurvivalState() for _ in range(B)]
    for gen in range(G):
        F = np.stack([s[gen] for s in seqs])
        got = _run_survive(F, ref, P, seed, gen, state)
        for b in range(B):
            r = mo.survive(F[b], P, ost[b], ref, asp, 0.05, seed, gen)
            nr = len(np.concatenate(r.fronts))
            ctx = f"gen {gen} state {b}"
            assert got["nr"][b] == nr, ctx
            np.testing.assert_array_equal(got["order"][b, :nr], np.concatenate(r.fronts), ctx)
            np.testing.assert_array_equal(got["nadir"][b], r.nadir, ctx)
            np.testing.assert_array_equal(got["niche"][b, :nr], r.niche, ctx)
            np.testing.assert_array_equal(got["dist"][b, :nr], r.dist, ctx)
            np.testing.assert_array_equal(got["surv"][b], r.survivors, ctx)


@pytest.mark.parametrize("P,O", [(203, 100), (13, 30), (643, 320)])
def test_tournament_selection_vs_oracle(P, O):
    from moeva2_amd import _native

    B = 3
    par = torch.empty((B, (O + 1) // 2, 2), dtype=torch.int32, device="cuda")
    _native.select_parents(B, P, O, 1234, 7, par)
    ref = mo.tournament_parents(P, O, 1234, 7)
    got = par.cpu().numpy()
    for b in range(B):  # stream key 0: identical draws for every state (moeva2.py:163)
        np.testing.assert_array_equal(got[b], ref)


# ------------------------------------------------------------------ variation
@pytest.mark.parametrize("kind", ["two_point", "sbx"])
@pytest.mark.parametrize("name", ["botnet", "lcld", "lcld_augmented"])
def test_variation_vs_oracle(name, kind):
    """Crossover + mutation of the device (k_gen) against the oracle on identical parents and
    Philox draws: two-point (the reference's operator, moeva2.py:90-101) and the SBX option
    (north_star; real_sbx / int_sbx with eta 30).  Against the reference-faithful oracle
    (np.power): integer genes exact, real genes 1e-12; against the oracle with the engine's
    pow (device_order.det_pow): every gene bit-identical."""
    from oracle.device_order import det_pow
    from moeva2_amd.problem import get_engine

    p = Project(name)
    c, clf, sc = make_constraints(name), make_classifier(name), make_scaler(name)
    eng = get_engine(c, clf, sc, 2)
    eng.set_crossover(kind, 30.0, 0.9)
    B, P, O = 3, 40, 24
    X0 = p.x[:B]
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X0]
    eng.set_states(X0, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    rng = np.random.default_rng(3)
    pops, gls, gus = [], [], []
    for b in range(B):
        prob = p.problem(X0[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        types = mo.genetic_types(p.lay)
        isr = np.array([t == "real" for t in types])
        g = rng.uniform(gl, gu, size=(P, gl.shape[0]))
        g[:, ~isr] = np.round(g[:, ~isr])
        g[:5] = mo.initial_population(prob, 1)[0]
        pops.append(g)
        gls.append(gl)
        gus.append(gu)
    pop = torch.as_tensor(np.stack(pops), device="cuda")
    parents = mo.tournament_parents(P, O, 99, 5)
    par = torch.as_tensor(np.tile(parents[None], (B, 1, 1)).astype(np.int32), device="cuda")
    off = torch.empty((B, O, p.lay.V), dtype=torch.float64, device="cuda")
    eng.variation(P, O, 99, 5, pop, par, off)
    got = off.cpu().numpy()
    types = mo.genetic_types(p.lay)
    masks = [np.array([t == "real" for t in types]), np.array([t == "int" for t in types])]
    isr = masks[0]
    eng.set_crossover("two_point")
    for b in range(B):
        pX = np.stack([pops[b][parents[:, 0]], pops[b][parents[:, 1]]])
        if kind == "sbx":
            ref = mo.sbx_crossover(pX, masks, gls[b], gus[b], 99, 5, 30.0, 0.9)[:O]
        else:
            ref = mo.crossover(pX, masks, 99, 5)[:O]
        ref_np = mo.mutation(ref, gls[b], gus[b], types, 99, 5)
        np.testing.assert_array_equal(got[b][:, ~isr], ref_np[:, ~isr])
        np.testing.assert_allclose(got[b][:, isr], ref_np[:, isr], rtol=1e-12, atol=1e-12)
        if kind == "sbx":
            ref = mo.sbx_crossover(pX, masks, gls[b], gus[b], 99, 5, 30.0, 0.9,
                                   pow_fn=det_pow)[:O]
        ref_det = mo.mutation(ref, gls[b], gus[b], types, 99, 5, pow_fn=det_pow)
        np.testing.assert_array_equal(got[b], ref_det)
    if kind == "sbx":  # the option changes the children (and keeps them in bounds)
        cx2 = mo.crossover(np.stack([pops[0][parents[:, 0]], pops[0][parents[:, 1]]]), masks,
                           99, 5)[:O]
        assert not np.array_equal(got[0], mo.mutation(cx2, gls[0], gus[0], types, 99, 5))
        assert np.all(got >= np.stack(gls)[:, None] - 1e-9) and \
            np.all(got <= np.stack(gus)[:, None] + 1e-9)


# ------------------------------------------------------------------ attack chain
def _attack(name, X, n_gen, seed, hist=0, P=23, O=10, mode="auto", crossover="two_point",
            norm=2):
    from moeva2_amd.problem import get_engine
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    c, clf, sc = make_constraints(name), make_classifier(name), make_scaler(name)
    eng = get_engine(c, clf, sc, norm)
    eng.set_attack_mode(mode)
    eng.set_crossover(crossover)
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    ref = energy_ref_dirs(3, P - 3, seed=1) if P - 3 in (200, 640) else \
        mo_ref_dirs(P - 3)
    eng.attack_run(n_gen, P, O, seed, ref, 0.05, hist)
    B, V = X.shape[0], eng.prog.V
    g = torch.empty((B, P, V), dtype=torch.float64, device="cuda")
    F = torch.empty((B, P, 3), dtype=torch.float64, device="cuda")
    eng.attack_population(g, F)
    h = None
    if hist:
        h = torch.empty((B, P + (n_gen - 1) * O, 3 if hist == 1 else 3 + eng.prog.C),
                        dtype=torch.float64, device="cuda")
        eng.attack_history(h)
    torch.cuda.synchronize()
    return eng, g, F, h, ref


PLANOVF_LIB = os.path.join(os.path.dirname(RES), "lib", "libmoeva_mi355x_planovf.so")


@pytest.mark.parametrize("cx", ["two_point", "sbx"])
def test_plan_overflow_paths_bit_exact(cx, tmp_path):
    """k_genc's plan-overflow paths (a row with more stored mutations than the
    variation plan holds: two-point rows are redone through the OVF branch, SBX rows through
    mutate_row_full) are reached about once per million rows with PLAN_MUT = 8.  The
    plan-overflow build (`make planovf`: MV_PLAN_CAP = 1) flags every row with two or more
    stored mutations -- about a quarter of the rows at one expected mutation per row -- so
    those paths carry the attack.  Its populations must be bit-identical to the default
    build's and to the oracle's engine-order attack (oracle/device_order.py)."""
    import subprocess
    import sys

    from moeva2_amd.problem import build_device_program
    from oracle import device_order as do

    if not os.path.exists(PLANOVF_LIB):
        pytest.fail(f"{PLANOVF_LIB} missing: build it with `make -C "
                    "moeva2-ijcai22-replication_amd/csrc planovf` (__graft_entry__.build())")
    name, B, G, P, O = "botnet", 4, 6, 43, 20
    out = str(tmp_path / "planovf.npz")
    env = dict(os.environ, MOEVA_MI355X_LIB=PLANOVF_LIB)
    runner = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "planovf_run.py")
    subprocess.run([sys.executable, runner, out, name, str(B), str(G), str(P), str(O), cx],
                   env=env, check=True, timeout=240)
    d = np.load(out)
    p = Project(name)
    X = p.x[:B]
    eng, g, F, _, ref = _attack(name, X, G, 77, P=P, O=O, crossover=cx)
    np.testing.assert_array_equal(d["genes"], g.cpu().numpy())
    np.testing.assert_array_equal(d["F"], F.cpu().numpy())
    c = make_constraints(name)
    codes = build_device_program(c).op_code
    fixed = _fixed_features(p, eng.stored_genes())

    def ev(prob, genes, return_g=False):
        return do.evaluate_device_order(prob, genes, codes, return_g, fixed=fixed)

    for b in (0, B - 1):
        r = mo.run_attack(p.problem(X[b]), ref, G, P, O, 77, crossover_kind=cx,
                          evaluate_fn=ev, pow_fn=do.det_pow)
        np.testing.assert_array_equal(d["genes"][b], r.pop_X)
        np.testing.assert_array_equal(d["F"][b], r.pop_F)


def mo_ref_dirs(n):
    from moeva2_amd.attacks.moeva2.ref_dirs import riesz_energy_dirs

    return riesz_energy_dirs(3, n, seed=1, n_max_iter=200)


@pytest.mark.parametrize("name,B,P,O,G,hist,cx", [
    ("botnet", 9, 203, 100, 6, 1, "two_point"), ("botnet_augmented", 3, 43, 20, 5, 2, "two_point"),
    ("lcld", 37, 203, 100, 7, 2, "two_point"), ("lcld_augmented", 11, 43, 20, 6, 1, "two_point"),
    ("lcld", 3, 643, 320, 3, 0, "two_point"), ("botnet", 5, 43, 20, 6, 1, "sbx"),
    ("lcld", 9, 43, 20, 6, 2, "sbx")])
def test_attack_chain_deterministic(name, B, P, O, G, hist, cx, monkeypatch):
    """Two runs of the per-phase chain (k_gen, k_cons, k_mlp2, k_survive per generation) give
    bit-identical genes, objectives and history, with 1 and 4 state groups; the retired
    whole-attack schedule is rejected."""
    X = Project(name).x[:B]
    monkeypatch.setenv("MV_GROUPS", "1")
    e1, g1, F1, h1, _ = _attack(name, X, G, 13, hist=hist, P=P, O=O, mode="chain", crossover=cx)
    monkeypatch.setenv("MV_GROUPS", "4")
    _, g2, F2, h2, _ = _attack(name, X, G, 13, hist=hist, P=P, O=O, mode="auto", crossover=cx)
    np.testing.assert_array_equal(g1.cpu().numpy(), g2.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy(), F2.cpu().numpy())
    if hist:
        np.testing.assert_array_equal(h1.cpu().numpy(), h2.cpu().numpy())
    with pytest.raises(ValueError):
        e1.set_attack_mode("whole")


@pytest.mark.parametrize("name,B,P,O,G,hist,norm", [
    ("lcld", 37, 203, 100, 5, 2, 2), ("lcld_augmented", 11, 43, 20, 6, 2, 2),
    ("lcld", 5, 643, 320, 3, 1, 2), ("lcld", 7, 43, 20, 6, 2, np.inf),
    ("lcld_augmented", 3, 203, 100, 4, 1, np.inf)])
def test_narrow_rows_match_wave_kernels(monkeypatch, name, B, P, O, G, hist, norm):
    """k_narrow (one lane per row: variation, decode, f2, ML row, constraint program) is
    bit-identical to k_gen + k_cons (one wave per row) -- genes, F and the full history
    with every G column -- for both norms and both LCLD programs."""
    X = Project(name).x[:B]
    monkeypatch.setenv("MV_NARROW", "1")
    _, g1, F1, h1, _ = _attack(name, X, G, 17, hist=hist, P=P, O=O, mode="chain", norm=norm)
    monkeypatch.setenv("MV_NARROW", "0")
    _, g0, F0, h0, _ = _attack(name, X, G, 17, hist=hist, P=P, O=O, mode="chain", norm=norm)
    np.testing.assert_array_equal(g1.cpu().numpy(), g0.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy(), F0.cpu().numpy())
    np.testing.assert_array_equal(h1.cpu().numpy(), h0.cpu().numpy())


@pytest.mark.parametrize("name,B,P,O,G,hist,cx", [
    ("botnet", 9, 203, 100, 5, 2, "two_point"), ("botnet", 5, 43, 20, 6, 1, "sbx"),
    ("botnet", 4, 643, 320, 3, 0, "two_point")])
def test_slim_program_matches_full(monkeypatch, name, B, P, O, G, hist, cx):
    """k_genc's phase 2 with the slim program region (DIFF / RATIO_SAFE / ABS_SUMDIFF ops:
    region S of the problem blob, the op words from HBM) is bit-identical to the full
    region A: genes, F and the full history with every G column."""
    X = Project(name).x[:B]
    monkeypatch.setenv("MV_SLIM", "1")
    e1, g1, F1, h1, _ = _attack(name, X, G, 29, hist=hist, P=P, O=O, mode="chain", crossover=cx)
    assert e1.prog.C > 0
    monkeypatch.setenv("MV_SLIM", "0")
    _, g0, F0, h0, _ = _attack(name, X, G, 29, hist=hist, P=P, O=O, mode="chain", crossover=cx)
    np.testing.assert_array_equal(g1.cpu().numpy(), g0.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy(), F0.cpu().numpy())
    if hist:
        np.testing.assert_array_equal(h1.cpu().numpy(), h0.cpu().numpy())


def _fixed_features(p, stored):
    """Feature mask of the genes the attack's compact layout does not store (IDENT problems:
    gene g is mutable feature g)."""
    fixed = np.zeros(p.lay.mutable_mask.shape[0], bool)
    fixed[np.where(p.lay.mutable_mask)[0][~stored]] = True
    return fixed


@pytest.mark.parametrize("name,cx", [("botnet", "two_point"), ("botnet", "sbx"),
                                     ("botnet_augmented", "two_point")])
def test_compact_layout_attack_objectives_bit_exact(name, cx):
    """The attack's compact gene layout (mv_get_stored_genes): on the shipped botnet states
    the 120 integer genes with xl == xu == x_init are not stored.  The final population's
    fixed genes are their bounds, and its F is bit-identical to the oracle's objectives in
    the engine's order with those features evaluated as immutable (device_order ``fixed``)."""
    from oracle import device_order as do
    from moeva2_amd.problem import build_device_program

    p = Project(name)
    c = make_constraints(name)
    codes = build_device_program(c).op_code
    X = p.x[:5]
    eng, g, F, _, _ = _attack(name, X, 5, 41, P=43, O=20, crossover=cx)
    stored = eng.stored_genes()
    assert (~stored).sum() == 120, (~stored).sum()
    fixed = _fixed_features(p, stored)
    genes, F = g.cpu().numpy(), F.cpu().numpy()
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        np.testing.assert_array_equal(genes[b][:, ~stored], np.broadcast_to(gl[~stored],
                                                                            genes[b][:, ~stored].shape))
        ref = do.evaluate_device_order(prob, genes[b], codes, fixed=fixed)
        np.testing.assert_array_equal(F[b], ref)


@pytest.mark.parametrize("cx", ["two_point", "sbx"])
def test_compact_layout_tracks_full_layout(monkeypatch, cx):
    """MV_COMPACT=0 stores every gene.  Both layouts consume the same draws over all 432
    genes, so the populations are the same ones up to the last-bit differences of f1 / f2
    (the compact layout leaves the fixed features' zero distance terms out and folds their
    constant classifier terms into the bias): most states end bit-identical, and the
    compact run's F agrees with the full layout's re-evaluation of its own genes."""
    p = Project("botnet")
    X = p.x[:8]
    monkeypatch.setenv("MV_COMPACT", "0")
    e0, g0, F0, _, _ = _attack("botnet", X, 6, 43, P=43, O=20, crossover=cx)
    assert e0.stored_genes().all()
    monkeypatch.setenv("MV_COMPACT", "1")
    e1, g1, F1, _, _ = _attack("botnet", X, 6, 43, P=43, O=20, crossover=cx)
    assert (~e1.stored_genes()).sum() == 120
    g0, g1n = g0.cpu().numpy(), g1.cpu().numpy()
    same = sum(np.array_equal(g0[b], g1n[b]) for b in range(X.shape[0]))
    print(cx, "bit-identical final populations", same, "/", X.shape[0])
    assert same >= X.shape[0] // 2
    F2 = torch.empty_like(F1)
    e1.evaluate(g1, F2)  # the full layout (every gene) on the compact run's genes
    torch.cuda.synchronize()
    F1n, F2n = F1.cpu().numpy(), F2.cpu().numpy()
    np.testing.assert_allclose(F1n[..., 0], F2n[..., 0], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(F1n[..., 1], F2n[..., 1], rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(F1n[..., 2], F2n[..., 2])


def test_gene_layout_is_the_jobs_not_the_batchs():
    """The compact layout is derived from the states it is bound with.  A job split into
    batches or shards (generate_sharded) passes the WHOLE job's layout (mv_gene_layout ->
    mv_set_gene_layout), so a state runs in the same layout whichever states share its batch.
    Here state 4 has a non-integral value in one of the 120 fixed features: the job keeps that
    gene stored, a batch of states 0-2 alone would not, and with the job's layout the batch's
    results are bit-identical to the job's.  A layout that leaves out a gene some bound state
    can change is refused."""
    from moeva2_amd._native import NativeError
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2

    name = "botnet"
    c = make_constraints(name)
    p = Project(name)
    m = Moeva2(os.path.join(RES, PROJECTS[name][1]), c, ml_scaler=make_scaler(name), norm=2,
               n_gen=5, n_pop=40, n_offsprings=20, seed=7, state_streams=True)
    X = p.x[:6].copy()
    lay0 = m.gene_layout(X)
    assert (~lay0).sum() == 120
    g = int(np.where(~lay0)[0][0])
    f = int(np.where(p.lay.mutable_mask)[0][g])  # IDENT: gene g <-> mutable feature g
    X[4, f] += 0.5
    lay = m.gene_layout(X)
    assert lay[g] and (~lay).sum() == 119
    assert (~m.gene_layout(X[:3])).sum() == 120  # the batch alone would leave gene g out
    g_job, F_job, _ = m.generate(X, 1, return_device=True)
    assert np.array_equal(m.last_engine.stored_genes(), lay)
    g_b, F_b, _ = m.generate(X[:3], 1, return_device=True, gene_layout=lay)
    assert np.array_equal(m.last_engine.stored_genes(), lay)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(g_b.cpu().numpy(), g_job.cpu().numpy()[:3])
    np.testing.assert_array_equal(F_b.cpu().numpy(), F_job.cpu().numpy()[:3])
    m.generate(X[:3], 1, return_device=True)  # default: the batch's own layout again
    assert (~m.last_engine.stored_genes()).sum() == 120
    with pytest.raises(NativeError, match="not fixed"):
        m.generate(X, 1, return_device=True, gene_layout=lay0)


def test_gene_layout_request_applies_to_one_binding():
    """mv_set_gene_layout applies to the NEXT mv_set_states only: after a batch
    bound with a job's layout, a DefaultProblem on the same shared engine binds a state the
    job never held in its own derived layout (a stale request would leave out a gene that
    state can change and refuse it).  A refused request leaves the previous binding intact."""
    from moeva2_amd._native import NativeError
    from moeva2_amd.attacks.moeva2.default_problem import DefaultProblem
    from moeva2_amd.attacks.moeva2.feature_encoder import get_encoder_from_constraints
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2

    name = "botnet"
    c = make_constraints(name)
    p = Project(name)
    sc = make_scaler(name)
    m = Moeva2(os.path.join(RES, PROJECTS[name][1]), c, ml_scaler=sc, norm=2, n_gen=3,
               n_pop=40, n_offsprings=20, seed=7)
    X = p.x[:6].copy()
    lay0 = m.gene_layout(X)
    g = int(np.where(~lay0)[0][0])
    f = int(np.where(p.lay.mutable_mask)[0][g])
    x_new = X[5].copy()
    x_new[f] += 0.5  # gene g is no longer fixed in this state
    m.generate(X[:3], 1, return_device=True, gene_layout=lay0)
    eng = m.last_engine
    clf = m._get_classifier()
    enc = get_encoder_from_constraints(c, x_new)
    prob = DefaultProblem(x_new, clf, 1, enc, c, True, ml_scaler=sc, norm=2)
    assert prob._engine is eng  # the shared engine
    rng = np.random.default_rng(3)
    xg = enc.ml_to_genetic(x_new[None])[0]
    lo, hi = enc.get_min_max_genetic()
    rows = np.clip(xg + rng.normal(0, 1, (8, xg.shape[0])) * (hi - lo) * 0.01, lo, hi)
    rows[:, [t != "real" for t in enc.get_type_mask_genetic()]] = np.rint(
        rows[:, [t != "real" for t in enc.get_type_mask_genetic()]])
    F_shared = prob.evaluate(rows)
    assert eng.stored_genes()[g]  # derived from x_new, not the batch's request
    from moeva2_amd.attacks.moeva2.classifier import Classifier, load_model

    clf2 = Classifier(load_model(os.path.join(RES, PROJECTS[name][1])))  # a fresh engine
    prob2 = DefaultProblem(x_new, clf2, 1, get_encoder_from_constraints(c, x_new), c, True,
                           ml_scaler=sc, norm=2)
    assert prob2._engine is not eng
    np.testing.assert_array_equal(F_shared, prob2.evaluate(rows))
    # a refused request: the previous binding (x_new) stays bound and usable
    eng.set_gene_layout(lay0)
    with pytest.raises(NativeError, match="not fixed"):
        eng.set_states(x_new[None], *[a[None] for a in c.get_feature_min_max(x_new)], 1)
    assert eng.B == 1
    genes = torch.from_numpy(rows).cuda()[None]
    F = torch.empty((1, rows.shape[0], 3), dtype=torch.float64, device="cuda")
    eng.evaluate(genes, F)
    np.testing.assert_array_equal(F[0].cpu().numpy(), F_shared)


@pytest.mark.parametrize("name,G,hist", [("botnet", 25, "reduced"), ("lcld", 12, "full"),
                                         ("lcld", 1, "reduced")])
def test_generate_results_front_and_history(name, G, hist):
    """Moeva2.generate's results from the device: res.pop = the final population, res.X /
    res.F = its non-dominated members computed on the device (mv_attack_front), bit-identical
    to the host relation (pareto_operation.py:35-51 as a numpy broadcast) on the same final
    F; res.history = mv_attack_history's rows entry by entry; the results pickle (the
    driver's legacy results_{hash}.npy) and convert (results_to_history) like lists."""
    import pickle

    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2, _non_dominated
    from moeva2_amd.attacks.moeva2.utils import results_to_history

    c = make_constraints(name)
    p = Project(name)
    m = Moeva2(os.path.join(RES, PROJECTS[name][1]), c, ml_scaler=make_scaler(name), norm=2,
               n_gen=G, n_pop=40, n_offsprings=20, save_history=hist, seed=5)
    X = p.x[:7]
    res = m.generate(X, 1)
    g_d, F_d, h_d = m.generate(X, 1, return_device=True)  # the same attack (same seed)
    genes, F, hh = g_d.cpu().numpy(), F_d.cpu().numpy(), h_d.cpu().numpy()
    P, O = 43, 20
    partial = 0
    for b, r in enumerate(res):
        np.testing.assert_array_equal(r.pop.get("X"), genes[b])
        np.testing.assert_array_equal(np.stack([ind.F for ind in r.pop]), F[b])
        nd = _non_dominated(F[b])
        partial += int(not nd.all())
        np.testing.assert_array_equal(r.X, genes[b][nd])
        np.testing.assert_array_equal(r.F, F[b][nd])
        assert len(r.history) == G
        np.testing.assert_array_equal(r.history[0], hh[b, :P])
        np.testing.assert_array_equal(r.history[-1], hh[b, P + (G - 2) * O:] if G > 1
                                      else hh[b, :P])
        assert r.pareto.shape == (0, genes.shape[2])
    if G == 1:
        assert partial == 0  # P copies of the initial state: none dominates another
    ref_hist = np.array([[g.tolist() for i, g in enumerate(list(r.history)) if i > 0]
                         for r in res])  # utils.py:70-76 on plain lists
    if G > 1:
        np.testing.assert_array_equal(results_to_history(res), ref_hist)
    back = pickle.loads(pickle.dumps(res))
    for r0, r1 in zip(res, back):
        np.testing.assert_array_equal(r0.X, r1.X)
        np.testing.assert_array_equal(r0.pop.get("X"), r1.pop.get("X"))
        np.testing.assert_array_equal(r0.history[G // 2], r1.history[G // 2])


def test_device_buffers_of_another_gpu_are_refused():
    """Entry points check that their buffers live on the engine's GPU (api.cpp on_device):
    a one-GPU box can only show that buffers of the engine's own device pass and that the
    ObjectiveCalculator builds its objects on the device of its tensors."""
    from moeva2_amd.attacks.moeva2.objective_calculator import ObjectiveCalculator

    name = "botnet"
    c, sc = make_constraints(name), make_scaler(name)
    calc = ObjectiveCalculator(make_classifier(name), c, 1, {"f1": 0.5, "f2": 4.0},
                               min_max_scaler=sc, ml_scaler=sc, norm=2)
    p = Project(name)
    xi = torch.from_numpy(p.x[:2]).cuda()
    x = xi[:, None, :].repeat(1, 3, 1).contiguous()
    obj = calc.calculate_objectives_device(xi, x)
    assert list(calc._devs) == [0] and calc._devs[0][0].device == 0
    assert calc._devs[0][1].device == 0 and calc._devs[0][2].device == 0
    np.testing.assert_array_equal(obj.cpu().numpy(), calc.calculate_objectives_3d(p.x[:2],
                                                                                   x.cpu().numpy()))
    with pytest.raises(ValueError):
        calc.calculate_objectives_device(xi.cpu(), x)


def test_attack_invariants_lcld():
    """Whole device loop: bounds, integrality, F == re-evaluation, history layout.  (Each
    generation's kernels are pinned bit-exactly above; the loop is compared end to end
    through the success rate.)"""
    p = Project("lcld")
    X = p.x[:2]
    eng, g, F, h, ref = _attack("lcld", X, 6, 11, hist=1)
    assert np.isfinite(F.cpu().numpy()).all()
    gen = g.cpu().numpy()
    # population within the genetic bounds, integer genes integral
    for b in range(2):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        assert np.all(gen[b] >= gl) and np.all(gen[b] <= gu)
        types = mo.genetic_types(p.lay)
        isr = np.array([t == "real" for t in types])
        np.testing.assert_array_equal(gen[b][:, ~isr], np.round(gen[b][:, ~isr]))
    # F of the final population equals a fresh evaluation of its genes
    F2 = torch.empty_like(F)
    eng.evaluate(g, F2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(F2.cpu().numpy(), F.cpu().numpy())
    # first history block = the initial population's F (identical rows)
    hh = h.cpu().numpy()
    assert hh.shape == (2, 23 + 5 * 10, 3)
    np.testing.assert_array_equal(hh[:, :23], np.repeat(hh[:, :1], 23, axis=1))


def test_attack_deterministic_and_batch_invariant():
    p = Project("botnet")
    X = p.x[:4]
    _, g1, F1, _, _ = _attack("botnet", X, 5, 3)
    _, g2, F2, _, _ = _attack("botnet", X, 5, 3)
    np.testing.assert_array_equal(g1.cpu().numpy(), g2.cpu().numpy())
    _, g3, F3, _, _ = _attack("botnet", X[2:], 5, 3)  # a shard: same states, other positions
    np.testing.assert_array_equal(g1.cpu().numpy()[2:], g3.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy()[2:], F3.cpu().numpy())


def test_attack_state_groups_bit_identical(monkeypatch):
    """mv_attack_run splits the states into groups on separate streams (MV_GROUPS): the
    populations must not depend on the grouping."""
    p = Project("botnet")
    X = p.x[:9]
    monkeypatch.setenv("MV_GROUPS", "1")
    _, g1, F1, _, _ = _attack("botnet", X, 4, 5)
    monkeypatch.setenv("MV_GROUPS", "4")
    _, g4, F4, _, _ = _attack("botnet", X, 4, 5)
    np.testing.assert_array_equal(g1.cpu().numpy(), g4.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy(), F4.cpu().numpy())


def test_moeva2_generate_api_lcld():
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2
    from moeva2_amd.attacks.moeva2.utils import results_to_history, results_to_numpy_results
    from moeva2_amd.attacks.moeva2.feature_encoder import get_encoder_from_constraints

    c = make_constraints("lcld")
    p = Project("lcld")
    m = Moeva2(os.path.join(RES, PROJECTS["lcld"][1]), c, ml_scaler=make_scaler("lcld"), norm=2,
               n_gen=4, n_pop=200, n_offsprings=100, save_history="full", seed=42)
    res = m.generate(p.x[:3], 1)
    assert len(res) == 3 and res[0].pop_size == 203 and len(res[0].pop) == 203
    xa = results_to_numpy_results(res, get_encoder_from_constraints(c))
    assert xa.shape == (3, 203, 47)
    hist = results_to_history(res)
    assert hist.shape == (3, 3, 100, 13)
    assert res[0].pareto.shape == (0, 15)
    assert res[0].X.shape[1] == 15 and res[0].F.shape[1] == 3


def test_generate_sharded_real_engine_world1():
    """Moeva2.generate_sharded with the real engine on a one-rank RCCL group (the multi-GPU
    path's padding + all_gather around Moeva2.generate(return_device=True)): the gathered
    populations equal an unsharded generate of the same states and seed."""
    import socket

    import torch.distributed as dist

    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2

    c = make_constraints("lcld")
    p = Project("lcld")
    m = Moeva2(os.path.join(RES, PROJECTS["lcld"][1]), c, ml_scaler=make_scaler("lcld"), norm=2,
               n_gen=5, n_pop=40, n_offsprings=20, seed=11)
    X = p.x[:5]
    g0, F0, _ = m.generate(X, 1, return_device=True)
    g0, F0 = g0.cpu().numpy(), F0.cpu().numpy()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        g1, F1 = m.generate_sharded(X, 1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(g1.cpu().numpy(), g0)
        np.testing.assert_array_equal(F1.cpu().numpy(), F0)
    finally:
        dist.destroy_process_group()


def test_generate_scored_sharded_real_engine_world1():
    """Moeva2.generate_scored_sharded on a one-rank RCCL group: the gathered per-state o1..o7
    flags equal the ObjectiveCalculator's verdict on an unsharded generate of the same states
    (success_rate_3d, objective_calculator.py:121-128), the successful candidates are the
    reference's _get_one_successful(max_inputs=1) picks (:153-182), and per-state
    streams keyed by the global state index give the same populations unsharded."""
    import socket

    import torch.distributed as dist

    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2
    from moeva2_amd.attacks.moeva2.objective_calculator import ObjectiveCalculator

    name = "botnet"
    c = make_constraints(name)
    p = Project(name)
    sc = make_scaler(name)
    m = Moeva2(os.path.join(RES, PROJECTS[name][1]), c, ml_scaler=sc, norm=2, n_gen=30,
               n_pop=40, n_offsprings=20, seed=11, state_streams=True)
    X = p.x[:6]
    calc = ObjectiveCalculator(make_classifier(name), c, 1, {"f1": 0.5, "f2": 4.0},
                               min_max_scaler=sc, ml_scaler=sc, norm=2)
    res = m.generate(X, 1)
    x_f = np.stack([m._encoder.genetic_to_ml(np.stack([ind.X for ind in r.pop]), X[b])
                    for b, r in enumerate(res)])
    obj = calc.calculate_objectives_3d(X, x_f)
    resp = np.stack([calc._objective_respected(o) for o in obj])
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        flags, best = m.generate_scored_sharded(X, 1, calc)
    finally:
        dist.destroy_process_group()
    np.testing.assert_array_equal(flags, resp.any(axis=1))
    np.testing.assert_array_equal(flags.mean(axis=0), calc.success_rate_3d(X, x_f))
    for b in range(X.shape[0]):
        ok = resp[b][:, 6]
        if ok.any():
            # _get_one_successful(max_inputs=1) literally: the f1 argsort indexed by the o7
            # mask in original row order (stable among equal f1)
            sorted_index = np.argsort(obj[b][:, 1], kind="stable")
            np.testing.assert_array_equal(best[b], x_f[b][sorted_index[ok][0]])
            sel = calc._select_successful(obj[b], x_f[b], "misclassification", "asc", 1)
            assert np.sort(obj[b][:, 1])[np.argmax(ok)] == obj[b][sorted_index[ok][0], 1]
            assert sel.shape == (1, x_f.shape[2])
        else:
            assert np.isnan(best[b]).all()


def test_success_rate_matches_oracle_attack():
    """End to end (north_star): the constrained success rates o1..o7
    (objective_calculator.py:86-119) of the device attack against the oracle's CPU attack
    on the same LCLD states, budget and seed.  Both consume identical Philox draws and the
    survival is bit-exact on identical objectives (test above), so the trajectories part
    only where the fp32 classifier's summation order (MFMA vs BLAS, ~1e-7 relative) flips a
    comparison between two near-equal f1 values -- e.g. a child whose only mutation barely
    moves the classifier.  Populations then diverge, so the end-to-end bar is the success
    rates (north_star: within 1 pp, or one state at this B)."""
    p = Project("lcld")
    B, G, P, O, seed = 48, 15, 43, 20, 7
    X = p.x[:B]
    _, g, _, _, ref = _attack("lcld", X, G, seed, P=P, O=O)
    genes = g.cpu().numpy()
    sc, mn = p.ml

    def fn(xi, xs):
        return mo.objectives_calc(xi, xs, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    x_dev, x_cpu, same = [], [], 0
    for b in range(B):
        r = mo.run_attack(p.problem(X[b]), ref, G, P, O, seed)
        same += int(np.array_equal(r.pop_X, genes[b]))
        x_cpu.append(mo.genetic_to_ml(p.lay, r.pop_X, X[b]))
        x_dev.append(mo.genetic_to_ml(p.lay, genes[b], X[b]))
    sr_dev = mo.success_rate_3d(X, x_dev, fn, 0.25, 0.2)
    sr_cpu = mo.success_rate_3d(X, x_cpu, fn, 0.25, 0.2)
    print("identical final populations:", same, "/", B, "o1..o7 dev", sr_dev, "cpu", sr_cpu)
    assert np.all(np.abs(sr_dev - sr_cpu) <= max(0.01, 1.0 / B) + 1e-12), (sr_dev, sr_cpu)


def test_sbx_attack_matches_oracle_attack():
    """The SBX option end to end: device attack vs the oracle's attack with sbx_crossover on
    the same LCLD states, budget and seed (success rates within 1 pp or one state)."""
    p = Project("lcld")
    B, G, P, O, seed = 24, 10, 43, 20, 5
    X = p.x[:B]
    _, g, _, _, ref = _attack("lcld", X, G, seed, P=P, O=O, crossover="sbx")
    genes = g.cpu().numpy()
    sc, mn = p.ml

    def fn(xi, xs):
        return mo.objectives_calc(xi, xs, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    x_dev, x_cpu, same = [], [], 0
    for b in range(B):
        r = mo.run_attack(p.problem(X[b]), ref, G, P, O, seed, crossover_kind="sbx")
        same += int(np.array_equal(r.pop_X, genes[b]))
        x_cpu.append(mo.genetic_to_ml(p.lay, r.pop_X, X[b]))
        x_dev.append(mo.genetic_to_ml(p.lay, genes[b], X[b]))
    sr_dev = mo.success_rate_3d(X, x_dev, fn, 0.25, 0.2)
    sr_cpu = mo.success_rate_3d(X, x_cpu, fn, 0.25, 0.2)
    print("sbx identical final populations:", same, "/", B, sr_dev, sr_cpu)
    assert np.all(np.abs(sr_dev - sr_cpu) <= max(0.01, 1.0 / B) + 1e-12), (sr_dev, sr_cpu)


def _host_lcld_constraints():
    """The shipped LCLD class with its device program withheld: a plugin the engine cannot
    compile, evaluated by its own numpy ``evaluate`` (here the reference's numpy path as
    restated by the oracle, lcld_constraints.py:168-223)."""
    from moeva2_amd.examples.lcld.lcld_constraints import LcldConstraints

    feat = os.path.join(RES, PROJECTS["lcld"][0])

    class HostLcld(LcldConstraints):
        def device_program(self):
            raise NotImplementedError

        def get_nb_constraints(self):
            return 10

        def evaluate(self, x, use_tensors=False):
            return mo.lcld_constraints(np.atleast_2d(x))

    return HostLcld(feat, feat.replace("features", "constraints"))


class _NumpyMLP:
    """A non-Dense-wrapper model: only predict_proba (the oracle's fp32 forward)."""

    def __init__(self, name):
        p = Project(name)
        self.w, self.b = p.weights, p.biases

    def predict_proba(self, x):
        return mo.mlp_predict_proba(np.asarray(x, np.float64), self.w, self.b)


def test_hosted_constraints_plugin_default_problem():
    """A Constraints subclass without a device program goes through its own evaluate on the
    host: DefaultProblem._evaluate F equals the device program's F (f3 to
    1e-12; f1, f2 identical) and the full history carries the host G."""
    from moeva2_amd.attacks.moeva2.default_problem import DefaultProblem
    from moeva2_amd.attacks.moeva2.feature_encoder import get_encoder_from_constraints

    p = Project("lcld")
    x0 = p.x[3]
    ch, cd = _host_lcld_constraints(), make_constraints("lcld")
    clf, sc = make_classifier("lcld"), make_scaler("lcld")
    rng = np.random.default_rng(1)
    prob = p.problem(x0)
    gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
    g = np.repeat(mo.initial_population(prob, 1), 30, axis=0)
    k = rng.integers(0, p.lay.V, size=30)
    g[np.arange(30), k] = np.round(rng.uniform(gl[k], gu[k]))
    outs = []
    for c in (ch, cd):
        pr = DefaultProblem(x0, clf, 1, get_encoder_from_constraints(c, x0), c, True,
                            save_history="full", ml_scaler=sc, norm=2)
        out = {}
        pr._evaluate(g, out)
        outs.append((out["F"], pr.get_history()[0]))
    np.testing.assert_array_equal(outs[0][0][:, :2], outs[1][0][:, :2])
    np.testing.assert_allclose(outs[0][0][:, 2], outs[1][0][:, 2], rtol=1e-12, atol=0)
    np.testing.assert_allclose(outs[0][1], outs[1][1], rtol=1e-12, atol=0)


@pytest.mark.parametrize("which", ["constraints", "classifier"])
def test_hosted_plugins_attack(which):
    """Moeva2.generate with a host plugin (constraints without a device program, or a model
    with only predict_proba) runs the host-driven loop around the device calls: it tracks
    the all-device attack (same draws; only the host columns' rounding differs), its final
    objectives are the plugin's own values, and with save_history="full" the history's G
    columns are the plugin's clamped ``evaluate`` (default_problem.py:93-97, 137-140)."""
    from moeva2_amd.attacks.moeva2.classifier import Classifier
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2

    p = Project("lcld")
    B, G, P, O = 8, 4, 203, 100
    X = p.x[:B]
    model = os.path.join(RES, PROJECTS["lcld"][1])
    host = Moeva2(model, _host_lcld_constraints() if which == "constraints"
                  else make_constraints("lcld"), ml_scaler=make_scaler("lcld"), norm=2,
                  n_gen=G, n_pop=200, n_offsprings=O, seed=4, save_history="full")
    if which == "classifier":
        host._classifier = Classifier(_NumpyMLP("lcld"))
    dev = Moeva2(model, make_constraints("lcld"), ml_scaler=make_scaler("lcld"), norm=2,
                 n_gen=G, n_pop=200, n_offsprings=O, seed=4, save_history="full")
    gh, Fh, Hh = host.generate(X, 1, return_device=True)
    gd, Fd, Hd = dev.generate(X, 1, return_device=True)
    gh, Fh, gd, Fd, Hh, Hd = (t.cpu().numpy() for t in (gh, Fh, gd, Fd, Hh, Hd))
    assert Hh.shape == Hd.shape == (B, P + (G - 1) * O, 3 + 10)
    same = [b for b in range(B) if np.array_equal(gh[b], gd[b])]
    best_h, best_d = Fh[:, :, 0].min(axis=1), Fd[:, :, 0].min(axis=1)
    print(which, "identical final populations", len(same), "/", B, "mean best f1 host",
          best_h.mean(), "device", best_d.mean())
    assert len(same) >= B // 2
    # every state, diverged or not, reaches the same progress
    assert abs(best_h.mean() - best_d.mean()) <= 0.02, (best_h, best_d)
    for b in same:
        np.testing.assert_allclose(Fh[b], Fd[b], rtol=1e-5, atol=1e-12)
        np.testing.assert_allclose(Hh[b, :, 3:], Hd[b, :, 3:], rtol=1e-12, atol=1e-12)
    for b in range(B):  # host columns are the plugin's values on the final population
        x_f = mo.genetic_to_ml(p.lay, gh[b], X[b])
        if which == "constraints":
            gg = mo.lcld_constraints(x_f)
            np.testing.assert_array_equal(Fh[b, :, 2], (gg * (gg > 0)).sum(1))
            # history: G columns sum to f3; the initial rows are the clamped plugin G of x_init
            np.testing.assert_array_equal(Hh[b, :, 3:].sum(1), Hh[b, :, 2])
            x0 = mo.genetic_to_ml(p.lay, mo.initial_population(p.problem(X[b]), P), X[b])
            g0 = mo.lcld_constraints(x0)
            np.testing.assert_array_equal(Hh[b, :P, 3:], g0 * (g0 > 0))
        else:
            sc, mn = p.ml
            f1 = mo.mlp_predict_proba(x_f * sc + mn, p.weights, p.biases)[:, 1]
            np.testing.assert_array_equal(Fh[b, :, 0], f1.astype(np.float64))


def _objcalc(name, norm=2, thr=(0.5, 4), ml=True):
    from moeva2_amd.attacks.moeva2.objective_calculator import ObjectiveCalculator

    sc = make_scaler(name)
    return ObjectiveCalculator(make_classifier(name), make_constraints(name), minimize_class=1,
                               thresholds={"f1": thr[0], "f2": thr[1]}, min_max_scaler=sc,
                               norm=norm, ml_scaler=sc if ml else None)


def _check_obj(obj, ref):
    """CV and f2 are fp64 sums (order differs from numpy): 1e-12 relative; f1 is fp32."""
    np.testing.assert_allclose(obj[..., 0], ref[..., 0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(obj[..., 1], ref[..., 1], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(obj[..., 2], ref[..., 2], rtol=1e-12, atol=1e-15)


def test_objective_calculator_matches_reference_golden(golden):
    """Device ObjectiveCalculator (mv_objcalc_run) against the reference's own
    ObjectiveCalculator outputs (objective_calculator.py:44-119, golden vectors)."""
    d = golden("objective_calculator_botnet.npz")
    calc = _objcalc("botnet")
    obj = calc.calculate_objectives_3d(d["x_init"], d["x_attacks"])
    for i in range(4):
        _check_obj(obj[i], d[f"obj{i}"])
        np.testing.assert_array_equal(calc._objective_respected(obj[i]), d[f"resp{i}"])
        np.testing.assert_array_equal(calc._objective_array(d["x_init"][i], d["x_attacks"][i]),
                                      d[f"resp{i}"])
    np.testing.assert_array_equal(calc.success_rate_3d(d["x_init"], d["x_attacks"]),
                                  d["success_rate"])
    assert list(calc.success_rate_3d_df(d["x_init"], d["x_attacks"]).columns) == \
        [f"o{i}" for i in range(1, 8)]
    sa, idx = calc.get_successful_attacks(d["x_init"], d["x_attacks"],
                                          return_index_success=True)
    assert idx.shape == (4,) and sa.shape[1] == 756


@pytest.mark.parametrize("norm", [2, np.inf])
def test_objective_calculator_lcld_ohe_against_oracle(norm):
    """LCLD carries one-hot groups (utils.py:43-54): device objectives of attacked
    populations against the oracle restatement, L2 and Linf, plus the success rates."""
    p = Project("lcld")
    X = p.x[:12]
    _, g, _, _, _ = _attack("lcld", X, 6, 11, P=23, O=10)
    genes = g.cpu().numpy()
    xs = np.stack([mo.genetic_to_ml(p.lay, genes[b], X[b]) for b in range(X.shape[0])])
    xs[:, 0] = X  # one exact origin per state
    sc, mn = p.ml
    calc = _objcalc("lcld", norm=norm, thr=(0.25, 0.2))
    obj = calc.calculate_objectives_3d(X, xs)

    def fn(xi, x):
        return mo.objectives_calc(xi, x, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, "inf" if norm == np.inf else 2)

    for b in range(X.shape[0]):
        _check_obj(obj[b], fn(X[b], xs[b]))
    np.testing.assert_array_equal(calc.success_rate_3d(X, xs),
                                  mo.success_rate_3d(X, xs, fn, 0.25, 0.2))
    # ragged list input takes the per-state path and agrees
    np.testing.assert_array_equal(calc.success_rate_3d(X, [e for e in xs]),
                                  calc.success_rate_3d(X, xs))


def test_objective_calculator_range_assert():
    """objective_calculator.py:72-76: a candidate outside the scaler range raises."""
    p = Project("lcld")
    X = p.x[:2]
    xs = np.repeat(X[:, None], 3, axis=1).copy()
    calc = _objcalc("lcld", thr=(0.25, 0.2))
    calc.calculate_objectives_3d(X, xs)
    sc, mn = p.ml
    j = int(np.argmax(sc))
    xs[1, 2, j] = (2.0 - mn[j]) / sc[j]  # scales to 2.0
    with pytest.raises(AssertionError):
        calc.calculate_objectives_3d(X, xs)
    # a NaN candidate fails the same np.all range asserts in the reference (NaN comparisons
    # are False), so it is never scored as a successful attack
    xs = np.repeat(X[:, None], 3, axis=1).copy()
    xs[0, 1, 0] = np.nan
    with pytest.raises(AssertionError):
        calc.calculate_objectives_3d(X, xs)


@pytest.mark.parametrize("which", ["constraints", "classifier", "both"])
def test_objective_calculator_host_plugins(which):
    """objective_calculator.py:44-64 scores any Constraints subclass and any predict_proba
    model: a constraints object without a device program is evaluated by its own
    ``evaluate``, a model that is not a Dense MLP by its own ``predict_proba``, on the host;
    the one-hot term, CV, scaling checks and f2 stay on the device (mv_objcalc_score).
    Objectives and success rates equal the oracle's restatement."""
    from moeva2_amd.attacks.moeva2.classifier import Classifier
    from moeva2_amd.attacks.moeva2.objective_calculator import ObjectiveCalculator

    p = Project("lcld")
    X = p.x[:10]
    _, g, _, _, _ = _attack("lcld", X, 5, 3, P=23, O=10)
    genes = g.cpu().numpy()
    xs = np.stack([mo.genetic_to_ml(p.lay, genes[b], X[b]) for b in range(X.shape[0])])
    sc, mn = p.ml
    cons = _host_lcld_constraints() if which in ("constraints", "both") else make_constraints("lcld")
    clf = (Classifier(_NumpyMLP("lcld")) if which in ("classifier", "both")
           else make_classifier("lcld"))
    scaler = make_scaler("lcld")
    calc = ObjectiveCalculator(clf, cons, 1, {"f1": 0.25, "f2": 0.2}, min_max_scaler=scaler,
                               norm=2, ml_scaler=scaler)
    _, ceng, mlp = calc._device()
    assert (ceng is None) == (which in ("constraints", "both"))
    assert (mlp is None) == (which in ("classifier", "both"))
    obj = calc.calculate_objectives_3d(X, xs)

    def fn(xi, x):
        return mo.objectives_calc(xi, x, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    for b in range(X.shape[0]):
        _check_obj(obj[b], fn(X[b], xs[b]))
    np.testing.assert_array_equal(calc.success_rate_3d(X, xs),
                                  mo.success_rate_3d(X, xs, fn, 0.25, 0.2))
    bad = xs.copy()
    bad[1, 2, int(np.argmax(sc))] = (2.0 - mn[int(np.argmax(sc))]) / sc[int(np.argmax(sc))]
    with pytest.raises(AssertionError):
        calc.calculate_objectives_3d(X, bad)


def test_moeva_driver_hosted_plugins(tmp_path, monkeypatch):
    """04_moeva.py end to end with host plugins: the attack (host-driven loop) and its
    success scoring (ObjectiveCalculator host fallback) run on a Constraints subclass
    without a device program and a predict_proba-only model; the metrics equal the oracle's
    success rates of the saved x_attacks."""
    import json

    from moeva2_amd.attacks.moeva2 import moeva2 as mv2
    from moeva2_amd.config_parser.config_parser import get_config, get_dict_hash
    from moeva2_amd.experiments.united import moeva_run

    monkeypatch.setattr(moeva_run, "_constraints", lambda *a, **k: _host_lcld_constraints())
    monkeypatch.setattr(moeva_run, "load_model", lambda path: _NumpyMLP("lcld"))
    monkeypatch.setattr(mv2, "load_model", lambda path: _NumpyMLP("lcld"))
    cfg_dir = os.path.join(os.path.dirname(RES), "config")
    c = get_config(["-c", f"{cfg_dir}/moeva.yaml", "-c", f"{cfg_dir}/rq1.lcld.static.yaml",
                    "-p", "seed=7", "-p", "budget=4", "-p", "n_initial_state=5",
                    "-p", f"dirs.results={tmp_path}", "-j", '{"eps_list":[0.2,0.4]}'])
    h = get_dict_hash(c)
    m = moeva_run.run(c, verbose=False)
    xa = np.load(tmp_path / f"x_attacks_moeva_{h}.npy")
    assert xa.shape == (5, 203, 47)
    on_disk = json.load(open(tmp_path / f"metrics_moeva_{h}.json"))
    p = Project("lcld")
    sc, mn = p.ml

    def fn(xi, x):
        return mo.objectives_calc(xi, x, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    for k, eps in enumerate((0.2, 0.4)):
        sr = mo.success_rate_3d(p.x[:5], xa, fn, 0.25, eps)
        np.testing.assert_array_equal([on_disk["objectives_list"][k][f"o{i}"]
                                       for i in range(1, 8)], sr)
        assert m["objectives_list"][k] == on_disk["objectives_list"][k]


def test_moeva_driver_outputs(tmp_path):
    """04_moeva.py:27-142 output contract: results / x_attacks / x_history / metrics /
    config files named by the config hash; metrics = ObjectiveCalculator success rates of
    x_attacks; a second run with the same config is skipped."""
    import json

    from moeva2_amd.config_parser.config_parser import get_config, get_dict_hash
    from moeva2_amd.experiments.united.moeva_run import run

    cfg_dir = os.path.join(os.path.dirname(RES), "config")
    c = get_config(["-c", f"{cfg_dir}/moeva.yaml", "-c", f"{cfg_dir}/rq1.lcld.static.yaml",
                    "-p", "seed=42", "-p", "budget=5", "-p", "n_initial_state=6",
                    "-p", f"dirs.results={tmp_path}", "-j", '{"eps_list":[0.2,0.4]}'])
    h = get_dict_hash(c)
    m = run(c, verbose=False)
    xa = np.load(tmp_path / f"x_attacks_moeva_{h}.npy")
    xh = np.load(tmp_path / f"x_history_moeva_{h}.npy")
    assert xa.shape == (6, 203, 47) and xh.shape == (6, 4, 100, 13)
    assert (tmp_path / f"results_{h}.npy").exists() and (tmp_path / f"config_moeva_{h}.yaml").exists()
    on_disk = json.load(open(tmp_path / f"metrics_moeva_{h}.json"))
    assert on_disk["config_hash"] == h and len(on_disk["objectives_list"]) == 2
    assert list(on_disk["objectives_list"][0]) == [f"o{i}" for i in range(1, 8)]
    p = Project("lcld")
    sc, mn = p.ml

    def fn(xi, x):
        return mo.objectives_calc(xi, x, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    for k, eps in enumerate((0.2, 0.4)):
        sr = mo.success_rate_3d(p.x[:6], xa, fn, 0.25, eps)
        np.testing.assert_array_equal([m["objectives_list"][k][f"o{i}"] for i in range(1, 8)], sr)
    assert run(c, verbose=False) is None


def test_moeva_driver_augmented_reconstruction(tmp_path):
    """rq4 form: lcld_augmented attack with the evaluation constraints and the
    reconstruction branch (04_moeva.py:43-53, 97-103, 116-120)."""
    from moeva2_amd.config_parser.config_parser import get_config, get_dict_hash
    from moeva2_amd.experiments.united.moeva_run import run

    cfg_dir = os.path.join(os.path.dirname(RES), "config")
    c = get_config(["-c", f"{cfg_dir}/rq4.lcld.moeva_augmented.yaml", "-p", "budget=3",
                    "-p", "n_initial_state=4", "-p", f"dirs.results={tmp_path}",
                    "-j", '{"reconstruction":true,"save_history":"reduced",'
                          '"paths":{"important_features":"./data/lcld/important_features.npy"}}'])
    m = run(c, verbose=False)
    xa = np.load(tmp_path / f"x_attacks_moeva_{get_dict_hash(c)}.npy")
    assert xa.shape == (4, 203, 57)
    # reconstructed XOR columns agree with augment_data of the base columns
    from moeva2_amd.examples.utils import augment_data

    imp = np.load(os.path.join(RES, "data/lcld/important_features.npy"))
    np.testing.assert_array_equal(xa, augment_data(xa[..., :47], imp))
    assert 0.0 <= m["objectives_list"][0]["o7"] <= 1.0


def test_attack_default_population_640(monkeypatch):
    """Moeva2's default n_pop 640 / n_offsprings 320 (moeva2.py:44-46): survival on the
    objective arrays of the oracle's attack is bit-exact, the device attack keeps its
    invariants and does not depend on the state grouping (HBM dominance scratch offsets)."""
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    p = Project("lcld")
    B, G, P, O, seed = 2, 3, 643, 320, 5
    ref = energy_ref_dirs(3, 640, seed=1)
    asp = np.full((1, 3), 1.0 / 3.0)
    seqs = [_oracle_attack_merges(p.problem(p.x[b]), ref, G, P, O, seed) for b in range(B)]
    state = dict(ideal=np.full((B, 3), np.inf), worst=np.full((B, 3), -np.inf),
                 extreme=np.zeros((B, 9)), has=np.zeros(B, np.int32))
    ost = [mo.SurvivalState() for _ in range(B)]
    for gen in range(G):
        F = np.stack([s[gen] for s in seqs])
        got = _run_survive(F, ref, P, seed, gen, state)
        for b in range(B):
            r = mo.survive(F[b], P, ost[b], ref, asp, 0.05, seed, gen)
            np.testing.assert_array_equal(got["surv"][b], r.survivors, f"gen {gen} state {b}")
    X = p.x[:5]
    monkeypatch.setenv("MV_GROUPS", "1")
    eng, g1, F1, _, _ = _attack("lcld", X, 4, 9, P=P, O=O)
    monkeypatch.setenv("MV_GROUPS", "4")
    _, g4, F4, _, _ = _attack("lcld", X, 4, 9, P=P, O=O)
    np.testing.assert_array_equal(g1.cpu().numpy(), g4.cpu().numpy())
    np.testing.assert_array_equal(F1.cpu().numpy(), F4.cpu().numpy())
    F2 = torch.empty_like(F1)
    eng.evaluate(g1, F2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(F2.cpu().numpy(), F1.cpu().numpy())


def test_success_rate_matches_oracle_attack_botnet():
    """The headline config's shape (botnet, P = 203, O = 100, L2, eps 4, thr 0.5): device
    attack vs the oracle's CPU attack on the same shipped states, budget and seed; o1..o7
    within max(1 pp, one state)."""
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    p = Project("botnet")
    B, G, P, O, seed = 12, 100, 203, 100, 3
    X = p.x[:B]
    _, g, _, _, ref = _attack("botnet", X, G, seed, P=P, O=O)
    np.testing.assert_array_equal(ref, energy_ref_dirs(3, 200, seed=1))
    genes = g.cpu().numpy()
    sc, mn = p.ml

    def fn(xi, xs):
        return mo.objectives_calc(xi, xs, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    x_dev, x_cpu = [], []
    for b in range(B):
        r = mo.run_attack(p.problem(X[b]), ref, G, P, O, seed)
        x_cpu.append(mo.genetic_to_ml(p.lay, r.pop_X, X[b]))
        x_dev.append(mo.genetic_to_ml(p.lay, genes[b], X[b]))
    sr_dev = mo.success_rate_3d(X, x_dev, fn, 0.5, 4)
    sr_cpu = mo.success_rate_3d(X, x_cpu, fn, 0.5, 4)
    # at this budget few botnet states flip (the reference runs 1000 generations), so also
    # compare the attack's progress: each state's best f1 in its final population
    best_dev = np.array([fn(X[b], x_dev[b])[:, 1].min() for b in range(B)])
    best_cpu = np.array([fn(X[b], x_cpu[b])[:, 1].min() for b in range(B)])
    print("o1..o7 dev", sr_dev, "cpu", sr_cpu, "best f1 dev", best_dev.mean(), "cpu",
          best_cpu.mean(), "max |diff|", np.abs(best_dev - best_cpu).max())
    assert np.all(np.abs(sr_dev - sr_cpu) <= max(0.01, 1.0 / B) + 1e-12), (sr_dev, sr_cpu)
    assert abs(best_dev.mean() - best_cpu.mean()) <= 0.01, (best_dev, best_cpu)
