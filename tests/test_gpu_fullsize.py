"""Full-size correctness of the non-headline BASELINE configs: every
state of configs[2], [3] and [4] at its full state count, so the size-specific paths run
under a check -- configs[3]'s HBM dominance scratch (100,000 x 963 x 16 words, 12.3 GB),
configs[2]'s full history (4,000 states x 100 generations, 7.4 GB), the grid and 64-bit
offset arithmetic at these B.  For each:
  * batch invariance: states {0, B/2, B-1} are bit-identical to a B = 3 run of the same
    states (every draw is keyed by the row inside its state, so a state's attack does not
    depend on the batch);
  * the final F equals mv_evaluate of the final genes (bit-exact in the full gene layout;
    configs[4]'s compact layout folds its fixed features, so f1 to 1e-5 / f2 to 1e-12 / f3
    exact, as tests/test_gpu_parity.py::test_compact_layout_tracks_full_layout);
  * genes inside the genetic bounds, integer genes integral, everything finite;
  * pinned to the oracle: states {0, B/2, B-1} of the full-size run
    against oracle/device_order's engine-order attack of the same states, seed and budget
    (configs[2] / [3]: final genes, f1, f2 and the history's f1 / f2 bit-identical; f3 and
    G to 1e-12 relative: the device's pow in the LCLD installment identity is its libm's,
    the restatement's np.power); configs[4]'s 512-wide
    classifier runs k_mlp, whose summation order the engine-order restatement does not
    cover, so there the picked states' final F is checked against the oracle's evaluation in
    the reference's arithmetic (f1 1e-5 relative, f2 / f3 1e-12: north_star's tolerances).
Reference shapes: config/rq4.lcld.moeva_augmented.yaml:12-14 (4,000 states),
src/attacks/moeva2/moeva2.py:44-46 (the 640 / 320 defaults of configs[3])."""
import dataclasses
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import moeva_oracle as mo
from oracle.problems import Project

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def bounds_batch(c, X):
    """Constraints.get_feature_min_max(dynamic_input=x) for every row of X, vectorised
    (lcld_constraints.py:237-263: 'dynamic' bounds are the input itself)."""
    fmin, fmax = c._feature_min, c._feature_max
    mind = fmin.astype(str) == "dynamic"
    maxd = fmax.astype(str) == "dynamic"
    lo = np.zeros(fmin.shape[0])
    hi = np.zeros(fmax.shape[0])
    lo[~mind] = fmin[~mind].astype(np.float64)
    hi[~maxd] = fmax[~maxd].astype(np.float64)
    xl = np.repeat(lo[None], X.shape[0], 0)
    xu = np.repeat(hi[None], X.shape[0], 0)
    xl[:, mind] = X[:, mind]
    xu[:, maxd] = X[:, maxd]
    return xl, xu


def genetic_bounds_batch(lay, xl, xu):
    """oracle genetic_bounds (feature_encoder.py:145-163) for every row."""
    mxl, mxu = xl[:, lay.mutable_mask], xu[:, lay.mutable_mask]
    n = int(lay.no_ohe_mask.sum())
    gl = np.empty((xl.shape[0], lay.V))
    gu = np.empty((xl.shape[0], lay.V))
    gl[:, :n] = mxl[:, lay.no_ohe_mask]
    gu[:, :n] = mxu[:, lay.no_ohe_mask]
    for k, m in enumerate(lay.ohe_masks):
        gl[:, n + k] = 0.0
        gu[:, n + k] = m.shape[0] - 1
    return gl, gu


def run(workload, X, n_gen, hist):
    """One attack of the bench workload's engine on states X: (engine, genes, F, history)
    on the device."""
    import bench
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    w = bench.WORKLOADS[workload]
    eng, c = bench.build_engine(w, 0)
    xl, xu = bounds_batch(c, X)
    eng.set_states(X, xl, xu, 1)
    P, O = w["n_pop"] + 3, w["n_off"]
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    eng.attack_run(n_gen, P, O, 42, ref, 0.05, hist)
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
    return eng, c, g, F, h


def oracle_attack(workload, project, c, X, picks, n_gen, hist):
    """The engine-order oracle attack (oracle/device_order.py: the engine's summation orders
    and det_pow; moeva_oracle.run_attack: the same Philox draws) of the picked states."""
    import bench
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs
    from moeva2_amd.problem import build_device_program
    from oracle import device_order as do

    w = bench.WORKLOADS[workload]
    p = Project(project)
    codes = build_device_program(c).op_code
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)

    def ev(prob, genes, return_g=False):
        return do.evaluate_device_order(prob, genes, codes, return_g)

    mode = {0: None, 1: "reduced", 2: "full"}[hist]
    return [mo.run_attack(p.problem(X[b], norm=w["norm"]), ref, n_gen, w["n_pop"] + 3,
                          w["n_off"], 42, save_history=mode, evaluate_fn=ev,
                          pow_fn=do.det_pow) for b in picks]


def check_full(workload, project, n_states, n_gen, hist, compact, pin="attack"):
    import bench

    X = bench.load_states(dict(bench.WORKLOADS[workload], n_states=n_states))
    B = X.shape[0]
    assert B == n_states
    pick = [0, B // 2, B - 1]
    eng, c, g, F, h = run(workload, X, n_gen, hist)
    assert bool(torch.isfinite(g).all()) and bool(torch.isfinite(F).all())
    # F == re-evaluation of the final genes (mv_evaluate: the full gene layout), all states
    F2 = torch.empty_like(F)
    eng.evaluate(g, F2)
    torch.cuda.synchronize()
    if compact:
        torch.testing.assert_close(F[..., 0], F2[..., 0], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(F[..., 1], F2[..., 1], rtol=1e-12, atol=1e-15)
        assert torch.equal(F[..., 2], F2[..., 2])
    else:
        assert torch.equal(F, F2)
    # bounds and integrality, all states
    p = Project(project)
    xl, xu = bounds_batch(c, X)
    gl, gu = genetic_bounds_batch(p.lay, xl, xu)
    gl_d, gu_d = torch.from_numpy(gl).cuda()[:, None, :], torch.from_numpy(gu).cuda()[:, None, :]
    assert bool(((g >= gl_d) & (g <= gu_d)).all())
    isr = torch.from_numpy(np.array([t == "real" for t in mo.genetic_types(p.lay)])).cuda()
    gi = g[..., ~isr]
    assert torch.equal(gi, torch.round(gi))
    # batch invariance: the three picked states alone
    gs, Fs, hs = g[pick].cpu().numpy(), F[pick].cpu().numpy(), None
    if h is not None:
        hs = h[pick].cpu().numpy()
    del g, F, F2, h, gl_d, gu_d
    eng3, _, g3, F3, h3 = run(workload, np.ascontiguousarray(X[pick]), n_gen, hist)
    np.testing.assert_array_equal(g3.cpu().numpy(), gs)
    np.testing.assert_array_equal(F3.cpu().numpy(), Fs)
    if hs is not None:
        np.testing.assert_array_equal(h3.cpu().numpy(), hs)
        assert np.isfinite(hs).all()
    del g3, F3, h3, eng3
    torch.cuda.empty_cache()
    # pinned to the oracle on the picked states
    if pin == "attack":
        for k, r in enumerate(oracle_attack(workload, project, c, X, pick, n_gen, hist)):
            np.testing.assert_array_equal(gs[k], r.pop_X)  # the whole trajectory
            np.testing.assert_array_equal(Fs[k][:, :2], r.pop_F[:, :2])
            # f3 and G: the LCLD installment identity's pow is the device libm's (numpy's
            # np.power in the restatement), ~1 ulp apart before its cancellation
            np.testing.assert_allclose(Fs[k][:, 2], r.pop_F[:, 2], rtol=1e-12, atol=0)
            if hs is not None:
                hr = np.concatenate(r.history)
                np.testing.assert_array_equal(hs[k][:, :2], hr[:, :2])
                np.testing.assert_allclose(hs[k][:, 2:], hr[:, 2:], rtol=1e-12, atol=0)
    elif pin == "evaluate":
        import bench

        W = bench.synthetic_mlp(bench.WORKLOADS[workload]["model"])
        for k, b in enumerate(pick):
            prob = p.problem(X[b], norm=bench.WORKLOADS[workload]["norm"])
            prob = dataclasses.replace(prob, weights=W.weights, biases=W.biases)
            ref = mo.evaluate(prob, gs[k])
            np.testing.assert_allclose(Fs[k][:, 0], ref[:, 0], rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(Fs[k][:, 1:], ref[:, 1:], rtol=1e-12, atol=1e-15)
    return eng


def test_configs3_scaleout_full_state_count():
    """configs[3]: 100,000 LCLD-shaped states x P 643 / O 320 (N = 963: the dominance
    bitsets in the 12.3 GB HBM scratch), 3 generations."""
    eng = check_full("synthetic.lcld.scaleout", "lcld", 100000, 3, 0, compact=False)
    assert eng.stored_genes().all()


def test_configs2_augmented_full_history():
    """configs[2]: rq4.lcld.moeva_augmented, all 4,000 states, the full 100-generation budget
    with the full history (F | G per evaluation, 7.4 GB)."""
    check_full("rq4.lcld.moeva_augmented", "lcld_augmented", 4000, 100, 2, compact=False)


def test_configs4_wide_mlp_full_state_count():
    """configs[4]: 10,000 botnet-shaped states with the 756-512-512-256-2 MLP (k_mlp), 3
    generations, compact gene layout."""
    eng = check_full("synthetic.botnet.wide", "botnet", 10000, 3, 0, compact=True,
                     pin="evaluate")
    assert (~eng.stored_genes()).sum() == 120
