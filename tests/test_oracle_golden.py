"""Pin the CPU oracle against golden vectors produced by the REFERENCE's own code
(tests/golden/make_golden.py imports src/attacks/moeva2/* and src/examples/*)."""
import numpy as np
import pytest

from oracle import moeva_oracle as mo
from oracle.problems import Project


@pytest.fixture(scope="module")
def projects():
    return {n: Project(n) for n in ("lcld", "lcld_augmented", "botnet", "botnet_augmented")}


@pytest.mark.parametrize("name,fixture", [
    ("botnet", "botnet_constraints.npz"),
    ("botnet_augmented", "botnet_aug_constraints.npz"),
    ("lcld", "lcld_constraints.npz"),
    ("lcld_augmented", "lcld_aug_constraints.npz"),
])
def test_constraints_match_reference(projects, golden, name, fixture):
    d = golden(fixture)
    g = projects[name].constraints(d["x"])
    assert g.shape == d["g"].shape
    np.testing.assert_array_equal(g > 0, d["g"] > 0)  # satisfied masks: exact
    np.testing.assert_allclose(g, d["g"], rtol=1e-13, atol=0)


def test_augment_data_matches_reference(projects, golden):
    d = golden("lcld_aug_constraints.npz")
    out = mo.augment_data(d["augmented"][:, :47], projects["lcld"].important)
    np.testing.assert_array_equal(out, d["augmented"])


@pytest.mark.parametrize("name,fixture", [
    ("botnet", "problem_botnet.npz"), ("lcld", "problem_lcld.npz"),
    ("lcld_augmented", "problem_lcld_aug.npz")])
def test_encoder_and_evaluate_match_reference(projects, golden, name, fixture):
    d = golden(fixture)
    p = projects[name]
    for s, x in enumerate(d["x_init"]):
        for norm, tag in ((2, "l2"), (np.inf, "linf")):
            prob = p.problem(x, norm=norm)
            gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
            np.testing.assert_array_equal(gl, d[f"s{s}_xl"])
            np.testing.assert_array_equal(gu, d[f"s{s}_xu"])
            types = mo.genetic_types(p.lay)
            np.testing.assert_array_equal(np.array([t == "real" for t in types]),
                                          d[f"s{s}_isreal"])
            np.testing.assert_array_equal(mo.ml_to_genetic(p.lay, x)[0], d[f"s{s}_g0"])
            genes = d[f"s{s}_genes"]
            np.testing.assert_array_equal(mo.genetic_to_ml(p.lay, genes, x), d[f"s{s}_x_ml"])
            F, G = mo.evaluate(prob, genes, return_g=True)
            ref = d[f"s{s}_F_{tag}"]
            np.testing.assert_allclose(F[:, 0], ref[:, 0], rtol=1e-5, atol=1e-7)  # fp32 MLP
            np.testing.assert_allclose(F[:, 1], ref[:, 1], rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(F[:, 2], ref[:, 2], rtol=1e-12, atol=0)
            hist = d[f"s{s}_hist_{tag}"]
            np.testing.assert_array_equal(G > 0, hist[:, 3:] > 0)
            np.testing.assert_allclose(G, hist[:, 3:], rtol=1e-12, atol=0)


def test_dominance_matches_reference(golden):
    d = golden("dominance.npz")
    np.testing.assert_array_equal(mo.domination_matrix(d["f"]), d["m"])


def test_polynomial_mutation_matches_reference(golden):
    d = golden("polynomial_mutation.npz")
    for k in range(2):
        y = mo.polynomial_mutation(d[f"c{k}_x"], d[f"c{k}_xl"], d[f"c{k}_xu"], 20.0,
                                   d[f"c{k}_do"], d[f"c{k}_rand"])
        # np.power is libm/SVML-build dependent in the last bits (numpy 1.26 vs 2.2 here)
        np.testing.assert_allclose(y, d[f"c{k}_y"], rtol=1e-13, atol=1e-14)


def test_two_point_crossover_matches_reference(golden):
    d = golden("two_point_crossover.npz")
    for k in range(3):
        X = d[f"c{k}_x"]
        _, nm, nv = X.shape
        M = mo.two_point_mask(nv, nm, d[f"c{k}_cuts"])
        y0 = np.where(M, X[1], X[0])
        y1 = np.where(M, X[0], X[1])
        np.testing.assert_array_equal(np.stack([y0, y1]), d[f"c{k}_y"])


def test_objective_calculator_matches_reference(projects, golden):
    d = golden("objective_calculator_botnet.npz")
    p = projects["botnet"]
    sc, mn = p.ml

    def fn(xi, xs):
        return mo.objectives_calc(xi, xs, p.constraints, p.types, sc, mn, p.weights, p.biases,
                                  1, sc, mn, 2)

    for i in range(4):
        obj = fn(d["x_init"][i], d["x_attacks"][i])
        np.testing.assert_allclose(obj, d[f"obj{i}"], rtol=1e-5, atol=1e-9)
        np.testing.assert_array_equal(mo.objectives_respected(obj, 0.5, 4), d[f"resp{i}"])
    sr = mo.success_rate_3d(d["x_init"], d["x_attacks"], fn, 0.5, 4)
    np.testing.assert_array_equal(sr, d["success_rate"])


def test_lu_solve3_matches_numpy():
    rng = np.random.default_rng(0)
    for _ in range(200):
        M = rng.normal(size=(3, 3))
        b = np.ones(3)
        np.testing.assert_allclose(mo.lu_solve3(M, b), np.linalg.solve(M, b), rtol=1e-9)
    assert mo.lu_solve3(np.zeros((3, 3)), np.ones(3)) is None


def test_nds_fronts_partition_and_order():
    rng = np.random.default_rng(1)
    F = rng.integers(0, 5, size=(120, 3)).astype(float)
    fronts, rank = mo.fast_non_dominated_sort(F, 10 ** 8)
    allf = np.concatenate(fronts)
    assert sorted(allf.tolist()) == list(range(120))
    M = mo.domination_matrix(F)
    for i, f in enumerate(fronts):
        for j in f:  # nobody in the same or a later front dominates j
            dom = np.where(M[:, j] == 1)[0]
            assert np.all(rank[dom] < i)
    assert list(fronts[0]) == sorted(fronts[0])
