"""The premise of the attack's compact gene layout (csrc/api.cpp stored_genes,
mv_get_stored_genes), checked on the reference-faithful oracle (CPU, no engine): an integer
gene whose bounds are equal and whose initial value is that bound in every state never
changes -- two-point crossover and SBX exchange equal values, polynomial mutation of an
integer gene is rounded and clamped back into [xl, xu] = {value}
(softmax_mutation.py:60-108, moeva2.py:90-111) -- so the attack may leave it out of the
pool and evaluate its feature as immutable."""
import numpy as np
import pytest

from oracle import moeva_oracle as mo
from oracle.problems import Project


def fixed_genes(p, X):
    """stored_genes' rule restated: integer genes with xl == xu == x_init in every state."""
    types = np.asarray(mo.genetic_types(p.lay))
    fixed = types == "int"
    for x in X:
        prob = p.problem(x)
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        g0 = mo.ml_to_genetic(p.lay, x[None, :])[0]
        fixed &= (gl == gu) & (g0 == gl) & (np.rint(g0) == g0)
    return fixed


@pytest.fixture(scope="module")
def botnet():
    return Project("botnet")


def test_fixed_gene_counts():
    """botnet / botnet_augmented: 120 of the genes are fixed on the shipped states (features
    whose dataset minimum equals maximum); the LCLD problems have none."""
    for name, n in [("botnet", 120), ("botnet_augmented", 120), ("lcld", 0)]:
        p = Project(name)
        assert fixed_genes(p, p.x[:64]).sum() == n, name


@pytest.mark.parametrize("kind", ["two_point", "sbx"])
def test_variation_never_moves_fixed_genes(botnet, kind):
    """Crossover + mutation of 4000 children (each fixed gene is drawn for mutation ~9
    times): the fixed genes keep their bound, bit for bit."""
    p = botnet
    X = p.x[:3]
    fixed = fixed_genes(p, X)
    types = mo.genetic_types(p.lay)
    masks = [np.array([t == "real" for t in types]), np.array([t == "int" for t in types])]
    rng = np.random.default_rng(5)
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, gu = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        pop = rng.uniform(gl, gu, size=(60, gl.shape[0]))
        pop[:, masks[1]] = np.round(pop[:, masks[1]])
        pop[:, fixed] = gl[fixed]
        par = rng.integers(0, 60, size=(2000, 2))
        pX = np.stack([pop[par[:, 0]], pop[par[:, 1]]])
        if kind == "sbx":
            off = mo.sbx_crossover(pX, masks, gl, gu, 11 + b, 3)
        else:
            off = mo.crossover(pX, masks, 11 + b, 3)
        do, _ = mo.mutation_draws(off.shape[0], gl.shape[0], 11 + b, 3)
        assert do[:, fixed].sum() > 100  # the fixed genes are drawn for mutation
        off = mo.mutation(off, gl, gu, types, 11 + b, 3)
        np.testing.assert_array_equal(off[:, fixed], np.broadcast_to(gl[fixed], off[:, fixed].shape))


def test_oracle_attack_keeps_fixed_genes(botnet):
    """A whole oracle attack (pymoo loop restated) on two botnet states: the final
    populations hold every fixed gene at its bound."""
    p = botnet
    X = p.x[:2]
    fixed = fixed_genes(p, X)
    ref = mo_ref(20)
    for b in range(X.shape[0]):
        prob = p.problem(X[b])
        gl, _ = mo.genetic_bounds(p.lay, prob.xl, prob.xu)
        r = mo.run_attack(prob, ref, 6, 23, 10, 9)
        np.testing.assert_array_equal(r.pop_X[:, fixed],
                                      np.broadcast_to(gl[fixed], r.pop_X[:, fixed].shape))


def mo_ref(n):
    from moeva2_amd.attacks.moeva2.ref_dirs import riesz_energy_dirs

    return riesz_energy_dirs(3, n, seed=1, n_max_iter=50)
