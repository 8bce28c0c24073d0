"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every symbol
declared in include/moeva_mi355x.h (no compute calls), the host-side builders
(device constraint programs, genetic layout) restate the reference, and the API mirror's
argument checks behave like src/attacks/moeva2/moeva2.py."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, PKG, RES, ROOT
from oracle import moeva_oracle as mo
from oracle.problems import Project

HEADER = os.path.join(ROOT, "include", "moeva_mi355x.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mv_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from moeva2_amd import _native

    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_native.EXPORTED)


# ---------------------------------------------------------------------------------------
# numpy statement of the device op program (mirrors csrc/eval.hip eval_op) -- test only
def run_program(prog, x):
    code, arg, k, pool = prog.arrays()
    out = np.zeros((x.shape[0], len(code)))
    with np.errstate(divide="ignore", invalid="ignore"):
        for c, (op, a, kk) in enumerate(zip(code, arg, k)):
            if op == 1:
                v = x[:, a[0]] - x[:, a[1]]
            elif op == 2:
                b = x[:, a[1]]
                v = np.where(b != 0, x[:, a[0]] / np.where(b != 0, b, 1), 0.0) - kk[0]
            elif op == 3:
                v = np.abs(x[:, pool[a[0]:a[1]]].sum(1) - x[:, pool[a[1]:a[2]]].sum(1))
            elif op == 4:
                r = x[:, a[2]] / 1200.0
                base = 1.0 + x[:, a[2]] / 1200.0
                v = np.abs(x[:, a[3]] - (x[:, a[0]] * r) * base ** x[:, a[1]]
                           / (base ** x[:, a[1]] - 1.0)) - kk[0]
            elif op == 5:
                v = np.abs((36.0 - x[:, a[0]]) * (60.0 - x[:, a[0]]))
            elif op == 6:
                v = np.abs(x[:, a[0]] - x[:, a[1]] / x[:, a[2]])
            elif op == 7:
                m = lambda f: np.floor(f / 100.0) * 12.0 + np.remainder(f, 100.0)  # noqa
                v = np.abs(x[:, a[0]] - (m(x[:, a[1]]) - m(x[:, a[2]])))
            elif op == 8:
                den = x[:, a[2]]
                ratio = np.where(den != 0, x[:, a[1]] / np.where(den != 0, den, 1), -1.0)
                ratio[(ratio == np.inf) | np.isnan(ratio)] = -1.0
                v = np.abs(x[:, a[0]] - ratio)
            elif op == 9:
                v = np.abs(x[:, a[0]] - ((x[:, a[1]] >= kk[0]) != (x[:, a[2]] >= kk[1])))
            else:
                raise AssertionError(op)
            out[:, c] = v
    out[out <= 1e-3] = 0.0
    return out


@pytest.mark.parametrize("name,cls,fixture,ncons", [
    ("lcld", "LcldConstraints", "lcld_constraints.npz", 10),
    ("lcld_augmented", "LcldAugmentedConstraints", "lcld_aug_constraints.npz", 20),
    ("botnet", "BotnetConstraints", "botnet_constraints.npz", 360),
    ("botnet_augmented", "BotnetAugmentedConstraints", "botnet_aug_constraints.npz", 531),
])
def test_device_constraint_programs_restate_reference(golden, name, cls, fixture, ncons):
    from moeva2_amd.experiments.united.utils import STR_TO_CONSTRAINTS_CLASS
    from oracle.problems import PROJECTS

    feat = os.path.join(RES, PROJECTS[name][0])
    cons = feat.replace("features", "constraints")
    c = STR_TO_CONSTRAINTS_CLASS[name](feat, cons)
    assert type(c).__name__ == cls
    prog = c.device_program()
    assert len(prog) == ncons == c.get_nb_constraints()
    d = golden(fixture)
    g = run_program(prog, d["x"])
    np.testing.assert_array_equal(g > 0, d["g"] > 0)
    np.testing.assert_allclose(g, d["g"], rtol=1e-13, atol=0)


@pytest.mark.parametrize("name,fixture", [("botnet", "problem_botnet.npz"),
                                          ("lcld", "problem_lcld.npz"),
                                          ("lcld_augmented", "problem_lcld_aug.npz")])
def test_feature_encoder_mirror(golden, name, fixture):
    from moeva2_amd.attacks.moeva2.feature_encoder import get_encoder_from_constraints
    from moeva2_amd.experiments.united.utils import STR_TO_CONSTRAINTS_CLASS
    from oracle.problems import PROJECTS

    feat = os.path.join(RES, PROJECTS[name][0])
    c = STR_TO_CONSTRAINTS_CLASS[name](feat, feat.replace("features", "constraints"))
    d = golden(fixture)
    for s, x in enumerate(d["x_init"]):
        enc = get_encoder_from_constraints(c, x)
        xl, xu = enc.get_min_max_genetic()
        np.testing.assert_array_equal(xl, d[f"s{s}_xl"])
        np.testing.assert_array_equal(xu, d[f"s{s}_xu"])
        t = enc.get_type_mask_genetic()
        np.testing.assert_array_equal(np.array([v == "real" for v in t]), d[f"s{s}_isreal"])
        np.testing.assert_array_equal(enc.ml_to_genetic(x[None])[0], d[f"s{s}_g0"])
        np.testing.assert_array_equal(enc.genetic_to_ml(d[f"s{s}_genes"], x), d[f"s{s}_x_ml"])
        kind, feat_, offs, ohe_feats, mut = enc.device_layout()
        assert kind.shape[0] == enc.get_genetic_v_length()
        assert np.all(np.diff(mut) > 0)


def test_moeva2_argument_checks_match_reference():
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2
    from moeva2_amd.examples.lcld.lcld_constraints import LcldConstraints

    feat = os.path.join(RES, "data/lcld/features.csv")
    c = LcldConstraints(feat, os.path.join(RES, "data/lcld/constraints.csv"))
    m = Moeva2(os.path.join(RES, "models/lcld/nn.npz"), c, n_gen=2, n_pop=10, n_offsprings=4)
    x = np.zeros((3, 47))
    with pytest.raises(ValueError):  # moeva2.py:179-182
        m.generate(x, np.array([1, 1]))
    with pytest.raises(ValueError):  # moeva2.py:74-79
        m.generate(np.zeros((3, 40)), 1)
    assert m.pop_size() == 13


def test_scaler_and_history_helpers():
    from moeva2_amd.attacks.moeva2.utils import (get_one_hot_encoding_constraints,
                                                 get_scaler_from_norm, results_to_history)

    s = get_scaler_from_norm(2, 756)
    np.testing.assert_array_equal(s.transform(np.array([[3.0]])),
                                  np.array([[3.0 * (1.0 / np.sqrt(756))]]))
    assert get_scaler_from_norm(np.inf, 10).transform(np.array([[0.5]]))[0, 0] == 0.5
    types = np.array(["real", "ohe0", "ohe0", "ohe1", "ohe1"], dtype=object)
    x = np.array([[0.3, 1, 0, 1, 1], [0.0, 0, 0, 0, 1]], float)
    np.testing.assert_array_equal(get_one_hot_encoding_constraints(types, x),
                                  mo.ohe_distance(types, x))

    class R:
        history = [np.zeros((5, 3)), np.ones((2, 3)), 2 * np.ones((2, 3))]

    h = results_to_history([R(), R()])
    assert h.shape == (2, 2, 2, 3)


def test_energy_ref_dirs_on_simplex():
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    for n in (200, 640):
        r = energy_ref_dirs(3, n, seed=1)
        assert r.shape == (n, 3)
        np.testing.assert_allclose(r.sum(1), 1.0, atol=1e-12)
        assert r.min() >= 0.0
        d = np.sqrt(((r[:, None] - r[None]) ** 2).sum(-1))
        np.fill_diagonal(d, np.inf)
        assert d.min() > 0.01  # well spread, no duplicates


def test_safe_loaders_execute_nothing():
    """The reference's pickles are decoded by an opcode walker: GLOBAL+REDUCE become inert
    records (nothing is imported or called)."""
    import pickle

    from moeva2_amd.io.safe_pickle import Obj, safe_load

    p = os.path.join(ROOT, "tests", ".tmp_evil.pkl")
    with open(p, "wb") as f:
        f.write(pickle.dumps({"a": [1, 2, 3]}, protocol=4))
    assert safe_load(p) == {"a": [1, 2, 3]}
    with open(p, "wb") as f:  # os.system('true') pickle
        f.write(b"cos\nsystem\n(S'true'\ntR.")
    try:
        rec = safe_load(p)
        assert isinstance(rec, Obj) and rec.cls == "os.system" and rec.args == ("true",)
    finally:
        os.remove(p)


def test_objective_calculator_device_path_refuses_host_or_mixed_tensors():
    """calculate_objectives_device runs on the GPU its tensors live on and builds its device
    objects there; host tensors (or tensors of two devices) are refused before any engine
    call (the objects used to be built on device 0 whatever the tensors' GPU)."""
    import torch

    from moeva2_amd.attacks.moeva2.objective_calculator import ObjectiveCalculator

    class _Cons:
        def get_feature_type(self):
            return np.array(["real"] * 4)

        def get_mutable_mask(self):
            return np.ones(4, bool)

    calc = ObjectiveCalculator.__new__(ObjectiveCalculator)
    calc._devs = {}
    with pytest.raises(ValueError, match="one GPU"):
        calc.calculate_objectives_device(torch.zeros(2, 4, dtype=torch.float64),
                                         torch.zeros(2, 3, 4, dtype=torch.float64))
    assert calc._devs == {}
