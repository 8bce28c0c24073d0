"""Generate golden vectors by importing the REFERENCE's own numpy hot-path code.

Run in THIS container only (the reference never travels to the GPU box):

    cd /root/reference && PYTHONPATH=/root/reference:/root/repo/tests/golden/refstubs \
        /opt/conda/bin/python3.9 /root/repo/tests/golden/make_golden.py

Python 3.9 + numpy 1.26 + scikit-learn 0.24.2 (the survey-time environment).
TensorFlow / pymoo / autograd are absent: ``refstubs/`` provides import-time names only.
Reference-shipped pickles are NOT unpickled: ``feat_idx`` comes from the repo's JSON
conversion (tools/import_reference_data.py), scalers from the repo's ``.npz``
conversion; the Keras classifier is a numpy fp32 forward of the converted weights.

Outputs (small .npz) land next to this script.  What each one pins is listed in
tests/golden/README.md.
"""
import json
import os
import sys

import numpy as np

np.float = float  # numpy>=1.24 removed these aliases; the reference still uses them
np.bool = bool
np.int = int

from sklearn.preprocessing import MinMaxScaler  # noqa: E402

from src.attacks.moeva2 import default_problem as dp  # noqa: E402
from src.attacks.moeva2 import feature_encoder as fe  # noqa: E402
from src.attacks.moeva2 import objective_calculator as oc  # noqa: E402
from src.attacks.moeva2 import pareto_operation as po  # noqa: E402
from src.attacks.moeva2 import softmax_crossover as sxc  # noqa: E402
from src.attacks.moeva2 import softmax_mutation as sxm  # noqa: E402
from src.attacks.moeva2.classifier import Classifier  # noqa: E402
from src.examples.botnet.botnet_augmented_constraints import BotnetAugmentedConstraints  # noqa
from src.examples.botnet.botnet_constraints import BotnetConstraints  # noqa: E402
from src.examples.lcld.lcld_augmented_constraints import LcldAugmentedConstraints  # noqa: E402
from src.examples.lcld.lcld_constraints import LcldConstraints  # noqa: E402
from src.experiments.botnet.features import augment_data  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
RES = os.path.join(os.path.dirname(os.path.dirname(OUT)), "moeva2-ijcai22-replication_amd",
                   "resources")


class NumpyMLP:
    """Stand-in for the Keras SavedModel (TF absent): fp32 Dense relu x3 + softmax."""

    def __init__(self, path):
        m = np.load(path)
        self.W = [m[f"W{i}"] for i in range(4)]
        self.b = [m[f"b{i}"] for i in range(4)]

    def predict_proba(self, x):
        h = np.asarray(x, np.float64).astype(np.float32)
        for i in range(4):
            h = h @ self.W[i] + self.b[i]
            if i < 3:
                h = np.maximum(h, np.float32(0))
        h = h - h.max(axis=1, keepdims=True)
        e = np.exp(h)
        return e / e.sum(axis=1, keepdims=True)


def sk_scaler(path):
    p = np.load(path)
    s = MinMaxScaler()
    s.scale_, s.min_ = p["scale_"], p["min_"]
    s.data_min_, s.data_max_ = p["data_min_"], p["data_max_"]
    s.data_range_ = s.data_max_ - s.data_min_
    s.n_features_in_ = s.scale_.shape[0]
    s.n_samples_seen_ = 2
    return s


def botnet_constraints(cls=BotnetConstraints, feat="features.csv", cons="constraints.csv",
                       imp="important_features_19.npy"):
    c = cls.__new__(cls)  # bypass __init__: it would pickle.load feat_idx.pickle
    c._provision_constraints_min_max(f"./data/botnet/{cons}")
    c._provision_feature_constraints(f"./data/botnet/{feat}")
    c._fit_scaler()
    with open(os.path.join(RES, "data/botnet/feat_idx.json")) as f:
        c.feat_idx = json.load(f)
    c.feat_idx_tf = c.feat_idx
    c.important_features = np.load(f"./data/botnet/{imp}")
    return c


def perturb(rng, c, X, n_per, frac=0.3):
    """Random in-bound perturbations of the mutable features (int-typed rounded)."""
    mm = c.get_mutable_mask().astype(bool)
    ftype = c.get_feature_type()
    out = []
    for x in X:
        xl, xu = c.get_feature_min_max(dynamic_input=x)
        xl = xl.astype(float)
        xu = xu.astype(float)
        for _ in range(n_per):
            y = x.copy()
            sel = mm & (rng.uniform(size=x.shape[0]) < frac)
            lo = xl[sel]
            hi = np.maximum(xu[sel], lo)
            v = rng.uniform(lo, hi)
            isint = np.array([t == "int" for t in ftype[sel]])
            v[isint] = np.round(v[isint])
            y[sel] = v
            out.append(y)
    return np.array(out)


def lcld_states(n):
    return np.load(os.path.join(RES, "data/lcld/x_candidates_synthetic.npy"))[:n]


def save(name, **arrs):
    np.savez_compressed(os.path.join(OUT, name), **arrs)
    print("wrote", name, {k: v.shape for k, v in arrs.items()})


def constraints_fixtures(rng):
    # ---- botnet (botnet_constraints.py:117-173)
    c = botnet_constraints()
    X0 = np.load("./data/botnet/x_candidates_common.npy")
    Xp = perturb(rng, c, X0[:8], 6)
    Xz = Xp[:4].copy()  # force the b == 0 branch of the pkts/bytes ratio (:305)
    fi = c.feat_idx
    for j in range(17):
        Xz[:, fi["pkts_out_sum_s_idx"][j]] = 0.0
    X = np.concatenate([X0[:8], Xp, Xz])
    save("botnet_constraints.npz", x=X, g=c.evaluate(X))
    # ---- botnet augmented (botnet_augmented_constraints.py)
    ca = botnet_constraints(BotnetAugmentedConstraints, "features_augmented_19.csv",
                            "constraints_augmented_19.csv")
    XA0 = np.load("./data/botnet/x_candidates_common_augmented.npy")
    XA = np.concatenate([XA0[:6], perturb(rng, ca, XA0[:4], 4)])
    save("botnet_aug_constraints.npz", x=XA, g=ca.evaluate(XA))
    # ---- lcld (lcld_constraints.py:168-223)
    cl = LcldConstraints("./data/lcld/features.csv", "./data/lcld/constraints.csv")
    L0 = lcld_states(16)
    Lp = perturb(rng, cl, L0[:8], 8, frac=0.4)
    Lz = Lp[:6].copy()
    Lz[:3, 11] = 0.0  # pub_rec == 0 -> masked ratio branch (:210-215)
    Lz[3:, 1] = 48.0  # term neither 36 nor 60
    X = np.concatenate([L0, Lp, Lz])
    save("lcld_constraints.npz", x=X, g=cl.evaluate(X))
    # ---- lcld augmented (lcld_augmented_constraints.py:176-234)
    cla = LcldAugmentedConstraints("./data/lcld/features_augmented.csv",
                                   "./data/lcld/constraints_augmented.csv")
    LA0 = np.load(os.path.join(RES, "data/lcld/x_candidates_synthetic_augmented.npy"))[:12]
    LAp = perturb(rng, cla, LA0[:6], 6, frac=0.4)
    XA = np.concatenate([LA0, LAp])
    save("lcld_aug_constraints.npz", x=XA, g=cla.evaluate(XA),
         augmented=augment_data(LA0[:, :47], cla.important_features))
    return c, cl, cla


def encoder_problem_fixtures(rng, c_bot, c_lcld, c_lcld_aug):
    specs = [
        ("botnet", c_bot, np.load("./data/botnet/x_candidates_common.npy")[:3],
         "models/botnet/nn.npz", "models/botnet/scaler.npz"),
        ("lcld", c_lcld, lcld_states(3), "models/lcld/nn.npz", "models/lcld/scaler.npz"),
        ("lcld_aug", c_lcld_aug,
         np.load(os.path.join(RES, "data/lcld/x_candidates_synthetic_augmented.npy"))[:3],
         "models/lcld/nn_augmented_moeva_best.npz", "models/lcld/scaler_augmented.npz"),
    ]
    for name, c, X, model, scaler in specs:
        clf = Classifier(NumpyMLP(os.path.join(RES, model)))
        mls = sk_scaler(os.path.join(RES, scaler))
        out = {"x_init": X}
        for s, x in enumerate(X):
            enc = fe.get_encoder_from_constraints(c, x)
            xl, xu = enc.get_min_max_genetic()
            types = enc.get_type_mask_genetic()
            g0 = enc.ml_to_genetic(x.reshape(1, -1))[0]
            # random genetic population inside the genetic bounds (ints rounded)
            n = 24
            isreal = np.array([t == "real" for t in types])
            G = rng.uniform(xl, np.maximum(xu, xl), size=(n, xl.shape[0]))
            G[:, ~isreal] = np.round(G[:, ~isreal])
            keep = rng.uniform(size=G.shape) < 0.6  # many genes equal to x_init's
            G = np.where(keep, g0[None, :], G)
            G[0] = g0
            out[f"s{s}_xl"], out[f"s{s}_xu"] = xl, xu
            out[f"s{s}_isreal"] = isreal
            out[f"s{s}_g0"] = g0
            out[f"s{s}_genes"] = G
            out[f"s{s}_x_ml"] = enc.genetic_to_ml(G, x)
            for norm in (2, np.inf):
                prob = dp.DefaultProblem(
                    x_initial_state=x, classifier=clf, minimize_class=1, encoder=enc,
                    constraints=c, scale_objectives=True, save_history="full",
                    ml_scaler=mls, norm=norm)
                res = {}
                prob._evaluate(G, res)
                tag = "l2" if norm == 2 else "linf"
                out[f"s{s}_F_{tag}"] = res["F"]
                out[f"s{s}_hist_{tag}"] = prob.get_history()[0]
        save(f"problem_{name}.npz", **out)


def operator_fixtures(rng):
    # dominance relation: pareto_operation.py:148-164 (copy of pymoo Dominator)
    F = rng.integers(0, 4, size=(40, 3)).astype(float)  # many ties / duplicates
    F = np.concatenate([F, rng.uniform(size=(40, 3))])
    save("dominance.npz", f=F, m=po.calc_domination_matrix(F, F))

    # polynomial mutation: softmax_mutation.py:60-108 with the softmax disabled
    sxm.softmax = lambda x, axis=None: x
    cases = {}
    for k, (n, v) in enumerate([(30, 12), (50, 5)]):
        xl = rng.uniform(-5, 0, v)
        xu = xl + rng.uniform(0.5, 10, v)
        xu[0] = xl[0] + 1.0
        X = rng.uniform(xl, xu, size=(n, v))
        X[:3] = xl  # at-bound parents
        X[3:6] = xu

        class P:
            pass

        prob = P()
        prob.xl, prob.xu, prob.n_var = xl, xu, 2  # prob = 1/n_var = 0.5: many mutations
        np.random.seed(1000 + k)
        do = np.random.random(X.shape) < 0.5
        rand = np.random.random(int(do.sum()))
        np.random.seed(1000 + k)
        Y = sxm.SoftmaxPolynomialMutation(eta=20)._do(prob, X)
        cases.update({f"c{k}_x": X, f"c{k}_xl": xl, f"c{k}_xu": xu, f"c{k}_do": do,
                      f"c{k}_rand": rand, f"c{k}_y": Y})
    save("polynomial_mutation.npz", **cases)

    # two-point crossover: softmax_crossover.py:14-42 with the softmax disabled
    sxc.softmax = lambda x, axis=None: x
    cases = {}
    for k, (nm, nv) in enumerate([(25, 9), (10, 2), (10, 3)]):
        X = rng.uniform(size=(2, nm, nv))
        np.random.seed(2000 + k)
        r = np.row_stack([np.random.permutation(nv - 1) + 1 for _ in range(nm)])[:, :2]
        np.random.seed(2000 + k)
        Y = sxc.SoftmaxPointCrossover(n_points=2)._do(None, X)
        cases.update({f"c{k}_x": X, f"c{k}_cuts": r, f"c{k}_y": Y})
    save("two_point_crossover.npz", **cases)


def objective_calculator_fixture(rng, c_bot):
    X0 = np.load("./data/botnet/x_candidates_common.npy")[:4]
    pops = np.stack([perturb(rng, c_bot, x[None, :], 10, frac=0.05) for x in X0])
    pops[:, 0] = X0  # the unperturbed state: constraints respected
    clf = Classifier(NumpyMLP(os.path.join(RES, "models/botnet/nn.npz")))
    mls = sk_scaler(os.path.join(RES, "models/botnet/scaler.npz"))
    calc = oc.ObjectiveCalculator(clf, c_bot, minimize_class=1,
                                  thresholds={"f1": 0.5, "f2": 4}, min_max_scaler=mls,
                                  ml_scaler=mls, norm=2)
    out = {"x_init": X0, "x_attacks": pops}
    for i in range(4):
        obj = calc._calculate_objective(X0[i], pops[i])
        out[f"obj{i}"] = obj
        out[f"resp{i}"] = calc._objective_respected(obj)
    out["success_rate"] = calc.success_rate_3d(X0, pops)
    save("objective_calculator_botnet.npz", **out)


def main():
    rng = np.random.default_rng(7)
    c_bot, c_lcld, c_lcld_aug = constraints_fixtures(rng)
    encoder_problem_fixtures(rng, c_bot, c_lcld, c_lcld_aug)
    operator_fixtures(rng)
    objective_calculator_fixture(rng, c_bot)


if __name__ == "__main__":
    main()
