"""MoEvA2 experiment driver (mirror of src/experiments/united/04_moeva.py:27-142).

Same configuration keys, same outputs under ``config["dirs"]["results"]``:

  results_{hash}.npy              legacy pickle of the per-state results (:90-91)
  x_attacks_{attack}_{hash}.npy   (B, P, D) final populations in ML space (:93-105)
  x_history_{attack}_{hash}.npy   (B, n_gen-1, O, 3 | 3+C) when save_history (:107-110)
  metrics_{attack}_{hash}.json    o1..o7 success rates per eps, time, config, hash (:112-139)
  config_{attack}_{hash}.yaml     (:141-142)

The attack runs every initial state in one device batch (Moeva2.generate) and the success
rates are scored on the device in one batch (ObjectiveCalculator.calculate_objectives_3d).
Paths are resolved as given (relative to the CWD, like the reference); when a reference
artefact is not there, the converted copy under the package's ``resources/`` is used
(``.model`` -> ``.npz`` weights, ``.joblib`` -> ``.npz`` scaler; tools/import_reference_data.py).
"""
import json
import os
import pickle
import time
import warnings
from itertools import combinations
from pathlib import Path

import numpy as np

from ...attacks.moeva2.classifier import Classifier, load_model
from ...attacks.moeva2.feature_encoder import get_encoder_from_constraints
from ...attacks.moeva2.moeva2 import Moeva2
from ...attacks.moeva2.objective_calculator import ObjectiveCalculator
from ...attacks.moeva2.utils import results_to_history, results_to_numpy_results
from ...config_parser.config_parser import get_config, get_dict_hash, save_config
from ...examples.utils import augment_data
from .utils import get_constraints_from_str

RESOURCES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))), "resources")


def resolve_path(path):
    """The path as given, else its converted copy under resources/ (same relative path)."""
    if path is None or os.path.exists(path):
        return path
    rel = os.path.normpath(path)
    while rel.startswith(".." + os.sep):
        rel = rel[3:]
    cands = [os.path.join(RESOURCES, rel)]
    stem, ext = os.path.splitext(cands[0])
    if ext in (".model", ".joblib"):
        cands.append(stem + ".npz")
    for c in cands:
        if os.path.exists(c):
            return c
    raise FileNotFoundError(f"{path} (also looked for {', '.join(cands)})")


class NpzScaler:
    """MinMaxScaler parameters converted to .npz (scale_, min_)."""

    def __init__(self, path):
        d = np.load(path, allow_pickle=False)
        self.scale_ = np.asarray(d["scale_"], np.float64)
        self.min_ = np.asarray(d["min_"], np.float64)

    def transform(self, x):
        x = np.array(x, dtype=np.float64, copy=True)
        x *= self.scale_
        x += self.min_
        return x


def load_scaler(path):
    path = resolve_path(path)
    if path.endswith(".npz"):
        return NpzScaler(path)
    from ...io.safe_pickle import load_minmax_scaler

    return load_minmax_scaler(path)  # joblib record read without unpickling


def filter_initial_states(x, start, size):
    """src/utils/__init__.py:15-19."""
    if size > -1:
        return x[start: start + size]
    return x


def _constraints(project_name, features, constraints, important=None):
    cls = get_constraints_from_str(project_name)
    if important:
        return cls(resolve_path(features), resolve_path(constraints), resolve_path(important))
    return cls(resolve_path(features), resolve_path(constraints))


def run(config, verbose=True):
    """04_moeva.py:27-142 for one configuration dict; returns the metrics dict."""
    warnings.simplefilter(action="ignore", category=FutureWarning)
    warnings.simplefilter(action="ignore", category=RuntimeWarning)
    out_dir = config["dirs"]["results"]
    config_hash = get_dict_hash(config)
    mid_fix = f"{config['attack_name']}"
    metrics_path = f"{out_dir}/metrics_{mid_fix}_{config_hash}.json"
    if os.path.exists(metrics_path):
        print(f"Configuration with hash {config_hash} already executed. Skipping")
        return None
    Path(out_dir).mkdir(parents=True, exist_ok=True)
    if verbose:
        print(config)

    paths = config["paths"]
    constraints = _constraints(config["project_name"], paths["features"], paths["constraints"],
                               paths.get("important_features"))
    x_initial_states = np.load(resolve_path(paths["x_candidates"]), allow_pickle=False)
    x_initial_states = filter_initial_states(x_initial_states, config["initial_state_offset"],
                                             config["n_initial_state"])
    scaler = load_scaler(paths["ml_scaler"])
    min_max_scaler = load_scaler(paths.get("min_max_scaler", paths["ml_scaler"]))
    constraints.check_constraints_error(x_initial_states)

    start_time = time.time()
    moeva = Moeva2(resolve_path(paths["model"]), constraints, problem_class=None,
                   l2_ball_size=0.0, norm=config["norm"], n_gen=config["budget"],
                   n_pop=config["n_pop"], n_offsprings=config["n_offsprings"],
                   scale_objectives=True, save_history=config.get("save_history"),
                   seed=config["seed"], n_jobs=config["system"]["n_jobs"], ml_scaler=scaler,
                   verbose=1)
    attacks = moeva.generate(x_initial_states, 1)
    consumed_time = time.time() - start_time

    with open(f"{out_dir}/results_{config_hash}.npy", "wb") as f:  # legacy (Pickler)
        pickle.dump(attacks, f)
    x_attacks = results_to_numpy_results(attacks, get_encoder_from_constraints(constraints))
    if config["reconstruction"]:
        important_features = constraints.important_features
        combi = -sum(1 for _ in combinations(range(len(important_features)), 2))
        x_attacks = augment_data(x_attacks[..., :combi], important_features)
    np.save(f"{out_dir}/x_attacks_{mid_fix}_{config_hash}.npy", x_attacks)
    if config.get("save_history"):
        np.save(f"{out_dir}/x_history_{mid_fix}_{config_hash}.npy", results_to_history(attacks))

    classifier = Classifier(load_model(resolve_path(paths["model"])))
    eval_constraints = constraints
    if config.get("evaluation", False):
        eval_constraints = _constraints(config["evaluation"]["project_name"], paths["features"],
                                        config["evaluation"]["constraints"])
    objective_lists = []
    for eps in config["eps_list"]:
        thresholds = {"f1": config["misclassification_threshold"], "f2": eps}
        calc = ObjectiveCalculator(classifier, eval_constraints, minimize_class=1,
                                   thresholds=thresholds, min_max_scaler=min_max_scaler,
                                   ml_scaler=scaler, norm=config["norm"])
        df = calc.success_rate_3d_df(x_initial_states, x_attacks)
        objective_lists.append(df.to_dict(orient="records")[0])

    metrics = {"objectives_list": objective_lists, "time": consumed_time, "config": config,
               "config_hash": config_hash}
    with open(metrics_path, "w") as f:
        json.dump(metrics, f)
    save_config(f"{out_dir}/config_{mid_fix}_", config)
    return metrics


def main(argv=None):
    t0 = time.time()
    out = run(get_config(argv))
    print(f"func:'run' took: {time.time() - t0:2.4f} sec")
    return out


if __name__ == "__main__":
    main()
