"""Experiment driver / sweep plumbing on CPU (no GPU calls): config parsing and hashing
(src/config_parser/config_parser.py) and path resolution.  The sweep runners
(src/run_rq*.py) are orchestration and out of scope."""
import hashlib
import json
import os

import numpy as np

from conftest import PKG

CFG = os.path.join(PKG, "config")


def test_config_merge_and_value_parsing():
    from moeva2_amd.config_parser.config_parser import get_config, value_parser

    assert value_parser("42") == 42 and isinstance(value_parser("42"), int)
    assert value_parser("0.2") == 0.2 and value_parser("1.5e-3") == 1.5e-3
    # YAML 1.1 (the reference's yaml.safe_load) reads "1e-3" as a string: kept as is
    assert value_parser("1e-3") == "1e-3"
    assert value_parser("flip+sat") == "flip+sat" and value_parser("-5") == -5
    c = get_config(["-c", f"{CFG}/moeva.yaml", "-c", f"{CFG}/rq1.lcld.static.yaml",
                    "-p", "seed=42", "-p", "budget=100", "-p", "system.n_jobs=3",
                    "-j", '{"eps_list":[0.2]}', "-j", '{"paths":{"model":"m.model"}}'])
    assert c["attack_name"] == "moeva" and c["n_pop"] == 200 and c["seed"] == 42
    assert c["budget"] == 100 and c["eps_list"] == [0.2]
    # deep merge replaces leaves only
    assert c["system"] == {"n_jobs": 3, "verbose": 1}
    assert c["paths"]["model"] == "m.model" and c["paths"]["features"].endswith("features.csv")


def test_config_source_order_and_errors(tmp_path):
    """-c files first, then -j, then -p, whatever the command-line order; leaves replace."""
    from moeva2_amd.config_parser.config_parser import get_config

    f = tmp_path / "a.json"
    f.write_text(json.dumps({"x": {"y": 1, "z": [1, 2]}, "n": "file"}))
    c = get_config(["-p", "n=7", "-j", '{"n": "inline", "x": {"z": [9]}}', "-c", str(f)])
    assert c == {"x": {"y": 1, "z": [9]}, "n": 7}
    assert get_config(["-p=x.y=2.5"]) == {"x": {"y": 2.5}}
    for bad in (["-q", "1"], ["-c"]):
        try:
            get_config(bad)
            raise AssertionError("expected SystemExit")
        except SystemExit:
            pass


def test_config_hash_is_md5_of_sorted_json():
    from moeva2_amd.config_parser.config_parser import get_config_hash, get_dict_hash

    d = {"b": 1, "a": {"y": [1, 2], "x": "s"}}
    assert get_dict_hash(d) == hashlib.md5(
        json.dumps(d, sort_keys=True).encode("utf-8")).hexdigest()
    assert get_config_hash(argv=["-j", json.dumps(d)]) == get_dict_hash(d)


def test_resolve_path_falls_back_to_converted_resources(tmp_path):
    from moeva2_amd.experiments.united.moeva_run import load_scaler, resolve_path

    p = resolve_path("./models/botnet/nn.model")
    assert p.endswith(os.path.join("models", "botnet", "nn.npz")) and os.path.exists(p)
    s = load_scaler("./models/lcld/scaler.joblib")
    assert s.scale_.shape == (47,)
    f = tmp_path / "x.npy"
    np.save(f, np.zeros(3))
    assert resolve_path(str(f)) == str(f)
    try:
        resolve_path("./nope/missing.npy")
        raise AssertionError("expected FileNotFoundError")
    except FileNotFoundError:
        pass
