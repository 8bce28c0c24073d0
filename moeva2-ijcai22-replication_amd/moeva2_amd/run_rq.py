"""Sweep runners for the MoEvA2 experiments (mirror of src/run_rq1.py, run_rq2.py,
run_rq3.py, MoEvA part).

For every seed x project x budget (rq2: x scenario, rq3: x model) one
``python -m moeva2_amd.experiments.united.04_moeva`` process is launched with the same
``-c/-p/-j`` arguments as the reference.  The C-PGD branch of the sweeps is out of scope
(DESIGN.md §7): it is logged and skipped.

    python -m moeva2_amd.run_rq1 -c config/rq1.lcld.yaml
"""
import json
import logging
import subprocess
import sys

from .config_parser.config_parser import get_config

TABULATOR = ">>>"
DRIVER = "moeva2_amd.experiments.united.04_moeva"


def build_commands(config, kind="rq1"):
    """Argument lists of the 04_moeva launches of one sweep (run_rq*.py:19-60)."""
    config_dir = config["config_dir"]
    eps_list_str = json.dumps({"eps_list": config["eps_list"]}, separators=(",", ":"))
    cmds = []
    if "moeva" not in config["attacks"]:
        return cmds
    for seed in config["seeds"]:
        for project in config["projects"]:
            for budget in config["budgets"]:
                base = [sys.executable, "-m", DRIVER, "-c", f"{config_dir}/moeva.yaml",
                        "-c", f"{config_dir}/{project}.yaml", "-p", f"seed={seed}",
                        "-p", f"budget={budget}"]
                if kind == "rq1":
                    cmds.append(base + ["-j", eps_list_str])
                elif kind == "rq2":
                    for scenario in config["scenari"]:
                        cmds.append(base + ["-j", json.dumps(scenario, separators=(",", ":")),
                                            "-j", eps_list_str])
                elif kind == "rq3":
                    for model in config["models"]:
                        model_conf = json.dumps({"paths": {"model": model}},
                                                separators=(",", ":"))
                        cmds.append(base + ["-j", model_conf, "-j", eps_list_str])
                else:
                    raise ValueError(kind)
    return cmds


def run(config, kind="rq1", launcher=subprocess.run):
    logger = logging.getLogger()
    if "pgd" in config.get("attacks", []):
        logger.info(f"{TABULATOR} C-PGD runs are out of scope for this engine: skipped")
    n = 0
    for cmd in build_commands(config, kind):
        logger.info(cmd)
        launcher(cmd)
        n += 1
    logger.info(f"{n} run executed.")
    return n


def main(kind, argv=None):
    logging.basicConfig(level=logging.INFO)
    return run(get_config(argv), kind)
