"""Dump the device attack's final populations at an e2e fixture's configuration
(development tool): python tools/e2e_dump.py e2e_lcld_rq1_g100.npz out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "moeva2-ijcai22-replication_amd"))
from test_gpu_e2e import GOLD, _device_attack  # noqa: E402
from oracle.problems import Project  # noqa: E402

d = np.load(os.path.join(GOLD, sys.argv[1]), allow_pickle=False)
name = str(d["project"])
B, G = int(d["n_states"]), int(d["n_gen"])
X = Project(name).x[:B]
genes = _device_attack(name, X, G, int(d["n_pop"]), int(d["n_offsprings"]), int(d["seed"]))
np.savez_compressed(sys.argv[2], genes=genes)
