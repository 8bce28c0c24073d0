"""Subprocess half of tests/test_gpu_parity.py::test_plan_overflow_paths_bit_exact: one
device attack with the library MOEVA_MI355X_LIB names (the plan-overflow build), the final
genes / F written to an npz.  argv: out.npz name n_states n_gen P O crossover."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root

import numpy as np  # noqa: E402

import conftest  # noqa: E402,F401  (package path)
from test_gpu_parity import _attack  # noqa: E402
from oracle.problems import Project  # noqa: E402


def main():
    out, name, B, G, P, O, cx = sys.argv[1:8]
    X = Project(name).x[:int(B)]
    _, g, F, _, _ = _attack(name, X, int(G), 77, P=int(P), O=int(O), crossover=cx)
    np.savez(out, genes=g.cpu().numpy(), F=F.cpu().numpy())


if __name__ == "__main__":
    main()
