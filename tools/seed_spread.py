"""Development check: the device attack's success rates over several seeds at a fixture's
configuration (spread of o1..o7 from the RNG alone), next to the fixture's oracle value."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_gpu_e2e as T  # noqa: E402
from oracle import moeva_oracle as mo  # noqa: E402
from oracle.problems import Project  # noqa: E402


def main():
    fixture = sys.argv[1]
    seeds = [int(s) for s in sys.argv[2].split(",")]
    d = np.load(os.path.join(T.GOLD, fixture), allow_pickle=False)
    name = str(d["project"])
    B, G = int(d["n_states"]), int(d["n_gen"])
    p = Project(name)
    X = p.x[:B]
    sc, mn = p.ml
    rates = []
    for seed in seeds:
        genes = T._device_attack(name, X, G, int(d["n_pop"]), int(d["n_offsprings"]), seed)
        resp = np.zeros((B, 7), bool)
        for b in range(B):
            x_f = mo.genetic_to_ml(p.lay, genes[b], X[b])
            obj = mo.objectives_calc(X[b], x_f, p.constraints, p.types, sc, mn, p.weights,
                                     p.biases, 1, sc, mn, 2)
            resp[b] = mo.objectives_respected(obj, float(d["thr"]), float(d["eps"])).any(0)
        rates.append(resp.mean(0))
        print(fixture, "seed", seed, np.round(resp.mean(0), 4), flush=True)
    r = np.array(rates)
    print(fixture, "device mean", np.round(r.mean(0), 4), "std", np.round(r.std(0, ddof=1), 4),
          "oracle(seed %d)" % int(d["seed"]), np.round(d["success_rate"], 4), flush=True)


if __name__ == "__main__":
    main()
