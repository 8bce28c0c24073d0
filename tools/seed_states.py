"""Development check: per-state device success over many seeds at a seeds fixture's
configuration, saved for comparison with the fixture's per-state oracle results.

    python tools/seed_states.py e2e_botnet_rq1_seeds.npz TAG [n_seeds] [n_gen]

writes gpurun_out/seed_states_TAG.npz: respected (S, B, 7), seeds, n_gen."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_gpu_e2e as T  # noqa: E402


def main():
    fixture, tag = sys.argv[1], sys.argv[2]
    n_seeds = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    d = np.load(os.path.join(T.GOLD, fixture), allow_pickle=False)
    G = int(sys.argv[4]) if len(sys.argv) > 4 else int(d["n_gen"])
    B = int(d["n_states"])
    seeds = list(range(2000, 2000 + n_seeds))
    t0 = time.time()
    _, _, resp, _ = T._device_seed_rates(str(d["project"]), B, G, int(d["n_pop"]),
                                         int(d["n_offsprings"]), float(d["eps"]),
                                         float(d["thr"]), seeds)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"seed_states_{tag}.npz"),
                        respected=resp, seeds=np.asarray(seeds), n_gen=G)
    sr = resp.mean(axis=1)
    print(tag, fixture, f"G={G}", "device mean", np.round(sr.mean(0), 4), "sd",
          np.round(sr.std(0, ddof=1), 4), f"{time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
