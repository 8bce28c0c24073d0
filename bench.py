"""MoEvA2 attack throughput on MI355X -- the BASELINE.json headline metric.

metric : candidate fitness evals/sec (whole node) = sum over states of
         P + (n_gen - 1) * O evaluations / wall-clock of one attack,
         plus the attack wall-clock per 1k states.
step   : one full MoEvA2 attack (all states, n_gen generations: init + evaluate, then
         (n_gen-1) x {tournament, crossover + mutation + evaluation, R-NSGA-III survival})
         on device-resident inputs, followed by the per-state result gather.
workload (N=1): configs[1] = rq1.botnet.static -- the 387 shipped CTU-13 botnet states,
         n_pop 200 (P = 203), n_offsprings 100, budget 1000 generations, L2, history
         "reduced" (config/moeva.yaml, config/rq1.botnet.static.yaml, config/rq1.botnet.yaml).
multi-GPU: states are independent (moeva2.py:194-205): every rank runs the same per-GPU
         workload on its own seed (weak scaling), no collective inside the attack; one
         all_gather of the per-state best misclassification value closes the step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "moeva2-ijcai22-replication_amd")
sys.path.insert(0, PKG)
RES = os.path.join(PKG, "resources")

WORKLOADS = {
    "rq1.botnet.static": dict(project="botnet", features="data/botnet/features.csv",
                              constraints="data/botnet/constraints.csv",
                              model="models/botnet/nn.npz", scaler="models/botnet/scaler.npz",
                              x="data/botnet/x_candidates_common.npy", n_pop=200, n_off=100,
                              n_gen=1000, norm=2, history="reduced"),
    "rq1.lcld.static": dict(project="lcld", features="data/lcld/features.csv",
                            constraints="data/lcld/constraints.csv", model="models/lcld/nn.npz",
                            scaler="models/lcld/scaler.npz",
                            x="data/lcld/x_candidates_synthetic.npy", n_pop=200, n_off=100,
                            n_gen=100, norm=2, history="full", n_states=64),
    # BASELINE.json configs[2]: LCLD vs the augmented (robust) model, full state set, 1 GPU
    "rq4.lcld.moeva_augmented": dict(project="lcld_augmented",
                                     features="data/lcld/features_augmented.csv",
                                     constraints="data/lcld/constraints_augmented.csv",
                                     model="models/lcld/nn_augmented_moeva_best.npz",
                                     scaler="models/lcld/scaler_augmented.npz",
                                     x="data/lcld/x_candidates_synthetic_augmented.npy",
                                     n_pop=200, n_off=100, n_gen=100, norm=2, history="full"),
    # configs[3]: synthetic scale-out, LCLD-shaped states x Moeva2's default n_pop 640
    "synthetic.lcld.scaleout": dict(project="lcld", features="data/lcld/features.csv",
                                    constraints="data/lcld/constraints.csv",
                                    model="models/lcld/nn.npz", scaler="models/lcld/scaler.npz",
                                    x="data/lcld/x_candidates_synthetic.npy", n_pop=640,
                                    n_off=320, n_gen=100, norm=2, history="False",
                                    n_states=100000),
    # configs[4]: botnet-shaped 756-feature workload, wider 4-layer MLP (random init, seed 7),
    # 10k states x 100 offspring = 1M candidates per generation
    "synthetic.botnet.wide": dict(project="botnet", features="data/botnet/features.csv",
                                  constraints="data/botnet/constraints.csv",
                                  model="synthetic:756-512-512-256-2:7",
                                  scaler="models/botnet/scaler.npz",
                                  x="data/botnet/x_candidates_common.npy", n_pop=200, n_off=100,
                                  n_gen=100, norm=2, history="False", n_states=10000),
}


def synthetic_mlp(spec):
    """'synthetic:d0-d1-...:seed' -> Dense relu..softmax weights ~ N(0, 1/fan_in)."""
    from moeva2_amd.io.tf_bundle import DenseMLP

    _, dims, seed = spec.split(":")
    dims = [int(d) for d in dims.split("-")]
    rng = np.random.default_rng(int(seed))
    W = [(rng.standard_normal((a, b)) / np.sqrt(a)).astype(np.float32)
         for a, b in zip(dims[:-1], dims[1:])]
    bs = [np.zeros(b, np.float32) for b in dims[1:]]
    return DenseMLP(W, bs, ["relu"] * (len(dims) - 2) + ["softmax"])


def load_states(w):
    """The workload's initial states; synthetic scale-outs tile the shipped set."""
    X = np.load(os.path.join(RES, w["x"]), allow_pickle=False)
    n = w.get("n_states")
    if n is not None:
        X = X[:n] if n <= X.shape[0] else np.resize(X, (n, X.shape[1]))
    return np.ascontiguousarray(X)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA (= f32 vector peak)


def eng_dims(eng):
    return eng.dims


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class NpScaler:
    def __init__(self, path):
        d = np.load(path)
        self.scale_, self.min_ = d["scale_"], d["min_"]


def build_engine(w, device):
    from moeva2_amd.attacks.moeva2.classifier import Classifier, load_model
    from moeva2_amd.experiments.united.utils import get_constraints_from_str
    from moeva2_amd.problem import get_engine

    c = get_constraints_from_str(w["project"])(os.path.join(RES, w["features"]),
                                               os.path.join(RES, w["constraints"]))
    if w["model"].startswith("synthetic:"):
        from moeva2_amd.attacks.moeva2.classifier import DenseMLPModel

        clf = Classifier(DenseMLPModel(synthetic_mlp(w["model"])))
    else:
        clf = Classifier(load_model(os.path.join(RES, w["model"])))
    eng = get_engine(c, clf, NpScaler(os.path.join(RES, w["scaler"])), w["norm"], True, device)
    return eng, c


def cpu_baseline(w, sample_states=1, sample_gens=100):
    """Oracle ("port") CPU statement of the same loop, 1 core, bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import moeva_oracle as mo
    from oracle.problems import Project

    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    from threadpoolctl import threadpool_limits

    p = Project(w["project"])
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O = w["n_pop"] + 3, w["n_off"]
    n_eval = 0
    with threadpool_limits(limits=1):  # one core: BLAS in the numpy MLP stays single-threaded
        t0 = time.perf_counter()
        for s in range(sample_states):
            mo.run_attack(p.problem(p.x[s], norm=w["norm"]), ref, sample_gens, P, O, seed=42,
                          save_history=w["history"])
            n_eval += P + (sample_gens - 1) * O
        dt = time.perf_counter() - t0
    return {"value": n_eval / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"{sample_states} {w['project']} state(s) x {sample_gens} generations "
                      f"(P={P}, O={O}) of oracle/moeva_oracle.run_attack, numpy, 1 process",
            "seconds": dt}


def data_note(w, B):
    src = {"botnet": "reference CTU-13 botnet x_candidates_common.npy",
           "lcld": "synthetic valid LCLD states (tools/make_synthetic_lcld.py)",
           "lcld_augmented": "synthetic valid LCLD states + augment_data XOR features"}
    n_file = np.load(os.path.join(RES, w["x"]), mmap_mode="r").shape[0]
    how = f"{B} states" + (f", the {n_file} shipped states tiled" if B > n_file else "")
    clf = ("random-init Dense MLP " + w["model"].split(":")[1]
           if w["model"].startswith("synthetic:") else "shipped classifier weights")
    return f"{src[w['project']]} ({how}) + {clf} and shipped scaler"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="rq1.botnet.static", choices=sorted(WORKLOADS))
    ap.add_argument("--n-gen", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--groups", type=int, default=None,
                    help="state groups (streams) of the timed attack; default: engine's choice. "
                         "--groups 1 makes every launch cover all states, like the roofline "
                         "pass, so rocprofv3 averages compare 1:1 with the bench's event times")
    ap.add_argument("--cpu-gens", type=int, default=300)
    ap.add_argument("--cpu-states", type=int, default=2)
    args = ap.parse_args()

    if args.groups:
        os.environ["MV_GROUPS"] = str(args.groups)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = local if world > 1 else 0
    torch.cuda.set_device(device)
    w = dict(WORKLOADS[args.workload])
    if args.n_gen:
        w["n_gen"] = args.n_gen
    from moeva2_amd.attacks.moeva2.moeva2 import history_mode
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    t_load = time.perf_counter()
    eng, c = build_engine(w, device)
    X = load_states(w)
    B = X.shape[0]
    bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
    eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]), 1)
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O, G = w["n_pop"] + 3, w["n_off"], w["n_gen"]
    hmode = history_mode(w["history"])
    V = eng.prog.V
    genes = torch.empty((B, P, V), dtype=torch.float64, device="cuda")
    F = torch.empty((B, P, 3), dtype=torch.float64, device="cuda")
    gathered = torch.empty((world, B), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t_load
    seed = 42 + rank

    def step():
        eng.attack_run(G, P, O, seed, ref, 0.05, hmode)
        eng.attack_population(genes, F)
        best = F[:, :, 0].min(dim=1).values.contiguous()
        if world > 1:
            dist.all_gather_into_tensor(gathered, best)
        else:
            gathered[0].copy_(best)

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup} done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    log(f"[rank {rank}] timed {args.steps} steps in {elapsed:.3f}s")

    evals_per_state = P + (G - 1) * O
    total_evals = world * B * evals_per_state * args.steps
    value = total_evals / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # ---- roofline of the dominant kernels, measured live with HIP events that the engine
    # records on the bench stream around every k_vary / k_mlp / k_survive launch
    eng.set_profiling(True)
    eng.attack_run(G, P, O, seed, ref, 0.05, hmode)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.set_profiling(False)
    ng = max(kt["generations"], 1)
    gen_ms = kt["gen_ms"] / ng
    cons_ms = kt["cons_ms"] / ng
    mlp_ms = kt["mlp_ms"] / ng
    surv_ms = kt["survive_ms"] / ng
    rows = B * O
    Dm = int(eng.prog.mut_feats.shape[0])
    Dm4 = (Dm + 3) // 4 * 4
    # algorithmic bytes per offspring row (SURVEY.md §8d form):
    #   k_gen : parent genes read + child genes written (2*V*8) + fp32 ML row (Dm4*4) + f2 (8)
    #   k_cons: child genes read (V*8) + f3 (8)
    #   k_survive: merged F read (N*3*8) + survivor/free slots + parents (4*(P+O+O)) per state
    gen_bytes = 2 * V * 8 + Dm4 * 4 + 8
    cons_bytes = V * 8 + 8
    surv_bytes_state = (P + O) * 3 * 8 + 4 * (P + 2 * O)
    dims = [Dm] + list(eng_dims(eng))[1:]
    mlp_flops = 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))

    # HBM bytes per launch from the committed rocprofv3 PMC passes of this workload
    # (tools/pmc_traffic.py: (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH correction)
    traffic = {}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if w["project"] == "botnet" and os.path.exists(tpath):
        with open(tpath) as fh:
            traffic = {k: v["traffic_bytes"] for k, v in json.load(fh).items()}

    def hbm(name, bytes_launch, ms, key):
        gbs = bytes_launch / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": traffic.get(key), "kernel": name,
                "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": ms}

    kernels = {
        "k_gen": hbm("k_gen (crossover + mutation + ML row + distance)", gen_bytes * rows, gen_ms,
                     "k_gen"),
        "k_cons": hbm("k_cons (constraint program, f3)", cons_bytes * rows, cons_ms,
                      "k_cons"),
        "k_mlp": {"bound": "mfma", "achieved": mlp_flops * rows / (mlp_ms * 1e-3) / 1e12,
                  "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                  "frac": mlp_flops * rows / (mlp_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
                  "traffic": traffic.get("k_mlp"), "kernel": "k_mlp (fp32 MFMA Dense chain)",
                  "algorithmic_flops_per_launch": mlp_flops * rows, "avg_launch_ms": mlp_ms},
        "k_survive": hbm("k_survive (R-NSGA-III survival + tournament; latency-bound)",
                         surv_bytes_state * B, surv_ms, "k_survive"),
    }
    dom = max(kernels, key=lambda k: kernels[k]["avg_launch_ms"])

    result = {
        "metric": "candidate fitness evals/sec (whole node) + attack wall-clock per 1k states",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data_note(w, B),
        "config": {"workload": args.workload, "states_per_gpu": B, "pop_size": P,
                   "n_offsprings": O, "n_gen": G, "norm": w["norm"], "history": w["history"],
                   "evals_per_state": evals_per_state, "classifier_dtype": "f32 (MFMA)",
                   "parallelism": f"states x{world} (independent per-rank shards)"},
        "attack_wall_clock_per_1k_states_s": elapsed / args.steps / (world * B) * 1000.0,
        "load_s": load_s,
        "roofline": kernels[dom],
        "kernels": kernels,
        "kernels_avg_ms_per_generation": {"k_gen": gen_ms, "k_cons": cons_ms, "k_mlp": mlp_ms,
                                          "k_survive": surv_ms, "dominant": dom},
    }
    if rank == 0 and not args.no_cpu_baseline and world == 1 and \
            not w["model"].startswith("synthetic:"):
        result["cpu_baseline"] = cpu_baseline(w, args.cpu_states, args.cpu_gens)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
