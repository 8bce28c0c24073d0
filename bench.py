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
multi-GPU: states are independent (moeva2.py:194-205).  Every step runs
         Moeva2.generate_sharded's path (moeva2_amd.distributed): rank r attacks its
         contiguous shard of the state set, no collective inside the attack, one
         all_gather of the final populations (genes + objectives) closes the step.
         Default (weak scaling): the workload's state set tiled x N, so every rank attacks
         one full copy.  --shard (strong scaling): the workload's states split over the
         ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W] [--shard]
                    [--crossover two_point|sbx] [--mlp-dtype fp32|bf16]
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
    # the per-GPU share of configs[1] under 8-GPU strong scaling (387 / 8 -> 48 states)
    "rq1.botnet.static.48": dict(project="botnet", features="data/botnet/features.csv",
                                 constraints="data/botnet/constraints.csv",
                                 model="models/botnet/nn.npz", scaler="models/botnet/scaler.npz",
                                 x="data/botnet/x_candidates_common.npy", n_pop=200, n_off=100,
                                 n_gen=1000, norm=2, history="reduced", n_states=48),
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

def global_states(X_all, world, shard):
    """The state set one step attacks over all ranks: the workload's states (strong
    scaling, --shard) or the workload's states tiled x world (weak scaling: rank r's
    shard_bounds slice is copy r)."""
    return X_all if shard else np.concatenate([X_all] * world)


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA (= f32 vector peak)
MFMA_BF16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)


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


_CPU_PROJECT = None


def _cpu_init(project):
    os.environ["OMP_NUM_THREADS"] = "1"
    from threadpoolctl import threadpool_limits

    threadpool_limits(1)  # one core per process: the numpy MLP's BLAS stays single-threaded
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    global _CPU_PROJECT
    from oracle.problems import Project

    _CPU_PROJECT = Project(project)


def _cpu_noop(_):
    return os.getpid()


def _cpu_state(args):
    s, n_pop, n_off, gens, norm, history = args
    from oracle import moeva_oracle as mo

    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs

    p = _CPU_PROJECT
    ref = energy_ref_dirs(3, n_pop, seed=1)
    mo.run_attack(p.problem(p.x[s % p.x.shape[0]], norm=norm), ref, gens, n_pop + 3, n_off,
                  seed=42, save_history=history)
    return n_pop + 3 + (gens - 1) * n_off


def cpu_affinity() -> int:
    """CPUs in this process's affinity mask (os.sched_getaffinity)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_cores():
    """Host cores the baseline uses: the process's affinity mask, capped by the box's CPU
    share (OMP_NUM_THREADS is set to it on the GPU box, whose affinity mask and
    os.cpu_count() cover the whole machine)."""
    n = cpu_affinity()
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return n


def cpu_baseline(w, sample_gens=None, cores=None, states_per_core=2):
    """The oracle's CPU statement of the same loop (eval + survival + variation, numpy):
    one process per host core (like the reference's joblib pool over states, n_jobs =
    cores), a bounded sample of the workload -- states_per_core whole attacks per core at
    the workload's generation budget (about 10 s of CPU work for botnet)."""
    from multiprocessing import get_context

    cores = cores or cpu_cores()
    sample_gens = sample_gens or w["n_gen"]
    P, O = w["n_pop"] + 3, w["n_off"]
    n_states = states_per_core * cores
    jobs = [(s, w["n_pop"], w["n_off"], sample_gens, w["norm"], w["history"])
            for s in range(n_states)]
    with get_context("spawn").Pool(cores, initializer=_cpu_init,
                                   initargs=(w["project"],)) as pool:
        pool.map(_cpu_noop, range(4 * cores))  # every worker started and initialised
        t0 = time.perf_counter()
        n_eval = sum(pool.map(_cpu_state, jobs, chunksize=1))
        dt = time.perf_counter() - t0
    return {"value": n_eval / dt, "unit": "evals/s", "cores": cores, "kind": "port",
            "sample": f"{n_states} {w['project']} states x {sample_gens} generations "
                      f"(P={P}, O={O}) of oracle/moeva_oracle.run_attack (numpy), one "
                      f"process per core; affinity mask {cpu_affinity()} CPUs, box CPU "
                      f"share (OMP_NUM_THREADS) {os.environ.get('OMP_NUM_THREADS', 'unset')}, "
                      f"os.cpu_count()={os.cpu_count()}",
            "affinity_cpus": cpu_affinity(),
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


PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest first: traffic measured on the current kernels wins


def load_traffic(workload):
    """Per-kernel HBM bytes per launch from the committed rocprofv3 PMC passes of `workload`
    (the per-phase kernel chain, the only schedule), newest profile round first; {} when that
    workload was never measured.  A kernel the current code no longer launches simply finds
    no entry (e.g. k_gen/k_cons of round 2 once k_genc replaced them)."""
    for rnd in PROFILE_ROUNDS:
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_traffic_{workload}_chain.json")
        if os.path.exists(path):
            with open(path) as fh:
                return {k: v["traffic_bytes"] for k, v in json.load(fh).items()
                        if isinstance(v, dict) and "traffic_bytes" in v}
    return {}


def run_workload(name, w, args, device, world, rank, steps, warmup, bf16, crossover,
                 profile_gens=None, warm_gens=None):
    """Bind the workload's states, time `steps` whole attacks (after `warmup` untimed ones of
    warm_gens generations, default the full budget), then the per-kernel HIP-event pass (one
    state group, profile_gens generations, default the full budget).  Returns the result
    dict (rank 0; None on the other ranks)."""
    import torch
    import torch.distributed as dist

    from moeva2_amd.attacks.moeva2.moeva2 import history_mode
    from moeva2_amd.attacks.moeva2.ref_dirs import energy_ref_dirs
    from moeva2_amd.distributed import generate_sharded, shard_bounds

    t_load = time.perf_counter()
    eng, c = build_engine(w, device)
    eng.set_attack_mode(args.mode)
    eng.set_crossover(crossover)
    eng.set_mlp_precision("bf16" if bf16 else "fp32")
    X_all = load_states(w)
    # weak scaling (default): the workload's state set tiled x N (rank r owns copy r);
    # strong (--shard): the workload's states split over the ranks.  Either way the step is
    # Moeva2.generate_sharded's path: each rank attacks its contiguous shard
    # (distributed.shard_bounds) and one all_gather returns every state's final population
    # (genes + objectives) to every rank (RCCL over xGMI).
    X_glob = global_states(X_all, world, args.shard)
    B_all = X_all.shape[0]
    states_total = X_glob.shape[0]
    lo, hi = shard_bounds(states_total, world, rank)
    X = X_glob[lo:hi]
    B = X.shape[0]
    if B:
        bounds = [c.get_feature_min_max(dynamic_input=x) for x in X]
        eng.set_states(X, np.array([b[0] for b in bounds]), np.array([b[1] for b in bounds]),
                       1)
    ref = energy_ref_dirs(3, w["n_pop"], seed=1)
    P, O, G = w["n_pop"] + 3, w["n_off"], w["n_gen"]
    hmode = history_mode(w["history"])
    V = eng.prog.V
    genes = torch.empty((B, P, V), dtype=torch.float64, device="cuda")
    F = torch.empty((B, P, 3), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t_load
    seed = 42  # the configs' seed, every state (moeva2.py:163)
    n_gen_run = [G]

    def attack(xs, mcs):  # the rank's shard is bound once, outside the timed region
        assert xs.shape[0] == B
        eng.attack_run(n_gen_run[0], P, O, seed, ref, 0.05, hmode)
        eng.attack_population(genes, F)
        return genes, F

    def empty():
        return genes[:0], F[:0]

    def step():
        return generate_sharded(attack, X_glob, 1, empty=empty)

    # warm-up attacks allocate the attack's buffers (their sizes do not depend on the budget
    # without history, so a short warm-up suffices then)
    n_gen_run[0] = warm_gens if (warm_gens and not hmode) else G
    for i in range(warmup):
        step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] {name}: warmup {i + 1}/{warmup} done")
    n_gen_run[0] = G
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert out[0].shape == (states_total, P, V)
    log(f"[rank {rank}] {name}: timed {steps} steps in {elapsed:.3f}s")

    evals_per_state = P + (G - 1) * O
    total_evals = states_total * evals_per_state * steps
    value = total_evals / elapsed
    ms_per_step = 1000.0 * elapsed / steps

    # ---- roofline of the dominant kernel, measured live with HIP events: the engine hands a
    # start / stop pair to every profiled launch (hipExtLaunchKernelGGL stamps the kernel's own
    # start and end, so the averages agree with rocprofv3's; events recorded around the launch
    # included ~8 us of dispatch gap per k_genc launch).  One state group, so each launch
    # covers all states of the rank like the rocprofv3 pass of the same command.
    if rank != 0:  # only rank 0 reports (it always owns states); the others are done
        return None
    eng.set_profiling(True)
    eng.attack_run(profile_gens or G, P, O, seed, ref, 0.05, hmode)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.set_profiling(False)
    rows = B * O
    Dm = int(eng.prog.mut_feats.shape[0])
    Dm4 = (Dm + 15) // 16 * 16
    # algorithmic work per candidate evaluation: bytes = 2*V*8 (offspring
    # genes written + read once as parents) + 3*8 (F); FLOPs = 2*sum(in*out) over the full
    # Dense chain (dims[0] = D).  The engine executes fewer FLOPs: the immutable features of
    # layer 1 are folded into a per-state bias (executed_flops below).
    eval_bytes = 2 * V * 8 + 3 * 8
    dims_full = list(eng_dims(eng))
    eval_flops = 2 * sum(a * b for a, b in zip(dims_full[:-1], dims_full[1:]))
    # the attack's compact gene layout (mv_get_stored_genes) evaluates its fixed genes'
    # features as immutable ones too: layer 0 runs over the stored genes only
    n_fixed = int((~eng.stored_genes()).sum())
    dims_exec = [Dm - n_fixed] + dims_full[1:]
    exec_flops = 2 * sum(a * b for a, b in zip(dims_exec[:-1], dims_exec[1:]))
    # per-kernel algorithmic bytes per offspring row:
    #   k_gen : parent genes read + child genes written (2*V*8) + fp32 ML row (Dm4*4) + f2 (8)
    #   k_cons: child genes read (V*8) + f3 (8)
    #   k_survive: merged F read (N*3*8) + survivor/free slots + parents (4*(P+O+O)) per state
    # xml_direct (mv_get_mlp_kernel = 1: IDENT problems whose classifier is k_mlp2 reading
    # the genes): k_gen writes no fp32 ML row, k_mlp2 reads the child genes itself
    prog = eng.prog
    xml_direct = kt["mlp_kernel"] in ("k_mlp2(genes)", "k_mlpr(genes)")
    gen_bytes = 2 * V * 8 + (0 if xml_direct else Dm4 * 4) + 8
    cons_bytes = V * 8 + 8
    surv_bytes_state = (P + O) * 3 * 8 + 4 * (P + 2 * O)

    # HBM bytes per launch from the committed rocprofv3 PMC passes of THIS workload and
    # schedule (tools/pmc_traffic.py: (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 correction)
    traffic = {}
    if crossover == "two_point" and not bf16:
        traffic = load_traffic(name)

    def hbm(kname, bytes_launch, ms, key):
        gbs = bytes_launch / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": traffic.get(key), "kernel": kname,
                "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": ms}

    ng = max(kt["generations"], 1)
    gen_ms = kt["gen_ms"] / ng
    cons_ms = kt["cons_ms"] / ng
    mlp_ms = kt["mlp_ms"] / ng
    surv_ms = kt["survive_ms"] / ng
    # achieved / frac on the FLOPs the kernel executes (immutable features folded into
    # the per-state bias); the full-chain algorithmic rate is reported beside it
    mlp_tfs = exec_flops * rows / (mlp_ms * 1e-3) / 1e12
    mlp_tfs_alg = eval_flops * rows / (mlp_ms * 1e-3) / 1e12
    mlp_peak = MFMA_BF16_PEAK_TFS if bf16 else MFMA_F32_PEAK_TFS
    kernels = {
        "k_gen": hbm("k_gen (crossover + mutation + ML row + distance)", gen_bytes * rows,
                     gen_ms, "k_gen"),
        "k_cons": hbm("k_cons (constraint program, f3)", cons_bytes * rows, cons_ms,
                      "k_cons"),
        "k_mlp": {"bound": "mfma", "achieved": mlp_tfs, "peak": mlp_peak,
                  "unit": "TFLOP/s", "frac": mlp_tfs / mlp_peak,
                  "traffic": traffic.get("k_mlp"),
                  "kernel": "%s (%s MFMA Dense chain)" % (kt["mlp_kernel"],
                                                           "bf16" if bf16 else "fp32"),
                  "achieved_algorithmic": mlp_tfs_alg,
                  "algorithmic_flops_per_launch": eval_flops * rows,
                  "executed_flops_per_launch": exec_flops * rows, "avg_launch_ms": mlp_ms},
        "k_survive": hbm("k_survive (R-NSGA-III survival + tournament + variation plan; "
                         "latency-bound)", surv_bytes_state * B, surv_ms, "k_survive"),
    }
    per_gen = {"k_gen": gen_ms, "k_cons": cons_ms, "k_mlp": mlp_ms, "k_survive": surv_ms}
    # LCLD-shaped rows run k_narrow (csrc/narrow.h narrow_ok): variation + decode + f2 +
    # constraint program in ONE launch; IDENT wave-per-row problems (the botnet shape) run
    # k_genc (k_gen and k_cons as two phases of one launch).  Either way the engine's
    # "k_gen" events bracket the one launch and its "k_cons" events an empty step, so the
    # pair is reported as one kernel with the combined algorithmic bytes.
    rk = kt.get("row_kernel", "k_gen+k_cons")
    if rk == "k_narrow":
        hist_b = {"full": 8 * (3 + prog.C), "reduced": 24}.get(w["history"], 0)
        nb = 2 * V * 8 + Dm4 * 4 + 16 + hist_b
        kernels.pop("k_gen")
        kernels.pop("k_cons")
        kernels["k_narrow"] = hbm("k_narrow (crossover + mutation + ML row + distance + "
                                  "constraint program, one lane per row)", nb * rows,
                                  gen_ms + cons_ms, "k_narrow")
        per_gen = {"k_narrow": gen_ms + cons_ms, "k_mlp": mlp_ms, "k_survive": surv_ms}
    elif rk == "k_genc":
        # parents read + child written once (2*V*8) + f2 + f3; phase 2 re-reads the child
        # rows its own workgroup just wrote (L2/MALL hits, not algorithmic HBM bytes)
        nb = gen_bytes + 8
        kernels.pop("k_gen")
        kernels.pop("k_cons")
        kernels["k_genc"] = hbm("k_genc (crossover + mutation + distance, then the "
                                "constraint program over the same rows; one launch)",
                                nb * rows, gen_ms + cons_ms, "k_genc")
        per_gen = {"k_genc": gen_ms + cons_ms, "k_mlp": mlp_ms, "k_survive": surv_ms}
    # the roofline kernel: the longest throughput-bound launch.  k_survive is a latency-bound
    # chain per state (a few KB of HBM traffic; its launch is as long as k_genc's at the
    # headline): it is reported in "kernels" and as "longest_launch", not as the roofline.
    per_gen["longest_launch"] = max(kernels, key=lambda k: kernels[k]["avg_launch_ms"])
    per_gen["dominant"] = max((k for k in kernels if k != "k_survive"),
                              key=lambda k: kernels[k]["avg_launch_ms"])
    dom = per_gen["dominant"]
    if args.shard:
        par = (f"generate_sharded: {B_all} states split over {world} rank(s) ({B} on rank "
               f"{rank}); one all_gather of the final populations")
    else:
        par = (f"generate_sharded: the {B_all} states tiled x{world} = {states_total}, "
               f"{B} per rank; one all_gather of the final populations")
    result = {
        "metric": "candidate fitness evals/sec (whole node) + attack wall-clock per 1k states",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data_note(w, B_all),
        "config": {"workload": name, "states": states_total, "states_per_gpu": B,
                   "pop_size": P, "n_offsprings": O, "n_gen": G, "norm": w["norm"],
                   "history": w["history"], "evals_per_state": evals_per_state,
                   "classifier_dtype": ("bf16 perf mode (bf16 MFMA, fp32 accumulate; not a "
                                        "parity result)" if bf16 else "f32 (MFMA)"),
                   "crossover": crossover,
                   "genes_stored": int(V) - n_fixed,
                   "schedule": "per-phase kernel chain",
                   "parallelism": par},
        "attack_wall_clock_per_1k_states_s": elapsed / steps / states_total * 1000.0,
        "load_s": load_s,
        "roofline": kernels[dom],
        "kernels": kernels,
        "kernels_avg_ms_per_generation": per_gen,
        "kernel_times_generations": ng,
        "algorithmic_per_eval": {"bytes": eval_bytes, "flops": eval_flops,
                                 "executed_flops": exec_flops},
    }
    del eng
    return result


def time_generate(w, device, reps=2):
    """The drop-in API end to end: Moeva2(...).generate(X, 1) on the workload's states, as
    04_moeva.py:71-88 times it (metrics.time) -- host arrays in, the list of per-state result
    objects out: bounds, state binding, the device attack, the final populations, their
    non-dominated members (res.X / res.F) and the history copied to the host, result
    objects.  Model / data loading (Moeva2's classifier, the engine's creation) happens in an
    untimed first call, like the reference's load phase before its clock starts; the first
    call's own wall is reported too (it also allocates the page-locked host buffers)."""
    import torch

    from moeva2_amd.attacks.moeva2.classifier import Classifier, load_model
    from moeva2_amd.attacks.moeva2.moeva2 import Moeva2
    from moeva2_amd.experiments.united.utils import get_constraints_from_str

    c = get_constraints_from_str(w["project"])(os.path.join(RES, w["features"]),
                                               os.path.join(RES, w["constraints"]))
    X = load_states(w)
    m = Moeva2(os.path.join(RES, w["model"]), c, ml_scaler=NpScaler(os.path.join(RES, w["scaler"])),
               norm=w["norm"], n_gen=w["n_gen"], n_pop=w["n_pop"], n_offsprings=w["n_off"],
               save_history=w["history"], seed=42, device=device)
    m._classifier = Classifier(load_model(os.path.join(RES, w["model"])))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = m.generate(X, 1)
    first = time.perf_counter() - t0
    del res
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        res = m.generate(X, 1)
        walls.append(time.perf_counter() - t0)
        n_front = sum(r.X.shape[0] for r in res)
        del res
    wall = min(walls)
    P, O, G = w["n_pop"] + 3, w["n_off"], w["n_gen"]
    evals = X.shape[0] * (P + (G - 1) * O)
    del m
    torch.cuda.empty_cache()
    return {"call": "Moeva2(...).generate(X, 1) -> list of per-state results (host arrays in, "
                    "pop / X / F / history on the host out)",
            "states": int(X.shape[0]), "history": w["history"], "evals_per_s": evals / wall,
            "wall_s": wall, "walls_s": walls, "first_call_wall_s": first,
            "attack_wall_clock_per_1k_states_s": wall / X.shape[0] * 1000.0,
            "front_members": int(n_front)}


# The other BASELINE.json configs, one full-config attack each after the headline (N = 1):
# (key, workload, classifier dtype, warm-up generations, profiled generations)
EXTRA_CONFIGS = [
    ("configs[0]", "rq1.lcld.static", "fp32", None, None),
    ("configs[2]", "rq4.lcld.moeva_augmented", "fp32", None, None),
    ("configs[3]", "synthetic.lcld.scaleout", "fp32", 3, 6),
    ("configs[4]", "synthetic.botnet.wide", "fp32", 3, 10),
    ("configs[4] bf16", "synthetic.botnet.wide", "bf16", 3, 10),
]


def extra_line(key, r):
    """The compact summary of one extra config's result."""
    dom = r["kernels_avg_ms_per_generation"]["dominant"]
    return {"value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
            "steps": r["steps"], "workload": r["config"]["workload"],
            "states": r["config"]["states"], "pop_size": r["config"]["pop_size"],
            "n_offsprings": r["config"]["n_offsprings"], "n_gen": r["config"]["n_gen"],
            "history": r["config"]["history"],
            "classifier_dtype": r["config"]["classifier_dtype"],
            "dominant_kernel": dom, "roofline": r["roofline"],
            "kernels_avg_ms_per_generation": r["kernels_avg_ms_per_generation"],
            "kernel_times_generations": r["kernel_times_generations"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="rq1.botnet.static", choices=sorted(WORKLOADS))
    ap.add_argument("--n-gen", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-generate", action="store_true",
                    help="skip the Moeva2.generate() end-to-end line (N = 1)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs' lines (N = 1 default: one full-config "
                         "attack each of configs[0], [2], [3], [4] after the headline)")
    ap.add_argument("--groups", type=int, default=None,
                    help="state groups (streams) of the timed attack; default: engine's choice. "
                         "--groups 1 makes every launch cover all states, like the roofline "
                         "pass, so rocprofv3 averages compare 1:1 with the bench's event times")
    ap.add_argument("--mode", default="auto", choices=["auto", "chain"],
                    help="attack schedule (the per-phase kernel chain; the whole-attack "
                         "kernel was retired)")
    ap.add_argument("--crossover", default="two_point", choices=["two_point", "sbx"])
    ap.add_argument("--mlp-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="classifier precision: fp32 (parity, default) or the bf16 perf mode "
                         "(a separately labelled line: f1 is not Keras's value)")
    ap.add_argument("--shard", action="store_true",
                    help="strong scaling: split the states over the ranks")
    ap.add_argument("--cpu-gens", type=int, default=None,
                    help="generations per state of the CPU baseline sample (default: the "
                         "workload's budget)")
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
    bf16 = args.mlp_dtype == "bf16"
    result = run_workload(args.workload, w, args, device, world, rank, args.steps, args.warmup,
                          bf16, args.crossover)
    if rank == 0:
        if world == 1 and not args.no_generate and not w["model"].startswith("synthetic:"):
            torch.cuda.empty_cache()
            g = time_generate(w, device)
            g["vs_engine_step"] = g["wall_s"] / (result["ms_per_step"] * 1e-3)
            result["generate"] = g
            log(f"generate(): {g['evals_per_s'] / 1e6:.1f} M evals/s, wall {g['wall_s']:.3f} s "
                f"({g['vs_engine_step']:.2f}x the engine step; first call {g['first_call_wall_s']:.3f} s)")
        if not args.no_cpu_baseline and world == 1 and not w["model"].startswith("synthetic:"):
            result["cpu_baseline"] = cpu_baseline(w, args.cpu_gens)
        # the other BASELINE configs (single GPU, default N = 1 run only): one timed
        # full-config attack each, with its own dominant kernel and roofline
        if world == 1 and not args.no_configs and not args.n_gen and args.workload == \
                "rq1.botnet.static" and args.crossover == "two_point" and not bf16:
            extra = {}
            for key, name, dt, wg, pg in EXTRA_CONFIGS:
                torch.cuda.empty_cache()
                r = run_workload(name, dict(WORKLOADS[name]), args, device, 1, 0, 1, 1,
                                 dt == "bf16", "two_point", profile_gens=pg, warm_gens=wg)
                extra[key] = extra_line(key, r)
                log(f"{key} {name} {dt}: {r['value'] / 1e6:.1f} M evals/s")
            result["configs"] = extra
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
