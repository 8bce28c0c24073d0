"""MoEvA2 attack API (mirror of src/attacks/moeva2/moeva2.py:35-207).

``generate(x, minimize_class)`` keeps the reference signature, argument checks and return
type (one EfficientResult / HistoryResult per initial state), but instead of one
pymoo.minimize per state in a joblib pool (moeva2.py:194-205) it binds ALL states to the
device and runs the whole R-NSGA-III loop on the MI355X (``mv_attack_run``): initial
population + evaluation, then (n_gen - 1) x {tournament, two-point crossover +
polynomial mutation + evaluation, survival}, with no host round trip.
"""
import secrets
import threading
import weakref

import numpy as np

from ...hosted import HostPlugins, hosted_attack
from ...problem import get_engine
from .classifier import Classifier, load_model
from .constraints import Constraints
from .feature_encoder import get_encoder_from_constraints
from .ref_dirs import energy_ref_dirs
from .result_process import EfficientResult, History, HistoryResult, Population

N_OBJ = 3
MU = 0.05  # RNSGA3 default shrink factor (pymoo 0.4.2.2)


def history_mode(save_history) -> int:
    """default_problem.py:137-140 substring tests on the (string) save_history."""
    if not save_history:
        return 0
    s = str(save_history)
    if "reduced" in s:
        return 1
    if "full" in s:
        return 2
    return 0


def _non_dominated(F):
    """Host form of mv_attack_front's mask (pareto_operation.py:35-51's relation), for the
    host-plugin loop, whose populations are not the engine's attack pool."""
    less = (F[:, None, :] < F[None, :, :]).any(-1)
    more = (F[:, None, :] > F[None, :, :]).any(-1)
    dominated = (less & ~more).any(0)
    return ~dominated


def _shard_offset(n_states, group=None) -> int:
    """Global index of this rank's first state under moeva2_amd.distributed's sharding (0
    without a process group): the per-state random streams are keyed by it."""
    import torch.distributed as dist

    from ...distributed import shard_bounds

    if not (dist.is_available() and dist.is_initialized()):
        return 0
    return shard_bounds(n_states, dist.get_world_size(group), dist.get_rank(group))[0]


def _touch(a, n_threads=8):
    """First-touch a fresh array from several threads (numpy's fill releases the GIL), so
    its page faults are taken in parallel: 930 MB in ~9 ms instead of ~46 ms on one core."""
    flat = a.reshape(-1)
    parts = np.array_split(flat, max(1, min(n_threads, flat.size // (1 << 18))))
    if len(parts) == 1:
        flat.fill(0)
        return
    ths = [threading.Thread(target=p.fill, args=(0,)) for p in parts]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def locked_empty(shape, dtype=np.float64):
    """A fresh host array in page-locked memory: numpy allocation, parallel first touch, then
    hipHostRegister, so a device -> host copy into it is one DMA at the PCIe rate (~53 GB/s
    on MI355X vs ~8 GB/s into fresh pageable memory); unregistered when the array is
    collected (numpy runs weakref callbacks before it frees the data).  If registration
    fails the array is returned pageable (the copies are then staged, still correct)."""
    import torch

    a = np.empty(shape, dtype)
    if a.nbytes == 0:
        return a
    _touch(a)
    cudart = torch.cuda.cudart()
    if int(cudart.cudaHostRegister(a.ctypes.data, a.nbytes, 0)) == 0:
        weakref.finalize(a, cudart.cudaHostUnregister, a.ctypes.data)
    return a


def _copy_to(dst, src):
    """Asynchronous device -> host copy of a device tensor into (a prefix of) a host array
    on the current stream (the caller synchronises)."""
    import torch

    if src.numel():
        torch.from_numpy(dst).copy_(src, non_blocking=True)


class Moeva2:
    def __init__(self, classifier_path: str, constraints: Constraints, ml_scaler=None,
                 problem_class=None, l2_ball_size=0.1, norm=np.inf, n_gen=625, n_pop=640,
                 n_offsprings=320, scale_objectives=True, save_history=False, seed=None,
                 n_jobs=-1, verbose=1, device: int = 0, crossover: str = "two_point",
                 sbx_eta: float = 30.0, mlp_dtype: str = "fp32",
                 state_streams: bool = False) -> None:
        self._classifier_path = classifier_path
        self._constraints = constraints
        self._ml_scaler = ml_scaler
        self._problem_class = problem_class
        self._n_gen = n_gen
        self._n_pop = n_pop
        self._n_offsprings = n_offsprings
        self._scale_objectives = scale_objectives
        self._save_history = save_history
        self._seed = seed
        self._n_jobs = n_jobs  # the device batch replaces the joblib pool
        self._verbose = verbose
        self._encoder = get_encoder_from_constraints(self._constraints)
        self.l2_ball_size = l2_ball_size
        self.norm = norm
        self.device = device
        # engine extension: "two_point" = the reference's operator (moeva2.py:90-101);
        # "sbx" = SimulatedBinaryCrossover (north_star; the stale moeva2.py:87 comment's
        # prob 0.9, eta 30)
        if crossover not in ("two_point", "sbx"):
            raise ValueError(f"crossover must be 'two_point' or 'sbx', got {crossover!r}")
        self._crossover = crossover
        self._sbx_eta = sbx_eta
        # engine extension: classifier precision, "fp32" (Keras's arithmetic, the parity
        # mode) or "bf16" (perf mode on bf16 MFMA; f1 no longer matches Keras)
        if mlp_dtype not in ("fp32", "bf16"):
            raise ValueError(f"mlp_dtype must be 'fp32' or 'bf16', got {mlp_dtype!r}")
        self._mlp_dtype = mlp_dtype
        # engine extension: per-state random streams (state b draws from Philox stream b of
        # the global state order) instead of the reference's shared draws -- the same attack
        # per state, independent outcomes across states (mv_set_state_streams)
        self._state_streams = bool(state_streams)
        self._classifier = None
        self._plugins = None
        self._ref = None
        self.last_engine = None

    def _check_input_size(self, x: np.ndarray) -> None:
        if x.shape[1] != self._encoder.mutable_mask.shape[0]:
            raise ValueError(
                f"Mutable mask has shape (n_features,): {self._encoder.mutable_mask.shape[0]}, "
                f"x has shaper (n_sample, n_features): {x.shape}. n_features must be equal.")

    def _get_classifier(self):
        if self._classifier is None:
            self._classifier = Classifier(load_model(self._classifier_path))
        return self._classifier

    def pop_size(self) -> int:
        """RNSGA3: n_ref_points * n_aspiration_dirs (1) + n_obj."""
        return self._n_pop + N_OBJ

    def _engine(self):
        eng = get_engine(self._constraints, self._get_classifier(), self._ml_scaler, self.norm,
                         self._scale_objectives, self.device)
        return eng

    def _bounds(self, x):
        """Per-state feature bounds (moeva2.py:141-142 -> get_encoder_from_constraints(c, x)
        -> constraints.get_feature_min_max(dynamic_input=x)), all states in one batched call
        when the constraints class offers it (the shipped ones), else state by state."""
        batch = getattr(self._constraints, "feature_min_max_batch", None)
        if batch is not None:
            return batch(x)
        bounds = [self._constraints.get_feature_min_max(dynamic_input=xi) for xi in x]
        xl = np.array([b[0] for b in bounds], np.float64).reshape(x.shape)
        xu = np.array([b[1] for b in bounds], np.float64).reshape(x.shape)
        return xl, xu

    def _host_plugins(self, clf):
        if self._plugins is None or self._plugins.classifier is not clf:
            self._plugins = HostPlugins(self._constraints, clf, self._ml_scaler)
        return self._plugins

    def gene_layout(self, x: np.ndarray) -> np.ndarray:
        """The engine's gene layout for a job over the states x (bool [V], True = stored;
        mv_gene_layout).  Pass it to generate(..., gene_layout=) of every batch or shard of
        the job so each state runs in the same layout whichever states share its batch."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        xl, xu = self._bounds(x)
        return self._engine().gene_layout(x, xl, xu)

    def generate(self, x: np.ndarray, minimize_class, return_device=False, first_state=0,
                 gene_layout=None):
        if isinstance(minimize_class, (int, np.integer)):
            minimize_class = np.repeat(minimize_class, x.shape[0])
        minimize_class = np.asarray(minimize_class)
        if x.shape[0] != minimize_class.shape[0]:
            raise ValueError(
                "minimize_class argument must be an integer or an array of shaper (x.shape[0])")
        self._check_input_size(x)
        if len(x.shape) != 2:
            raise ValueError(f"x ({x.shape}) must have 2 dimensions.")
        import torch

        x = np.ascontiguousarray(x, dtype=np.float64)
        B = x.shape[0]
        if B == 0:  # the reference's list comprehension over no states
            return self._empty_device() + (None,) if return_device else []
        clf = self._get_classifier()
        eng = self._engine()
        eng.set_crossover(self._crossover, self._sbx_eta)
        eng.set_mlp_precision(self._mlp_dtype)
        eng.set_state_streams(self._state_streams, first_state)
        xl, xu = self._bounds(x)
        # engine extension: a job split into batches / shards passes the whole job's layout
        # (mv_set_gene_layout applies to the next binding only, so a later binding on this
        # shared engine -- DefaultProblem's -- derives its own)
        eng.set_gene_layout(gene_layout)
        eng.set_states(x, xl, xu, minimize_class)
        P, O = self.pop_size(), self._n_offsprings
        seed = self._seed if self._seed is not None else secrets.randbits(63)
        if self._ref is None:
            self._ref = energy_ref_dirs(N_OBJ, self._n_pop, seed=1)
        ref = self._ref
        hmode = history_mode(self._save_history)
        plugins = self._host_plugins(clf)
        if plugins.any:
            # a plugin the engine cannot compile: host-driven loop around device calls
            g0 = self._encoder.ml_to_genetic(x)
            nonreal = np.asarray([t != "real" for t in self._encoder.get_type_mask_genetic()])
            g0[:, nonreal] = np.rint(g0[:, nonreal])
            genes, F, hist = hosted_attack(eng, plugins, g0, minimize_class, self._n_gen, P, O,
                                           int(seed), ref, MU, hmode)
        else:
            eng.attack_run(self._n_gen, P, O, int(seed), ref, MU, hmode)
            self.last_engine = eng
            if not return_device:
                return self._device_results(eng, x, P, O, hmode)
            V = eng.prog.V
            dev = torch.device("cuda", self.device)
            genes = torch.empty((B, P, V), dtype=torch.float64, device=dev)
            F = torch.empty((B, P, 3), dtype=torch.float64, device=dev)
            eng.attack_population(genes, F)
            hist = None
            if hmode:
                w = 3 if hmode == 1 else 3 + eng.prog.C
                hist = torch.empty((B, P + (self._n_gen - 1) * O, w), dtype=torch.float64,
                                   device=dev)
                eng.attack_history(hist)
        self.last_engine = eng
        if return_device:
            return genes, F, hist
        genes_h = genes.cpu().numpy()
        F_h = F.cpu().numpy()
        hist_h = hist.cpu().numpy() if hist is not None else None
        return [self._result(b, x[b], genes_h[b], F_h[b], hist_h, P, O) for b in range(B)]

    def generate_sharded(self, x: np.ndarray, minimize_class, group=None):
        """Multi-GPU form of generate: this rank attacks its contiguous slice of the states
        (moeva2_amd.distributed.shard_bounds) on its own GPU and one all_gather returns the
        final populations of every state to every rank: genes (B, P, V), F (B, P, 3)."""
        from ...distributed import generate_sharded

        layout = self.gene_layout(x)  # the whole job's: a state's layout is its shard's

        def attack(xs, mcs):
            genes, F, _ = self.generate(xs, mcs, return_device=True,
                                        first_state=_shard_offset(x.shape[0], group),
                                        gene_layout=layout)
            return genes, F

        return generate_sharded(attack, x, minimize_class, group, empty=self._empty_device)

    def generate_scored_sharded(self, x: np.ndarray, minimize_class, objective_calculator,
                                group=None):
        """generate_sharded + the success evaluation of 04_moeva.py:112-131, with only the
        verdict crossing the links: each rank attacks its slice, decodes its final
        populations on its GPU (FeatureEncoder.genetic_to_ml), scores them with
        ``objective_calculator`` (ObjectiveCalculator._calculate_objective on the device) and
        all-gathers per-state o1..o7 flags plus one successful candidate per state
        (moeva2_amd.distributed.success_flags).  Returns, on every rank, flags (B, 7) bool
        (their column means are success_rate_3d's o1..o7) and best (B, D) (NaN rows: no
        o7-successful candidate)."""
        import torch

        from ...distributed import generate_scored_sharded, success_flags

        D = int(x.shape[1])
        dev = torch.device("cuda", self.device)
        layout = self.gene_layout(x)

        def attack(xs, mcs):
            genes, _, _ = self.generate(xs, mcs, return_device=True,
                                        first_state=_shard_offset(x.shape[0], group),
                                        gene_layout=layout)
            xf = torch.empty((genes.shape[0], genes.shape[1], D), dtype=torch.float64,
                             device=dev)
            self.last_engine.decode(genes, xf)
            xi = torch.from_numpy(np.ascontiguousarray(xs, np.float64)).to(dev)
            obj = objective_calculator.calculate_objectives_device(xi, xf)
            return success_flags(obj, xf, objective_calculator._thresholds)

        flags, best = generate_scored_sharded(attack, x, minimize_class, D, group, dev)
        return flags.cpu().numpy().astype(bool), best.cpu().numpy()

    def _empty_device(self):
        """Zero-state (genes, F) device tensors of this attack's shapes."""
        import torch

        dev = torch.device("cuda", self.device)
        P, V = self.pop_size(), self._encoder.get_genetic_v_length()
        return (torch.empty((0, P, V), dtype=torch.float64, device=dev),
                torch.empty((0, P, 3), dtype=torch.float64, device=dev))

    def _device_results(self, eng, x, P, O, hmode):
        """The attack's per-state results straight from the engine: final populations
        (mv_attack_population), their non-dominated members (mv_attack_front: the result's
        X / F, pymoo's final `opt`) and the history, each copied to the host ONCE for all
        states by DMA into page-locked arrays that are prepared while the device still runs
        the attack; then O(B) result objects viewing them (result_process.py)."""
        import torch

        B, V = x.shape[0], eng.prog.V
        dev = torch.device("cuda", self.device)
        stream = torch.cuda.current_stream(dev)
        w = 3 if hmode == 1 else 3 + eng.prog.C
        rows = P + (self._n_gen - 1) * O
        # host side first (CPU work that overlaps the queued attack)
        genes_h = locked_empty((B, P, V))
        F_h = locked_empty((B, P, 3))
        X_h = locked_empty((B * P, V))
        Fx_h = locked_empty((B * P, 3))
        off_h = locked_empty((B + 1,), np.int32)
        hist_h = locked_empty((B, rows, w)) if hmode else None
        genes = torch.empty((B, P, V), dtype=torch.float64, device=dev)
        F = torch.empty((B, P, 3), dtype=torch.float64, device=dev)
        off = torch.empty(B + 1, dtype=torch.int32, device=dev)
        Xp = torch.empty((B * P, V), dtype=torch.float64, device=dev)
        Fp = torch.empty((B * P, 3), dtype=torch.float64, device=dev)
        eng.attack_front(None, off, Xp, Fp, stream=stream)
        eng.attack_population(genes, F, stream=stream)
        with torch.cuda.stream(stream):
            _copy_to(off_h, off)
            _copy_to(genes_h, genes)
            _copy_to(F_h, F)
            if hmode:
                eng.attack_history(torch.from_numpy(hist_h), stream=stream, host=True)
            stream.synchronize()
            n = int(off_h[B])
            _copy_to(X_h[:n], Xp[:n])
            _copy_to(Fx_h[:n], Fp[:n])
            stream.synchronize()
        offs = off_h.tolist()
        out = []
        for b in range(B):
            lo, hi = offs[b], offs[b + 1]
            res = {"pop": Population(genes_h[b], F_h[b]), "initial_state": x[b],
                   "n_gen": self._n_gen, "pop_size": P, "n_offsprings": O, "X": X_h[lo:hi],
                   "F": Fx_h[lo:hi], "pareto": np.empty((0, V))}
            if self._save_history:
                res["history"] = ([] if hist_h is None else
                                  History(hist_h[b], P, O, self._n_gen))
                out.append(HistoryResult(res))
            else:
                out.append(EfficientResult(res))
        return out

    def _result(self, b, x0, genes, F, hist, P, O):
        pop = Population(genes, F)
        nd = _non_dominated(F)
        res = {"pop": pop, "initial_state": x0, "n_gen": self._n_gen, "pop_size": P,
               "n_offsprings": O, "X": genes[nd], "F": F[nd],
               "pareto": np.empty((0, genes.shape[1]))}
        if self._save_history:
            res["history"] = [] if hist is None else History(hist[b], P, O, self._n_gen)
            return HistoryResult(res)
        return EfficientResult(res)
