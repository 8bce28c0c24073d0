"""ctypes binding of libmoeva_mi355x.so (include/moeva_mi355x.h).

This is the only door from Python to the engine.  There is no CPU fallback: if the
library is missing or no GPU is visible, the calls raise.  Device buffers are torch
tensors (PyTorch is used for HBM allocation and streams only).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MOEVA_MI355X_LIB", os.path.join(PKG_ROOT, "lib", "libmoeva_mi355x.so"))

MV_GENE_REAL, MV_GENE_INT, MV_GENE_OHE = 0, 1, 2
OP = dict(DIFF=1, RATIO_SAFE=2, ABS_SUMDIFF=3, LCLD_INSTALL=4, LCLD_TERM=5, ABS_RATIO=6,
          MONTHDIFF=7, RATIO_MASKED=8, XOR_AUG=9)

EXPORTED = [
    "mv_last_error", "mv_device_count", "mv_engine_create", "mv_engine_destroy",
    "mv_set_states", "mv_evaluate", "mv_decode", "mv_constraints", "mv_survive", "mv_select_parents",
    "mv_variation", "mv_attack_run", "mv_attack_population", "mv_attack_front",
    "mv_attack_history",
    "mv_set_profiling", "mv_get_kernel_times", "mv_get_phase_times", "mv_get_row_kernel",
    "mv_get_mlp_kernel", "mv_set_attack_mode",
    "mv_set_crossover", "mv_set_mlp_precision",
    "mv_get_attack_time", "mv_mlp_create", "mv_mlp_destroy",
    "mv_mlp_predict", "mv_objcalc_create", "mv_objcalc_destroy", "mv_objcalc_run",
    "mv_objcalc_score", "mv_det_pow", "mv_debug_checks", "mv_set_state_streams",
    "mv_debug_survival_dump", "mv_get_stored_genes", "mv_gene_layout", "mv_set_gene_layout",
]

_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)
_f32p = C.POINTER(C.c_float)


class ProblemDesc(C.Structure):
    _fields_ = [
        ("D", C.c_int32), ("V", C.c_int32), ("Dm", C.c_int32), ("C", C.c_int32),
        ("n_ohe", C.c_int32), ("gene_kind", _i32p), ("gene_feat", _i32p),
        ("ohe_offsets", _i32p), ("ohe_feats", _i32p), ("mut_feats", _i32p),
        ("ml_scale", _f64p), ("ml_min", _f64p), ("op_code", _i32p), ("op_arg", _i32p),
        ("op_karg", _f64p), ("n_pool", C.c_int32), ("idx_pool", _i32p), ("tol", C.c_double),
        ("norm", C.c_int32), ("scale_objectives", C.c_int32),
    ]


class ModelDesc(C.Structure):
    _fields_ = [("n_layers", C.c_int32), ("dims", _i32p), ("W", C.POINTER(_f32p)),
                ("b", C.POINTER(_f32p))]


class AttackParams(C.Structure):
    _fields_ = [("n_gen", C.c_int32), ("pop_size", C.c_int32), ("n_offsprings", C.c_int32),
                ("seed", C.c_uint64), ("n_ref", C.c_int32), ("ref_points", _f64p),
                ("mu", C.c_double), ("history", C.c_int32)]


class ObjCalcDesc(C.Structure):
    _fields_ = [("D", C.c_int32), ("n_ohe", C.c_int32), ("ohe_offsets", _i32p),
                ("ohe_feats", _i32p), ("mm_scale", _f64p), ("mm_min", _f64p),
                ("ml_scale", _f64p), ("ml_min", _f64p), ("norm", C.c_int32)]


class NativeError(RuntimeError):
    pass


_LIB = None


def lib():
    """Load the engine library (raises if it was not built: no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} not found: build it with `make -C moeva2-ijcai22-replication_amd/csrc`"
                " (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        L.mv_last_error.restype = C.c_char_p
        vp = C.c_void_p
        sig = {
            "mv_device_count": [_i32p],
            "mv_engine_create": [C.c_int32, C.POINTER(ProblemDesc), C.POINTER(ModelDesc),
                                 C.POINTER(vp)],
            "mv_set_states": [vp, C.c_int32, _f64p, _f64p, _f64p, _i32p, vp],
            "mv_evaluate": [vp, C.c_int32, vp, vp, vp, vp],
            "mv_decode": [vp, C.c_int32, vp, vp, vp],
            "mv_constraints": [vp, C.c_int32, vp, vp, vp],
            "mv_survive": [C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32, vp, C.c_double,
                           C.c_uint64, C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
            "mv_select_parents": [C.c_int32, C.c_int32, C.c_int32, C.c_uint64, C.c_int32, vp, vp],
            "mv_variation": [vp, C.c_int32, C.c_int32, C.c_uint64, C.c_int32, vp, vp, vp, vp],
            "mv_attack_run": [vp, C.POINTER(AttackParams), vp],
            "mv_attack_population": [vp, vp, vp, vp],
            "mv_attack_front": [vp, vp, vp, vp, vp, vp],
            "mv_attack_history": [vp, vp, vp],
            "mv_set_profiling": [vp, C.c_int32],
            "mv_get_kernel_times": [vp, _f64p, _f64p, _f64p, _i32p],
            "mv_get_phase_times": [vp, _f64p, _i32p],
            "mv_get_row_kernel": [vp, _i32p],
            "mv_get_mlp_kernel": [vp, _i32p],
            "mv_set_attack_mode": [vp, C.c_int32],
            "mv_set_crossover": [vp, C.c_int32, C.c_double, C.c_double],
            "mv_set_mlp_precision": [vp, C.c_int32],
            "mv_get_attack_time": [vp, _f64p, _i32p],
            "mv_mlp_create": [C.c_int32, C.POINTER(ModelDesc), C.POINTER(vp)],
            "mv_mlp_predict": [vp, C.c_int32, vp, vp, vp],
            "mv_objcalc_create": [C.c_int32, C.POINTER(ObjCalcDesc), C.POINTER(vp)],
            "mv_objcalc_run": [vp, vp, vp, C.c_int32, C.c_int32, vp, vp, C.c_int32, vp, vp, vp],
            "mv_objcalc_score": [vp, C.c_int32, C.c_int32, vp, vp, vp, C.c_int32, vp, C.c_int32,
                                 C.c_int32, vp, vp, vp],
            "mv_det_pow": [C.c_int64, _f64p, _f64p, _f64p],
            "mv_debug_checks": [_i32p, _i32p],
            "mv_set_state_streams": [vp, C.c_int32, C.c_int64],
            "mv_debug_survival_dump": [_f64p],
            "mv_get_stored_genes": [vp, _i32p, _i32p],
            "mv_gene_layout": [vp, C.c_int32, _f64p, _f64p, _f64p, _i32p, _i32p],
            "mv_set_gene_layout": [vp, _i32p, C.c_int32],
        }
        for name, args in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:  # an older build (A/B runs): the call itself will fail
                continue
            fn.argtypes = args
            fn.restype = C.c_int
        L.mv_engine_destroy.argtypes = [vp]
        L.mv_engine_destroy.restype = None
        L.mv_mlp_destroy.argtypes = [vp]
        L.mv_mlp_destroy.restype = None
        L.mv_objcalc_destroy.argtypes = [vp]
        L.mv_objcalc_destroy.restype = None
        _LIB = L
    return _LIB


def check(rc: int):
    if rc != 0:
        raise NativeError(f"libmoeva_mi355x error {rc}: {lib().mv_last_error().decode()}")


def debug_checks():
    """(compiled, record) of the device index checks (csrc/check.h; a -DMV_CHECKS build):
    record = [code, workgroup, thread, value, bound, failures], cleared by the call.
    Synchronises the device."""
    rec = (C.c_int32 * 8)()
    on = C.c_int32(0)
    check(lib().mv_debug_checks(rec, C.byref(on)))
    return bool(on.value), list(rec)[:6]


def debug_survival_dump() -> np.ndarray:
    """Checks builds: the first duplicate-survivor state's inputs (mv_debug_survival_dump)."""
    out = np.zeros(24 + 3 * 1024)
    check(lib().mv_debug_survival_dump(out.ctypes.data_as(_f64p)))
    return out


def det_pow(x, y) -> np.ndarray:
    """The engine's variation pow (csrc/detmath.h), host build: elementwise, broadcast."""
    x, y = np.broadcast_arrays(np.asarray(x, np.float64), np.asarray(y, np.float64))
    x, y = np.ascontiguousarray(x), np.ascontiguousarray(y)
    out = np.empty(x.shape, np.float64)
    f64 = lambda a: a.ctypes.data_as(_f64p)  # noqa: E731
    check(lib().mv_det_pow(x.size, f64(x), f64(y), f64(out)))
    return out


def _ptr(t):
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("expected a contiguous device tensor")
    return C.c_void_p(t.data_ptr())


def _stream(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _arr(a, dtype):
    a = np.ascontiguousarray(a, dtype=dtype)
    return a


def norm_code(norm) -> int:
    """2 for the L2 distance, 0 for L-inf; anything else is rejected like the reference
    DefaultProblem._obj_distance (default_problem.py:80-88 raises NotImplementedError)."""
    if isinstance(norm, str):
        norm = norm.strip().lower()
        if norm in ("2", "l2"):
            return 2
        if norm in ("inf", "np.inf", "linf"):
            return 0
    elif norm == 2:
        return 2
    elif norm == np.inf:
        return 0
    raise ValueError(f"norm {norm!r} is not supported (2 or np.inf)")


@dataclass
class DeviceProgram:
    """Host description of one problem: genetic layout + constraint program."""

    D: int
    gene_kind: np.ndarray  # (V,) int32
    gene_feat: np.ndarray  # (V,)
    ohe_offsets: np.ndarray  # (n_ohe+1,)
    ohe_feats: np.ndarray
    mut_feats: np.ndarray  # (Dm,) ascending
    op_code: np.ndarray  # (C,)
    op_arg: np.ndarray  # (C,4)
    op_karg: np.ndarray  # (C,2)
    idx_pool: np.ndarray
    tol: float = 1e-3

    @property
    def V(self):
        return int(self.gene_kind.shape[0])

    @property
    def C(self):
        return int(self.op_code.shape[0])


class Engine:
    """One engine per (device, problem, classifier)."""

    def __init__(self, prog: DeviceProgram, weights: Optional[Sequence[np.ndarray]],
                 biases: Optional[Sequence[np.ndarray]], ml_scale=None, ml_min=None, norm=2,
                 scale_objectives=True, device: int = 0):
        L = lib()
        self.prog = prog
        self.device = device
        keep = []

        def P(a, dt, ct):
            a = _arr(a, dt)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(ct))

        pd = ProblemDesc()
        pd.D = prog.D
        pd.V = prog.V
        pd.Dm = int(prog.mut_feats.shape[0])
        pd.C = prog.C
        pd.n_ohe = int(prog.ohe_offsets.shape[0]) - 1
        pd.gene_kind = P(prog.gene_kind, np.int32, C.c_int32)
        pd.gene_feat = P(prog.gene_feat, np.int32, C.c_int32)
        pd.ohe_offsets = P(prog.ohe_offsets, np.int32, C.c_int32)
        pd.ohe_feats = P(prog.ohe_feats if prog.ohe_feats.size else np.zeros(1), np.int32,
                         C.c_int32)
        pd.mut_feats = P(prog.mut_feats, np.int32, C.c_int32)
        pd.ml_scale = P(ml_scale, np.float64, C.c_double) if ml_scale is not None else None
        pd.ml_min = P(ml_min, np.float64, C.c_double) if ml_min is not None else None
        pd.op_code = P(prog.op_code, np.int32, C.c_int32)
        pd.op_arg = P(prog.op_arg, np.int32, C.c_int32)
        pd.op_karg = P(prog.op_karg, np.float64, C.c_double)
        pd.n_pool = int(prog.idx_pool.shape[0])
        pd.idx_pool = P(prog.idx_pool if prog.idx_pool.size else np.zeros(1), np.int32, C.c_int32)
        pd.tol = prog.tol
        pd.norm = norm_code(norm)
        pd.scale_objectives = int(bool(scale_objectives))
        md = ModelDesc()
        if weights is not None:
            n = len(weights)
            dims = [int(weights[0].shape[0])] + [int(w.shape[1]) for w in weights]
            md.n_layers = n
            md.dims = P(np.array(dims), np.int32, C.c_int32)
            Ws = (_f32p * n)(*[P(w, np.float32, C.c_float) for w in weights])
            bs = (_f32p * n)(*[P(b, np.float32, C.c_float) for b in biases])
            keep += [Ws, bs]
            md.W = Ws
            md.b = bs
        self._h = C.c_void_p()
        check(L.mv_engine_create(device, C.byref(pd), C.byref(md) if weights is not None else None,
                                 C.byref(self._h)))
        self.B = 0
        self.dims = dims if weights is not None else []
        self.n_out = dims[-1] if weights is not None else 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _LIB is not None:
            _LIB.mv_engine_destroy(h)
            self._h = None

    # -- per-state constants
    def set_states(self, x_init, xl, xu, minimize_class, stream=None, owner=None):
        """Bind B initial states (mv_set_states).  ``owner`` tags the binding so a caller
        that evaluates repeatedly on the same states (DefaultProblem) binds only once."""
        self.bound_by = None
        x_init = _arr(x_init, np.float64)
        xl = _arr(xl, np.float64)
        xu = _arr(xu, np.float64)
        mc = _arr(np.broadcast_to(np.asarray(minimize_class), (x_init.shape[0],)), np.int32)
        check(lib().mv_set_states(self._h, x_init.shape[0],
                                  x_init.ctypes.data_as(_f64p), xl.ctypes.data_as(_f64p),
                                  xu.ctypes.data_as(_f64p), mc.ctypes.data_as(_i32p),
                                  _stream(stream)))
        self.B = x_init.shape[0]
        self.bound_by = owner  # only once the engine holds these states

    def evaluate(self, genes, F, G=None, stream=None):
        """genes (B, n, V) fp64 device tensor -> F (B, n, 3) [, G (B, n, C)]."""
        check(lib().mv_evaluate(self._h, genes.shape[1], _ptr(genes), _ptr(F), _ptr(G),
                                _stream(stream)))

    def decode(self, genes, x, stream=None):
        """genes (B, n, V) -> ML-space rows x (B, n, D) (FeatureEncoder.genetic_to_ml)."""
        check(lib().mv_decode(self._h, genes.shape[1], _ptr(genes), _ptr(x), _stream(stream)))

    def constraints(self, x, G, stream=None):
        """x (n, D) fp64 device tensor -> G (n, C) (the numpy-path Constraints.evaluate)."""
        check(lib().mv_constraints(self._h, x.shape[0], _ptr(x), _ptr(G), _stream(stream)))

    def variation(self, P, O, seed, gen, pop, parents, off, stream=None):
        check(lib().mv_variation(self._h, P, O, seed, gen, _ptr(pop), _ptr(parents), _ptr(off),
                                 _stream(stream)))

    def attack_run(self, n_gen, pop_size, n_offsprings, seed, ref_points, mu=0.05, history=0,
                   stream=None):
        ref = _arr(ref_points, np.float64)
        self._ref_keep = ref
        prm = AttackParams(n_gen, pop_size, n_offsprings, seed, ref.shape[0],
                           ref.ctypes.data_as(_f64p), mu, history)
        check(lib().mv_attack_run(self._h, C.byref(prm), _stream(stream)))

    def attack_population(self, genes=None, F=None, stream=None):
        check(lib().mv_attack_population(self._h, _ptr(genes), _ptr(F), _stream(stream)))

    def attack_front(self, front=None, offsets=None, X=None, Fx=None, stream=None):
        """The final population's non-dominated members (mv_attack_front): front (B, P)
        uint8, offsets (B + 1,) int32 and the members' genes X (B * P, V) / objectives
        Fx (B * P, 3) packed by state in population order (first offsets[B] rows)."""
        check(lib().mv_attack_front(self._h, _ptr(front), _ptr(offsets), _ptr(X), _ptr(Fx),
                                    _stream(stream)))

    def attack_history(self, hist, stream=None, host=False):
        """History rows (B, P + (n_gen - 1) O, 3 | 3 + C) into a device tensor, or with
        host=True a contiguous host tensor -- page-locked (pinned / hipHostRegister'ed) for a
        direct DMA; mv_attack_history copies with hipMemcpyDefault."""
        if host:
            if hist.is_cuda or not hist.is_contiguous():
                raise ValueError("attack_history(host=True): a contiguous host tensor")
            p = C.c_void_p(hist.data_ptr())
        else:
            p = _ptr(hist)
        check(lib().mv_attack_history(self._h, p, _stream(stream)))

    def set_profiling(self, on: bool):
        check(lib().mv_set_profiling(self._h, int(on)))

    def set_crossover(self, kind: str = "two_point", eta: float = 30.0, prob: float = 0.9):
        """"two_point" (the reference's operator) or "sbx" (SimulatedBinaryCrossover)."""
        check(lib().mv_set_crossover(self._h, {"two_point": 0, "sbx": 1}[kind], float(eta),
                                     float(prob)))

    def set_state_streams(self, enabled: bool, first_state: int = 0):
        """Per-state random streams (engine option, off = the reference's shared draws):
        state b draws from Philox stream first_state + b, its GLOBAL index."""
        check(lib().mv_set_state_streams(self._h, 1 if enabled else 0, int(first_state)))
        self.state_streams = (bool(enabled), int(first_state))

    def stored_genes(self) -> np.ndarray:
        """The attack's gene layout for the bound states (mv_get_stored_genes): bool [V],
        False for a gene no attack on these states can change (integer, xl == xu == its
        initial value in every state), which the attack does not store or sum."""
        st = np.zeros(self.prog.V, np.int32)
        n = C.c_int32(0)
        check(lib().mv_get_stored_genes(self._h, st.ctypes.data_as(_i32p), C.byref(n)))
        return st.astype(bool)

    def gene_layout(self, x_init, xl, xu) -> np.ndarray:
        """The layout mv_set_states would derive for these states (mv_gene_layout; host
        computation): bool [V], True = stored."""
        x_init, xl, xu = (_arr(a, np.float64) for a in (x_init, xl, xu))
        st = np.zeros(self.prog.V, np.int32)
        n = C.c_int32(0)
        check(lib().mv_gene_layout(self._h, x_init.shape[0], x_init.ctypes.data_as(_f64p),
                                   xl.ctypes.data_as(_f64p), xu.ctypes.data_as(_f64p),
                                   st.ctypes.data_as(_i32p), C.byref(n)))
        return st.astype(bool)

    def set_gene_layout(self, stored=None):
        """Fix the layout of the next set_states calls (mv_set_gene_layout): bool [V] as
        gene_layout returned it for the whole job, or None to derive it per bound batch."""
        if stored is None:
            check(lib().mv_set_gene_layout(self._h, None, 0))
            return
        st = np.ascontiguousarray(np.asarray(stored, bool), np.int32)
        check(lib().mv_set_gene_layout(self._h, st.ctypes.data_as(_i32p), int(st.shape[0])))

    def set_mlp_precision(self, dtype: str = "fp32"):
        """Classifier precision of the fitness path: "fp32" (parity default) or "bf16" (perf
        mode: bf16 weights/activations on bf16 MFMA, fp32 accumulation)."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(f"mlp dtype {dtype!r}: 'fp32' or 'bf16'")
        check(lib().mv_set_mlp_precision(self._h, 1 if dtype == "bf16" else 0))
        self.mlp_dtype = dtype

    def set_attack_mode(self, mode: str):
        """"chain"/"auto": the per-phase kernel chain (k_gen, k_cons, k_mlp2, k_survive per
        generation), the engine's only schedule.  The whole-attack kernel ("whole") was
        retired (measured slower)."""
        if mode not in ("auto", "chain"):
            raise ValueError(f"attack mode {mode!r}: 'auto' or 'chain' (the whole-attack "
                             "kernel was retired)")
        check(lib().mv_set_attack_mode(self._h, {"auto": 0, "chain": 1}[mode]))

    def kernel_times(self):
        """Summed device ms of k_vary / k_mlp / k_survive over the last profiled attack."""
        tv, tm, ts = C.c_double(), C.c_double(), C.c_double()
        n = C.c_int32()
        check(lib().mv_get_kernel_times(self._h, C.byref(tv), C.byref(tm), C.byref(ts),
                                        C.byref(n)))
        ph = (C.c_double * 4)()
        check(lib().mv_get_phase_times(self._h, ph, C.byref(n)))
        rk = C.c_int32()
        check(lib().mv_get_row_kernel(self._h, C.byref(rk)))
        mk = C.c_int32()
        check(lib().mv_get_mlp_kernel(self._h, C.byref(mk)))
        return {"vary_ms": tv.value, "mlp_ms": tm.value, "survive_ms": ts.value,
                "gen_ms": ph[0], "cons_ms": ph[1], "generations": n.value,
                "row_kernel": ("k_gen+k_cons", "k_narrow", "k_genc")[rk.value],
                "mlp_kernel": {-1: None, 0: "k_mlp", 1: "k_mlp2(genes)", 2: "k_mlp2",
                               4: "k_mlpw", 5: "k_mlpw32", 6: "k_mlpr(genes)", 7: "k_mlpr"}[mk.value]}


def survive(F, ref_points, n_survive, mu, seed, gen, ideal, worst, extreme, has_extreme,
            survivors, rank=None, order=None, n_ranked=None, niche=None, dist=None, nadir=None,
            stream=None):
    """Batched R-NSGA-III survival on device tensors (see mv_survive)."""
    B, N, _ = F.shape
    check(lib().mv_survive(B, N, n_survive, _ptr(F), ref_points.shape[0], _ptr(ref_points), mu,
                           seed, gen, _ptr(ideal), _ptr(worst), _ptr(extreme), _ptr(has_extreme),
                           _ptr(survivors), _ptr(rank), _ptr(order), _ptr(n_ranked), _ptr(niche),
                           _ptr(dist), _ptr(nadir), _stream(stream)))


def select_parents(B, P, O, seed, gen, parents, stream=None):
    check(lib().mv_select_parents(B, P, O, seed, gen, _ptr(parents), _stream(stream)))


def device_count() -> int:
    n = C.c_int32()
    check(lib().mv_device_count(C.byref(n)))
    return n.value


def _model_desc(weights, biases, keep):
    n = len(weights)
    dims = np.array([int(weights[0].shape[0])] + [int(w.shape[1]) for w in weights], np.int32)
    Wc = [np.ascontiguousarray(w, np.float32) for w in weights]
    bc = [np.ascontiguousarray(b, np.float32) for b in biases]
    Ws = (_f32p * n)(*[w.ctypes.data_as(_f32p) for w in Wc])
    bs = (_f32p * n)(*[b.ctypes.data_as(_f32p) for b in bc])
    keep += [dims, Wc, bc, Ws, bs]
    md = ModelDesc()
    md.n_layers = n
    md.dims = dims.ctypes.data_as(_i32p)
    md.W = Ws
    md.b = bs
    return md


class Mlp:
    """Device classifier for Classifier.predict_proba (mv_mlp_*)."""

    def __init__(self, weights, biases, device=0):
        keep = []
        md = _model_desc(weights, biases, keep)
        self._h = C.c_void_p()
        check(lib().mv_mlp_create(device, C.byref(md), C.byref(self._h)))
        self.n_out = int(weights[-1].shape[1])
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _LIB is not None:
            _LIB.mv_mlp_destroy(h)
            self._h = None

    def predict(self, x, proba, stream=None):
        check(lib().mv_mlp_predict(self._h, x.shape[0], _ptr(x), _ptr(proba), _stream(stream)))


class ObjCalc:
    """Device ObjectiveCalculator._calculate_objective (mv_objcalc_*): one per (type mask,
    min_max_scaler, ml_scaler, norm)."""

    def __init__(self, D, ohe_groups, mm_scale, mm_min, ml_scale=None, ml_min=None, norm=2,
                 device=0):
        keep = []

        def P(a, dt, ct):
            a = np.ascontiguousarray(a, dt)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(ct))

        offs = np.zeros(len(ohe_groups) + 1, np.int32)
        for g, m in enumerate(ohe_groups):
            offs[g + 1] = offs[g] + len(m)
        feats = (np.concatenate([np.asarray(m, np.int32) for m in ohe_groups])
                 if ohe_groups else np.zeros(1, np.int32))
        d = ObjCalcDesc()
        d.D = int(D)
        d.n_ohe = len(ohe_groups)
        d.ohe_offsets = P(offs, np.int32, C.c_int32)
        d.ohe_feats = P(feats, np.int32, C.c_int32)
        d.mm_scale = P(mm_scale, np.float64, C.c_double)
        d.mm_min = P(mm_min, np.float64, C.c_double)
        if ml_scale is not None:
            d.ml_scale = P(ml_scale, np.float64, C.c_double)
            d.ml_min = P(ml_min, np.float64, C.c_double)
        d.norm = norm_code(norm)
        self._h = C.c_void_p()
        check(lib().mv_objcalc_create(device, C.byref(d), C.byref(self._h)))
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _LIB is not None:
            _LIB.mv_objcalc_destroy(h)
            self._h = None

    def run(self, engine: "Engine", mlp: "Mlp", x_init, x, minimize_class, obj, range_bad,
            stream=None):
        """x_init (B, D), x (B, n, D) device tensors -> obj (B, n, 3), range_bad (B, n)."""
        B, n = int(x.shape[0]), int(x.shape[1])
        check(lib().mv_objcalc_run(self._h, engine._h, mlp._h, B, n, _ptr(x_init), _ptr(x),
                                   int(minimize_class), _ptr(obj), _ptr(range_bad),
                                   _stream(stream)))

    def score(self, x_init, x, G, proba, minimize_class, obj, range_bad, stream=None):
        """Scoring with a caller-supplied constraint matrix G (B*n, C) (None: C = 0) and
        class probabilities proba (B*n, n_out), all device tensors (mv_objcalc_score)."""
        B, n = int(x.shape[0]), int(x.shape[1])
        C_ = 0 if G is None else int(G.shape[-1])
        check(lib().mv_objcalc_score(self._h, B, n, _ptr(x_init), _ptr(x), _ptr(G), C_,
                                     _ptr(proba), int(proba.shape[-1]), int(minimize_class),
                                     _ptr(obj), _ptr(range_bad), _stream(stream)))


_MLPS = {}


def predict_proba(mlp, x):
    """Host convenience: numpy rows (already ML-scaled) -> probabilities, on the GPU."""
    import torch

    m = _MLPS.get(id(mlp))
    if m is None:
        m = _MLPS[id(mlp)] = (Mlp(mlp.weights, mlp.biases), mlp)
    m = m[0]
    xd = torch.from_numpy(np.ascontiguousarray(np.atleast_2d(x), np.float64)).cuda(m.device)
    out = torch.empty((xd.shape[0], m.n_out), dtype=torch.float64, device=xd.device)
    m.predict(xd, out)
    return out.cpu().numpy()
