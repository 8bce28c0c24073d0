"""pymoo-Problem-compatible fitness (mirror of src/attacks/moeva2/default_problem.py:11-143).

``_evaluate(x, out)`` keeps the pymoo contract (x: (n, n_var) genetic rows,
out["F"]: (n, 3) float64) and runs on the MI355X through ``mv_evaluate``: decode,
encoder MinMax distance, ML scaler, the classifier's GEMM chain and the constraint
program all execute in one HIP kernel.
"""
import numpy as np

from ...hosted import HostPlugins
from ...problem import get_engine
from .classifier import Classifier
from .constraints import Constraints
from .feature_encoder import FeatureEncoder
from .utils import get_scaler_from_norm

NB_OBJECTIVES = 3


class DefaultProblem:
    def __init__(self, x_initial_state: np.ndarray, classifier: Classifier, minimize_class: int,
                 encoder: FeatureEncoder, constraints: Constraints, scale_objectives: True,
                 save_history=False, ml_scaler=None, norm=np.inf, device: int = 0):
        self.x_initial_ml = np.asarray(x_initial_state, np.float64)
        self.classifier = classifier
        self.minimize_class = minimize_class
        self._constraints = constraints
        self.encoder = encoder
        self.scale_objectives = scale_objectives
        self._save_history = save_history
        self.norm = norm
        self.x_initial_f_mm = encoder.normalise(self.x_initial_ml)
        self._f2_scaler = get_scaler_from_norm(norm, self.x_initial_f_mm.shape[0])
        self.xl, self.xu = encoder.get_min_max_genetic()
        self._ml_scaler = ml_scaler
        self._history = []
        self.last_pareto = {"X": np.empty((0, encoder.get_genetic_v_length())),
                            "F": np.empty((0, NB_OBJECTIVES))}
        self.nb_eval = 0
        # pymoo Problem attributes (default_problem.py:55-61)
        self.n_var = encoder.get_genetic_v_length()
        self.n_obj = NB_OBJECTIVES
        self.n_constr = 0
        self._engine = get_engine(constraints, classifier, ml_scaler, norm, scale_objectives,
                                  device)
        self._plugins = HostPlugins(constraints, classifier, ml_scaler)
        xl_f, xu_f = constraints.get_feature_min_max(dynamic_input=self.x_initial_ml)
        self._bind = (self.x_initial_ml[None, :], np.asarray(xl_f, np.float64)[None, :],
                      np.asarray(xu_f, np.float64)[None, :], np.array([minimize_class]))

    def get_initial_state(self):
        return self.x_initial_ml

    def get_history(self):
        return self._history

    def get_nb_objectives(self):
        return NB_OBJECTIVES

    def _evaluate(self, x, out, *args, **kwargs):
        import torch

        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
        if (x - self.xl < 0).sum() > 0 or (x - self.xu > 0).sum() > 0:
            print("Lower than lower bound.")  # default_problem.py:102-106
        eng = self._engine
        if getattr(eng, "bound_by", None) is not self:  # bind once, re-bind only if the
            eng.set_states(*self._bind, owner=self)     # shared engine was rebound since
        genes = torch.from_numpy(x).cuda()[None]
        F = torch.empty((1, x.shape[0], 3), dtype=torch.float64, device=genes.device)
        full = isinstance(self._save_history, str) and "full" in self._save_history
        host_g = full and self._plugins.host_constraints
        G = (torch.empty((1, x.shape[0], eng.prog.C), dtype=torch.float64, device=genes.device)
             if full and not host_g else None)
        eng.evaluate(genes, F, G)
        Gh = [] if host_g else None
        self._plugins.fill(eng, genes, F, [self.minimize_class], Gh)  # host plugins, if any
        if host_g:
            G = torch.as_tensor(Gh[0])
        out["F"] = F[0].cpu().numpy()
        self.nb_eval += x.shape[0]
        if isinstance(self._save_history, str) and "reduced" in self._save_history:
            self._history.append(out["F"])
        elif full:
            self._history.append(np.concatenate((out["F"], G[0].cpu().numpy()), axis=1))

    def evaluate(self, x, return_values_of=("F",)):
        out = {}
        self._evaluate(x, out)
        return out["F"]
