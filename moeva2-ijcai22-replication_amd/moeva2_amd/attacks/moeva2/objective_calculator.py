"""Success evaluation of attack results (mirror of src/attacks/moeva2/objective_calculator.py).

Same class, constructor and methods as the reference.  The per-candidate objectives
``[CV, f1, f2]`` of ``_calculate_objective`` (objective_calculator.py:44-84) run on the GPU
through ``mv_objcalc_run``: constraint program (the constraints object's device program),
one-hot consistency (utils.py:43-54), ``ml_scaler`` + classifier (fp32 MFMA), and the
min-max distance, for ALL initial states in one launch chain (``success_rate_3d`` and
``get_successful_attacks`` batch the states instead of looping per state).  The thresholding
and the per-state / per-column means (``_objective_respected``, :86-119) are the same numpy
as the reference.  A constraints object without a device program, or a classifier that is
not a Dense MLP, is evaluated by the user's own plugin (``evaluate`` / ``predict_proba``,
objective_calculator.py:50,64) and the rest is scored on the device (``mv_objcalc_score``);
nothing falls back to the oracle, and without the engine library this raises.
"""
from __future__ import annotations

from typing import List

import numpy as np

from .classifier import Classifier
from .constraints import Constraints
from .feature_encoder import get_encoder_from_constraints
from .utils import _pop_x, get_ohe_masks


class ObjectiveCalculator:
    def __init__(self, classifier: Classifier, constraints: Constraints, minimize_class: int,
                 thresholds: dict, min_max_scaler, norm=np.inf, ml_scaler=None,
                 problem_class=None, n_jobs=1, device=None):
        self._classifier = classifier
        self._constraints = constraints
        self._thresholds = thresholds
        self._ml_scaler = ml_scaler
        self._problem_class = problem_class
        self._minimize_class = minimize_class
        self._encoder = get_encoder_from_constraints(self._constraints)
        self._min_max_scaler = min_max_scaler
        self.norm = norm
        self.n_jobs = n_jobs
        # engine extension: the GPU of the host-array entry points (None: torch's current
        # device); calculate_objectives_device runs on the device its tensors live on
        self.device = device
        self._devs = {}  # device index -> (ObjCalc, constraint engine, Mlp)

    # -- device objects (built on first use)
    def _device(self, device=None):
        """(ObjCalc, constraint engine or None, device classifier or None) on ``device``
        (default: ``self.device``, else torch's current device), built once per device.  A
        Constraints object without a device program, or a classifier that is not a Dense MLP,
        is evaluated through its own ``evaluate`` / ``predict_proba`` on the host (the
        reference accepts any plugin, objective_calculator.py:44-64); the one-hot term, CV
        sum, scaling checks and distance stay on the device (mv_objcalc_score)."""
        import torch

        if device is None:
            device = self.device if self.device is not None else torch.cuda.current_device()
        device = int(device)
        objs = self._devs.get(device)
        if objs is None:
            from ..._native import Mlp, ObjCalc
            from ...problem import has_device_classifier, has_device_program

            masks = get_ohe_masks(self._constraints.get_feature_type())
            D = int(self._constraints.get_feature_type().shape[0])
            mls = self._ml_scaler
            oc = ObjCalc(D, [np.asarray(m, np.int32) for m in masks],
                         np.asarray(self._min_max_scaler.scale_, np.float64),
                         np.asarray(self._min_max_scaler.min_, np.float64),
                         None if mls is None else np.asarray(mls.scale_, np.float64),
                         None if mls is None else np.asarray(mls.min_, np.float64),
                         self.norm, device=device)
            ceng = None
            if (hasattr(self._constraints, "_constraint_engine")
                    and has_device_program(self._constraints)):
                ceng = self._constraints._constraint_engine(device)
            mlp = None
            if has_device_classifier(self._classifier):
                w = self._classifier.dense_weights()
                mlp = Mlp(w.weights, w.biases, device=device)
            objs = self._devs[device] = (oc, ceng, mlp)
        return objs

    def calculate_objectives_3d(self, x_initials, x):
        """Batched ``_calculate_objective``: x_initials (B, D), x (B, n, D) -> (B, n, 3).

        One device pass over every state (engine extension; the per-state method below
        calls it with B = 1)."""
        import torch

        from ...problem import ml_transform

        x_initials = np.ascontiguousarray(np.atleast_2d(x_initials), np.float64)
        x = np.ascontiguousarray(x, np.float64)
        if x.ndim != 3 or x.shape[0] != x_initials.shape[0] or x.shape[2] != x_initials.shape[1]:
            raise ValueError(f"x {x.shape} and x_initials {x_initials.shape} do not match")
        B, n, D = x.shape
        if B * n == 0:
            return np.zeros((B, n, 3))
        oc, ceng, mlp = self._device()
        dev = torch.device("cuda", oc.device)
        st = torch.cuda.current_stream(dev)
        xi = torch.from_numpy(x_initials).to(dev)
        xd = torch.from_numpy(x).to(dev)
        obj = torch.empty((B, n, 3), dtype=torch.float64, device=dev)
        bad = torch.empty((B, n), dtype=torch.int32, device=dev)
        if ceng is not None and mlp is not None:
            oc.run(ceng, mlp, xi, xd, self._minimize_class, obj, bad, stream=st)
        else:
            x_f = x.reshape(B * n, D)
            if ceng is not None:
                G = torch.empty((B * n, ceng.prog.C), dtype=torch.float64, device=dev)
                if ceng.prog.C > 0:
                    ceng.constraints(xd.view(B * n, D), G, stream=st)
            else:  # objective_calculator.py:50: the plugin's own numpy evaluate
                g = np.ascontiguousarray(self._constraints.evaluate(x_f), np.float64)
                G = torch.from_numpy(g.reshape(B * n, -1)).to(dev)
            x_ml = ml_transform(self._ml_scaler, x_f)  # :61-63
            if mlp is not None:
                xm = torch.from_numpy(np.ascontiguousarray(x_ml, np.float64)).to(dev)
                proba = torch.empty((B * n, mlp.n_out), dtype=torch.float64, device=dev)
                mlp.predict(xm, proba, stream=st)
            else:  # :64 Classifier.predict_proba of any model
                p = np.ascontiguousarray(self._classifier.predict_proba(x_ml), np.float64)
                proba = torch.from_numpy(p.reshape(B * n, -1)).to(dev)
            oc.score(xi, xd, G if G.shape[1] > 0 else None, proba, self._minimize_class, obj,
                     bad, stream=st)
        # objective_calculator.py:72-76: the scaled origin and candidates must lie in [0, 1]
        assert not bool(bad.any().item()), "candidate or initial state outside the scaler range"
        return obj.cpu().numpy()

    def calculate_objectives_device(self, x_initials, x):
        """``calculate_objectives_3d`` on device tensors (engine extension, no host copy):
        x_initials (B, D), x (B, n, D) fp64 on the GPU -> obj (B, n, 3) on the GPU.  Needs the
        device constraint program and classifier (host plugins: calculate_objectives_3d)."""
        import torch

        if not (x.is_cuda and x_initials.is_cuda) or x.device != x_initials.device:
            raise ValueError(f"x ({x.device}) and x_initials ({x_initials.device}) must be "
                             "tensors on one GPU")
        oc, ceng, mlp = self._device(x.device.index)
        if ceng is None or mlp is None:
            raise ValueError("calculate_objectives_device needs the device constraint program "
                             "and classifier; use calculate_objectives_3d for host plugins")
        B, n = x.shape[0], x.shape[1]
        obj = torch.empty((B, n, 3), dtype=torch.float64, device=x.device)
        if B * n == 0:
            return obj
        bad = torch.empty((B, n), dtype=torch.int32, device=x.device)
        oc.run(ceng, mlp, x_initials.contiguous(), x.contiguous(), self._minimize_class, obj, bad,
               stream=torch.cuda.current_stream(x.device))
        assert not bool(bad.any().item()), "candidate or initial state outside the scaler range"
        return obj

    def _calculate_objective(self, x_initial, x_f):
        x_f = np.atleast_2d(x_f)
        return self.calculate_objectives_3d(np.asarray(x_initial)[None, :], x_f[None])[0]

    def _objective_respected(self, objective_values):
        constraints_respected = objective_values[:, 0] <= 0
        misclassified = objective_values[:, 1] < self._thresholds["f1"]
        l2_in_ball = objective_values[:, 2] <= self._thresholds["f2"]
        return np.column_stack([
            constraints_respected,
            misclassified,
            l2_in_ball,
            constraints_respected * misclassified,
            constraints_respected * l2_in_ball,
            misclassified * l2_in_ball,
            constraints_respected * misclassified * l2_in_ball,
        ])

    def _objective_array(self, x_initial, x_f):
        return self._objective_respected(self._calculate_objective(x_initial, x_f))

    def success_rate(self, x_initial, x_f):
        return self._objective_array(x_initial, x_f).mean(axis=0)

    def at_least_one(self, x_initial, x_f):
        return np.array(self.success_rate(x_initial, x_f) > 0)

    def _objectives_per_state(self, x_initials, x):
        """[obj (n_i, 3)] per state; regular inputs go to the device in one batch."""
        x_initials = np.asarray(x_initials)
        if isinstance(x, np.ndarray) and x.ndim == 3:
            return list(self.calculate_objectives_3d(x_initials, x))
        return [self._calculate_objective(x_initials[i], e) for i, e in enumerate(x)]

    def success_rate_3d(self, x_initial, x):
        objs = self._objectives_per_state(x_initial, x)
        at_least_one = np.array([self._objective_respected(o).mean(axis=0) > 0 for o in objs])
        return at_least_one.mean(axis=0)

    def success_rate_3d_df(self, x_initial, x):
        import pandas as pd

        success_rates = self.success_rate_3d(x_initial, x)
        columns = ["o{}".format(i + 1) for i in range(success_rates.shape[0])]
        return pd.DataFrame(success_rates.reshape([1, -1]), columns=columns)

    def _pops_ml(self, results):
        initial_states = [result.initial_state for result in results]
        pops_x = [_pop_x(result.pop) for result in results]
        pops_x_f = [self._encoder.genetic_to_ml(pops_x[i], initial_states[i])
                    for i in range(len(results))]
        if len({p.shape for p in pops_x_f}) == 1:
            pops_x_f = np.stack(pops_x_f)
        return initial_states, pops_x_f

    def success_rate_genetic(self, results: List):
        initial_states, pops_x_f = self._pops_ml(results)
        return self.success_rate_3d(initial_states, pops_x_f)

    def get_success(self, x_initial, x_f):
        raise NotImplementedError

    def _select_successful(self, objective_values, x_generated, preferred_metrics, order,
                           max_inputs):
        """objective_calculator.py:152-185 after the objectives are known."""
        metrics_to_index = {"misclassification": 1, "distance": 2}
        objective_respected = self._objective_respected(objective_values)
        sorted_index = np.argsort(objective_values[:, metrics_to_index[preferred_metrics]])
        if order == "desc":
            sorted_index = sorted_index[::-1]
        sorted_index_success = sorted_index[objective_respected[:, -1]]
        if max_inputs > -1:
            sorted_index_success = sorted_index_success[:1]
        return x_generated[sorted_index_success]

    def _get_one_successful(self, x_initial, x_generated, preferred_metrics="misclassification",
                            order="asc", max_inputs=-1):
        objective_values = self._calculate_objective(x_initial, x_generated)
        return self._select_successful(objective_values, x_generated, preferred_metrics, order,
                                       max_inputs)

    def get_successful_attacks(self, x_initials, x_generated,
                               preferred_metrics="misclassification", order="asc",
                               max_inputs=-1, return_index_success=False):
        objs = self._objectives_per_state(x_initials, x_generated)
        successful_attacks = [
            self._select_successful(objs[i], np.asarray(x_generated[i]), preferred_metrics,
                                    order, max_inputs)
            for i in range(len(objs))]
        if return_index_success:
            index_success = np.array([len(e) >= 1 for e in successful_attacks])
        successful_attacks = np.concatenate(successful_attacks, axis=0)
        if return_index_success:
            return successful_attacks, index_success
        return successful_attacks

    def get_successful_attacks_results(self, results: List, preferred_metrics="misclassification",
                                       order="asc", max_inputs=-1):
        initial_states, pops_x_f = self._pops_ml(results)
        return self.get_successful_attacks(initial_states, pops_x_f, preferred_metrics, order,
                                           max_inputs)
