"""Constraints plugin interface (mirror of src/attacks/moeva2/constraints.py:8-77).

Same abstract surface as the reference; each concrete class additionally describes its
numpy path as a *device constraint program* (one op per constraint column, see
``include/moeva_mi355x.h`` MV_OP_*), which the HIP kernels evaluate.  ``evaluate`` runs
that program on the GPU through the C ABI; there is no CPU evaluation path.
"""
from __future__ import annotations

import abc
import logging
import os
from typing import List, Tuple, Union

import numpy as np
import pandas as pd

from ..._native import OP


class ConstraintProgram:
    """Builder for the device constraint program (op codes + operands + index pool)."""

    def __init__(self):
        self.code: List[int] = []
        self.arg: List[List[int]] = []
        self.karg: List[List[float]] = []
        self.pool: List[int] = []

    def add(self, op: str, a=(), k=()):
        a = list(a) + [0] * (4 - len(a))
        k = list(k) + [0.0] * (2 - len(k))
        self.code.append(OP[op])
        self.arg.append([int(v) for v in a])
        self.karg.append([float(v) for v in k])

    def add_sumdiff(self, first: List[int], second: List[int]):
        o0 = len(self.pool)
        self.pool.extend(int(v) for v in first)
        o1 = len(self.pool)
        self.pool.extend(int(v) for v in second)
        self.add("ABS_SUMDIFF", (o0, o1, len(self.pool)))

    def arrays(self):
        return (np.asarray(self.code, np.int32), np.asarray(self.arg, np.int32).reshape(-1, 4),
                np.asarray(self.karg, np.float64).reshape(-1, 2), np.asarray(self.pool, np.int32))

    def __len__(self):
        return len(self.code)


class Constraints(abc.ABC, metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def evaluate(self, x: np.ndarray, use_tensors: bool = False) -> np.ndarray:
        """(n_samples, n_features) -> (n_samples, n_constraints) distances to satisfaction."""
        raise NotImplementedError

    @abc.abstractmethod
    def get_nb_constraints(self) -> int:
        raise NotImplementedError

    @abc.abstractmethod
    def normalise(self, x: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    @abc.abstractmethod
    def get_constraints_min_max(self) -> Tuple[np.ndarray, np.ndarray]:
        raise NotImplementedError

    @abc.abstractmethod
    def get_mutable_mask(self) -> np.ndarray:
        raise NotImplementedError

    @abc.abstractmethod
    def get_feature_min_max(self, dynamic_input=None) -> Tuple[np.ndarray, np.ndarray]:
        raise NotImplementedError

    @abc.abstractmethod
    def fix_features_types(self, x) -> Union[np.ndarray, object]:
        raise NotImplementedError

    @abc.abstractmethod
    def get_feature_type(self) -> np.ndarray:
        raise NotImplementedError

    def device_program(self) -> ConstraintProgram:
        """The numpy path of ``evaluate`` as a device program (engine extension)."""
        raise NotImplementedError(
            f"{type(self).__name__} has no device constraint program; the MI355X engine "
            "evaluates constraints only through device programs")

    def check_constraints_error(self, x: np.ndarray):
        """constraints.py:73-77."""
        constraints = self.evaluate(x)
        constraints_violated = (constraints > 0).sum()
        if constraints_violated > 0:
            raise ValueError(f"Constraints not respected {constraints_violated} times.")


class TabularConstraints(Constraints):
    """CSV-provisioned constraints shared by the LCLD and botnet classes
    (lcld_constraints.py:225-279, botnet_constraints.py:178-232)."""

    tol = 1e-3

    def __init__(self, feature_path: str, constraints_path: str):
        self._feature_path = feature_path
        self._provision_constraints_min_max(constraints_path)
        self._provision_feature_constraints(feature_path)
        self._fit_scaler()
        self._engines = {}  # device index -> constraint-only Engine

    # -- provisioning (pandas.read_csv exactly like the reference: its C parser decides
    #    the last bits of the bounds)
    def _provision_feature_constraints(self, path: str) -> None:
        df = pd.read_csv(path, low_memory=False)
        self._feature_min = df["min"].to_numpy()
        self._feature_max = df["max"].to_numpy()
        self._mutable_mask = df["mutable"].to_numpy()
        self._feature_type = df["type"].to_numpy()

    def _provision_constraints_min_max(self, path: str) -> None:
        df = pd.read_csv(path, low_memory=False)
        self._constraints_min = df["min"].to_numpy()
        self._constraints_max = df["max"].to_numpy()

    def _fit_scaler(self) -> None:
        lo = np.asarray(self._constraints_min, np.float64)
        hi = np.asarray(self._constraints_max, np.float64)
        rng = hi - lo
        rng = np.where(rng == 0, 1.0, rng)
        self._c_scale = 1.0 / rng
        self._c_min = 0.0 - lo * self._c_scale

    def normalise(self, x: np.ndarray) -> np.ndarray:
        x = np.array(x, dtype=np.float64, copy=True)
        x *= self._c_scale
        x += self._c_min
        return x

    def get_constraints_min_max(self):
        return self._constraints_min, self._constraints_max

    def get_mutable_mask(self) -> np.ndarray:
        return self._mutable_mask

    def get_feature_type(self) -> np.ndarray:
        return self._feature_type

    def get_nb_constraints(self) -> int:
        return len(self.device_program())

    def fix_features_types(self, x):
        raise NotImplementedError("TensorFlow repair path (C-PGD) is out of scope")

    def get_feature_min_max(self, dynamic_input=None):
        """lcld_constraints.py:237-263: 'dynamic' bounds come from the input."""
        feature_min = np.array([0.0] * self._feature_min.shape[0])
        feature_max = np.array([0.0] * self._feature_max.shape[0])
        min_dynamic = self._feature_min.astype(str) == "dynamic"
        max_dynamic = self._feature_max.astype(str) == "dynamic"
        feature_min[~min_dynamic] = self._feature_min[~min_dynamic]
        feature_max[~max_dynamic] = self._feature_max[~max_dynamic]
        if dynamic_input is not None:
            feature_min[min_dynamic] = dynamic_input[min_dynamic]
            feature_max[max_dynamic] = dynamic_input[max_dynamic]
        dynamic_number = min_dynamic.sum() + max_dynamic.sum()
        if dynamic_number > 0 and dynamic_input is None:
            logging.getLogger().warning(
                f"{dynamic_number} feature min and max are dynamic but no input were provided.")
        return feature_min, feature_max

    def feature_min_max_batch(self, X: np.ndarray):
        """``get_feature_min_max(dynamic_input=x)`` for every row x of X at once (engine
        extension, Moeva2.generate's per-state bounds): (xl, xu), each (n, D) fp64, the
        same values as the per-row calls -- the static bounds are converted once exactly as
        lcld_constraints.py:248-249 converts them, the dynamic ones are X's own values."""
        X = np.asarray(X, dtype=np.float64)
        st = getattr(self, "_static_bounds", None)
        if st is None:
            st = self._static_bounds = self._static_min_max() + self._dynamic_masks()
        lo, hi, min_dyn, max_dyn = st
        return np.where(min_dyn, X, lo), np.where(max_dyn, X, hi)

    def _dynamic_masks(self):
        return (self._feature_min.astype(str) == "dynamic",
                self._feature_max.astype(str) == "dynamic")

    def _static_min_max(self):
        """The non-dynamic entries of get_feature_min_max, converted as it converts them
        (dynamic entries left at 0.0)."""
        min_dyn, max_dyn = self._dynamic_masks()
        feature_min = np.array([0.0] * self._feature_min.shape[0])
        feature_max = np.array([0.0] * self._feature_max.shape[0])
        feature_min[~min_dyn] = self._feature_min[~min_dyn]
        feature_max[~max_dyn] = self._feature_max[~max_dyn]
        return feature_min, feature_max

    # -- device evaluation
    def _constraint_engine(self, device=None):
        """The constraint-only engine on ``device`` (default: torch's current device), built
        on first use; every device gets its own, so a caller never hands one GPU's buffers
        to an engine on another."""
        import torch

        dev = torch.cuda.current_device() if device is None else int(device)
        eng = self._engines.get(dev)
        if eng is None:
            from ...problem import build_device_program
            from ..._native import Engine

            eng = self._engines[dev] = Engine(build_device_program(self), None, None,
                                              device=dev)
        return eng

    def evaluate(self, x: np.ndarray, use_tensors: bool = False) -> np.ndarray:
        if use_tensors:
            raise NotImplementedError("TensorFlow evaluation path (C-PGD) is out of scope")
        import torch

        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
        eng = self._constraint_engine()
        xd = torch.from_numpy(x).cuda(eng.device)
        g = torch.empty((x.shape[0], eng.prog.C), dtype=torch.float64, device=xd.device)
        eng.constraints(xd, g, stream=torch.cuda.current_stream(xd.device))
        return g.cpu().numpy()


def _resolve(path_hint: str, name: str) -> str:
    """Reference classes read './data/<project>/<name>' relative to the CWD; resolve the
    same file next to the features CSV first, then the CWD form."""
    here = os.path.join(os.path.dirname(os.path.abspath(path_hint)), name)
    return here if os.path.exists(here) else name
