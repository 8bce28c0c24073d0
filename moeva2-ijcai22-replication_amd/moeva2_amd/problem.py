"""Assemble the C-ABI problem description from the reference-shaped host objects
(Constraints + FeatureEncoder + classifier + ML scaler), and cache engines."""
from __future__ import annotations

import numpy as np

from ._native import DeviceProgram, Engine
from .attacks.moeva2.feature_encoder import get_encoder_from_constraints


def has_device_program(constraints) -> bool:
    """True when the Constraints object describes its numpy path as a device program (the
    shipped LCLD / botnet classes); any other subclass is evaluated by its own ``evaluate``
    on the host (SURVEY.md §8b plugin fallback)."""
    if not callable(getattr(constraints, "device_program", None)):
        return False  # a duck-typed plugin that does not derive from our Constraints
    try:
        constraints.device_program()
        return True
    except NotImplementedError:
        return False


def has_device_classifier(classifier) -> bool:
    """True for Dense(relu)...Dense(softmax) models the engine runs on MFMA; any other
    ``predict_proba`` model is called on the host."""
    try:
        classifier.dense_weights()
        return True
    except (NotImplementedError, AttributeError, ValueError):
        return False


def build_device_program(constraints, with_constraints=True) -> DeviceProgram:
    enc = get_encoder_from_constraints(constraints)
    kind, feat, offs, ohe_feats, mut_feats = enc.device_layout()
    if with_constraints:
        code, arg, karg, pool = constraints.device_program().arrays()
    else:  # host-evaluated constraints: the device program is empty (f3 filled by the host)
        code, arg, karg, pool = (np.zeros(0, np.int32), np.zeros((0, 4), np.int32),
                                 np.zeros((0, 2)), np.zeros(0, np.int32))
    return DeviceProgram(D=int(enc.mutable_mask.shape[0]), gene_kind=kind, gene_feat=feat,
                         ohe_offsets=offs, ohe_feats=ohe_feats, mut_feats=mut_feats,
                         op_code=code, op_arg=arg, op_karg=karg, idx_pool=pool,
                         tol=getattr(constraints, "tol", 1e-3))


def ml_transform(ml_scaler, x_f):
    """default_problem.py:119-121: ``ml_scaler.transform(x_f)`` (identity without a scaler);
    fitted-array records (scale_, min_) use the same multiply-add form."""
    if ml_scaler is None:
        return x_f
    if hasattr(ml_scaler, "transform"):
        return ml_scaler.transform(x_f)
    y = np.array(x_f, dtype=np.float64, copy=True)
    y *= np.asarray(ml_scaler.scale_, np.float64)
    y += np.asarray(ml_scaler.min_, np.float64)
    return y


def scaler_arrays(ml_scaler):
    """(scale_, min_) of a fitted MinMaxScaler-like object (sklearn or safe_pickle record)."""
    if ml_scaler is None:
        return None, None
    return (np.asarray(ml_scaler.scale_, np.float64), np.asarray(ml_scaler.min_, np.float64))


_ENGINES = {}


def get_engine(constraints, classifier, ml_scaler, norm, scale_objectives=True, device=0):
    """One engine per (constraints object, classifier weights, scaler, norm, device)."""
    key = (id(constraints), id(classifier), id(ml_scaler), str(norm), bool(scale_objectives),
           device)
    eng = _ENGINES.get(key)
    if eng is None:
        dev_clf = has_device_classifier(classifier)
        mlp = classifier.dense_weights() if dev_clf else None
        s, m = scaler_arrays(ml_scaler) if dev_clf else (None, None)
        eng = Engine(build_device_program(constraints, has_device_program(constraints)),
                     mlp.weights if mlp else None, mlp.biases if mlp else None, s, m, norm,
                     scale_objectives, device)
        _ENGINES[key] = (eng, constraints, classifier, ml_scaler)  # keep referents alive
        return eng
    return eng[0]
