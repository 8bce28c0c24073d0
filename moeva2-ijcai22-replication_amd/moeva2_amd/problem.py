"""Assemble the C-ABI problem description from the reference-shaped host objects
(Constraints + FeatureEncoder + classifier + ML scaler), and cache engines."""
from __future__ import annotations

import numpy as np

from ._native import DeviceProgram, Engine
from .attacks.moeva2.feature_encoder import get_encoder_from_constraints


def build_device_program(constraints) -> DeviceProgram:
    enc = get_encoder_from_constraints(constraints)
    kind, feat, offs, ohe_feats, mut_feats = enc.device_layout()
    code, arg, karg, pool = constraints.device_program().arrays()
    return DeviceProgram(D=int(enc.mutable_mask.shape[0]), gene_kind=kind, gene_feat=feat,
                         ohe_offsets=offs, ohe_feats=ohe_feats, mut_feats=mut_feats,
                         op_code=code, op_arg=arg, op_karg=karg, idx_pool=pool,
                         tol=getattr(constraints, "tol", 1e-3))


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
        mlp = classifier.dense_weights()
        s, m = scaler_arrays(ml_scaler)
        eng = Engine(build_device_program(constraints), mlp.weights, mlp.biases, s, m, norm,
                     scale_objectives, device)
        _ENGINES[key] = (eng, constraints, classifier, ml_scaler)  # keep referents alive
        return eng
    return eng[0]
