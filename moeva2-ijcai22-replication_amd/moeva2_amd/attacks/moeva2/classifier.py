"""Classifier wrapper (mirror of src/attacks/moeva2/classifier.py) + the Dense-MLP model the
engine runs on MFMA.

``load_model(path)`` replaces ``tf.keras.models.load_model`` (src/utils/in_out.py:111-127)
for the Keras Sequential(Dense...) classifiers shipped with the reference: a SavedModel
directory is read with the tensor-bundle reader (no TensorFlow), an ``.npz`` produced by
tools/import_reference_data.py is read directly.
"""
import os

import numpy as np

from ...io.tf_bundle import DenseMLP, load_dense_mlp


class DenseMLPModel:
    """Keras-equivalent Dense(relu)...Dense(softmax) model; predict_proba runs on the GPU."""

    def __init__(self, mlp: DenseMLP):
        if any(a != "relu" for a in mlp.activations[:-1]) or mlp.activations[-1] != "softmax":
            raise ValueError(f"unsupported activations {mlp.activations}")
        self.mlp = mlp

    def dense_weights(self) -> DenseMLP:
        return self.mlp

    def predict_proba(self, x: np.ndarray) -> np.ndarray:
        from ..._native import predict_proba

        return predict_proba(self.mlp, x)


def load_model(path: str) -> DenseMLPModel:
    if os.path.isdir(path):
        return DenseMLPModel(load_dense_mlp(path))
    if path.endswith(".npz") or os.path.exists(path + ".npz"):
        d = np.load(path if path.endswith(".npz") else path + ".npz", allow_pickle=False)
        n = sum(1 for k in d.files if k.startswith("W"))
        return DenseMLPModel(DenseMLP([d[f"W{i}"] for i in range(n)],
                                      [d[f"b{i}"] for i in range(n)],
                                      [str(a) for a in d["activations"]]))
    alt = path.replace(".model", ".npz")
    if alt != path and os.path.exists(alt):
        return load_model(alt)
    raise FileNotFoundError(path)


class Classifier:
    """Wrapper for classifier having a predict_proba method (classifier.py:11-41)."""

    def __init__(self, classifier, n_jobs=1, verbose=0) -> None:
        if hasattr(classifier, "predict_proba") and callable(getattr(classifier, "predict_proba")):
            self._classifier = classifier
        else:
            raise ValueError("The provided model does not have methods 'predict_proba'.")

    def predict_proba(self, x: np.ndarray) -> np.ndarray:
        proba = self._classifier.predict_proba(x)
        if proba.shape[1] == 1:
            proba = np.concatenate((1 - proba, proba), axis=1)
        return proba

    def dense_weights(self) -> DenseMLP:
        """Weights for the device GEMM chain (engine extension)."""
        if not hasattr(self._classifier, "dense_weights"):
            raise NotImplementedError(
                "the MI355X engine runs Dense-MLP classifiers (load_model); got "
                f"{type(self._classifier).__name__}")
        return self._classifier.dense_weights()
