"""Read Keras Dense-MLP weights from a TensorFlow SavedModel tensor bundle without TensorFlow.

The reference loads its classifiers with ``tf.keras.models.load_model``
(``src/utils/in_out.py:111-127``, called per initial state at
``src/attacks/moeva2/moeva2.py:137``).  TensorFlow is not part of this stack, so
this module parses the two on-disk pieces directly:

* ``variables/variables.index`` -- a LevelDB-format SSTable (48-byte footer ->
  index block -> data blocks, prefix-compressed keys) whose values are
  ``BundleEntryProto`` messages (dtype, shape, offset, size);
* ``variables/variables.data-00000-of-00001`` -- the raw little-endian tensor bytes.

Architecture (Dense + relu ... Dense + softmax) comes from ``keras_metadata.pb``
(a JSON blob inside a protobuf) -- see ``src/experiments/{lcld,botnet}/model.py:9-20``.
Nothing in the files is executed: only bytes are decoded.
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

_TABLE_MAGIC = 0xDB4775248B80FB57
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_}


def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _read_block(data: bytes, offset: int, size: int) -> List[Tuple[bytes, bytes]]:
    block = data[offset: offset + size]
    ctype = data[offset + size]  # block trailer: 1-byte compression type + crc32
    if ctype != 0:
        raise ValueError(f"compressed SSTable block (type {ctype}) is not supported")
    n_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * n_restarts
    pos = 0
    key = b""
    out = []
    while pos < end:
        shared, pos = _varint(block, pos)
        unshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos: pos + unshared]
        pos += unshared
        out.append((key, block[pos: pos + vlen]))
        pos += vlen
    return out


def _read_sstable(path: str) -> Dict[bytes, bytes]:
    with open(path, "rb") as f:
        data = f.read()
    magic = struct.unpack_from("<Q", data, len(data) - 8)[0]
    if magic != _TABLE_MAGIC:
        raise ValueError(f"{path}: not an SSTable (magic {magic:#x})")
    footer = data[len(data) - 48:]
    _, p = _varint(footer, 0)  # metaindex offset
    _, p = _varint(footer, p)  # metaindex size
    idx_off, p = _varint(footer, p)
    idx_size, p = _varint(footer, p)
    entries: Dict[bytes, bytes] = {}
    for _, handle in _read_block(data, idx_off, idx_size):
        boff, q = _varint(handle, 0)
        bsize, _ = _varint(handle, q)
        for k, v in _read_block(data, boff, bsize):
            entries[k] = v
    return entries


def _parse_fields(msg: bytes) -> Dict[int, list]:
    """Minimal protobuf wire-format decoder: field number -> list of raw values."""
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(msg):
        tag, pos = _varint(msg, pos)
        field, wire = tag >> 3, tag & 7
        if wire == 0:
            val, pos = _varint(msg, pos)
        elif wire == 1:
            val = msg[pos: pos + 8]
            pos += 8
        elif wire == 2:
            ln, pos = _varint(msg, pos)
            val = msg[pos: pos + ln]
            pos += ln
        elif wire == 5:
            val = msg[pos: pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
        out.setdefault(field, []).append(val)
    return out


@dataclass
class BundleEntry:
    dtype: type
    shape: Tuple[int, ...]
    offset: int
    size: int


def read_bundle_index(index_path: str) -> Dict[str, BundleEntry]:
    entries = {}
    for key, value in _read_sstable(index_path).items():
        if key == b"":  # BundleHeaderProto
            continue
        f = _parse_fields(value)
        dtype = _DTYPES.get(f.get(1, [0])[0])
        shape = ()
        if 2 in f:
            dims = _parse_fields(f[2][0]).get(2, [])
            shape = tuple(_parse_fields(d).get(1, [0])[0] for d in dims)
        entries[key.decode()] = BundleEntry(
            dtype, shape, f.get(4, [0])[0], f.get(5, [0])[0]
        )
    return entries


def read_bundle_tensors(model_dir: str) -> Dict[str, np.ndarray]:
    var_dir = os.path.join(model_dir, "variables")
    entries = read_bundle_index(os.path.join(var_dir, "variables.index"))
    with open(os.path.join(var_dir, "variables.data-00000-of-00001"), "rb") as f:
        blob = f.read()
    tensors = {}
    for name, e in entries.items():
        if e.dtype is None:
            continue
        arr = np.frombuffer(blob, dtype=e.dtype, count=e.size // np.dtype(e.dtype).itemsize,
                            offset=e.offset)
        tensors[name] = arr.reshape(e.shape).copy()
    return tensors


def _keras_layers(model_dir: str) -> List[dict]:
    path = os.path.join(model_dir, "keras_metadata.pb")
    with open(path, "rb") as f:
        raw = f.read()
    start = raw.find(b'{"name"')
    depth = 0
    for i in range(start, len(raw)):
        c = raw[i: i + 1]
        if c == b"{":
            depth += 1
        elif c == b"}":
            depth -= 1
            if depth == 0:
                meta = json.loads(raw[start: i + 1])
                break
    return [l for l in meta["config"]["layers"] if l["class_name"] == "Dense"]


@dataclass
class DenseMLP:
    """Weights of a Keras Sequential of Dense layers. ``weights[i]`` is (in, out)."""

    weights: List[np.ndarray]
    biases: List[np.ndarray]
    activations: List[str]

    @property
    def dims(self) -> List[int]:
        return [self.weights[0].shape[0]] + [w.shape[1] for w in self.weights]


def load_dense_mlp(model_dir: str) -> DenseMLP:
    tensors = read_bundle_tensors(model_dir)
    layers = _keras_layers(model_dir)
    weights, biases, acts = [], [], []
    for i, layer in enumerate(layers):
        k = f"layer_with_weights-{i}/kernel/.ATTRIBUTES/VARIABLE_VALUE"
        b = f"layer_with_weights-{i}/bias/.ATTRIBUTES/VARIABLE_VALUE"
        weights.append(np.ascontiguousarray(tensors[k], dtype=np.float32))
        biases.append(np.ascontiguousarray(tensors[b], dtype=np.float32))
        acts.append(layer["config"]["activation"])
    return DenseMLP(weights, biases, acts)
