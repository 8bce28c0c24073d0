"""Decode the reference's pickled data files WITHOUT executing anything from them.

The reference reads ``data/botnet/feat_idx.pickle`` with ``pickle.load``
(``src/examples/botnet/botnet_constraints.py:26-27``) and its ML scalers with
``joblib.load`` (``src/experiments/united/04_moeva.py:311``).  Both would run
arbitrary code from the file.  This module walks the pickle opcode stream with
``pickletools.genops`` (a pure parser) and interprets a whitelisted subset of
opcodes into plain data:

* containers / scalars (dict, list, tuple, int, float, str, bool, None);
* ``GLOBAL``/``STACK_GLOBAL`` + ``NEWOBJ``/``REDUCE``/``BUILD`` become inert
  :class:`Obj` records (class path, args, state) -- no import, no call;
* joblib's ``NumpyArrayWrapper`` records are followed by the raw array bytes in
  the stream (joblib <=0.17 layout, no alignment padding); those bytes are read
  into a ``numpy.ndarray`` with ``numpy.frombuffer``.
"""
from __future__ import annotations

import io
import pickletools
from dataclasses import dataclass, field
from typing import Any

import numpy as np


@dataclass
class Obj:
    cls: str
    args: tuple = ()
    state: Any = None
    items: dict = field(default_factory=dict)


_MARK = object()


def _dtype_from(obj: Obj) -> np.dtype:
    if not (isinstance(obj, Obj) and obj.cls == "numpy.dtype"):
        raise ValueError(f"unexpected dtype record {obj!r}")
    dt = np.dtype(obj.args[0])
    if isinstance(obj.state, tuple) and len(obj.state) > 1 and obj.state[1] in "<>|=":
        dt = dt.newbyteorder(obj.state[1])
    return dt


def safe_load(path: str) -> Any:
    with open(path, "rb") as f:
        stream = io.BytesIO(f.read())
    stack: list = []
    memo: dict = {}
    gen = pickletools.genops(stream)
    for op, arg, _pos in gen:
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name in ("EMPTY_DICT",):
            stack.append({})
        elif name in ("EMPTY_LIST",):
            stack.append([])
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT"):
            stack.append(int(arg))
        elif name in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE",
                      "SHORT_BINSTRING", "BINSTRING", "STRING"):
            stack.append(arg)
        elif name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            n = int(name[-1])
            t = tuple(stack[-n:])
            del stack[-n:]
            stack.append(t)
        elif name in ("TUPLE", "LIST", "APPENDS", "SETITEMS", "DICT"):
            k = max(i for i, v in enumerate(stack) if v is _MARK)
            items = stack[k + 1:]
            del stack[k:]
            if name == "TUPLE":
                stack.append(tuple(items))
            elif name == "LIST":
                stack.append(list(items))
            elif name == "DICT":
                stack.append(dict(zip(items[::2], items[1::2])))
            elif name == "APPENDS":
                stack[-1].extend(items)
            else:
                tgt = stack[-1]
                for kk, vv in zip(items[::2], items[1::2]):
                    if isinstance(tgt, Obj):
                        tgt.items[kk] = vv
                    else:
                        tgt[kk] = vv
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "SETITEM":
            v = stack.pop()
            kk = stack.pop()
            stack[-1][kk] = v
        elif name == "STACK_GLOBAL":
            nm = stack.pop()
            mod = stack.pop()
            stack.append(("__global__", f"{mod}.{nm}"))
        elif name == "GLOBAL":
            mod, nm = arg.split(" ")
            stack.append(("__global__", f"{mod}.{nm}"))
        elif name in ("NEWOBJ", "REDUCE"):
            args = stack.pop()
            g = stack.pop()
            if not (isinstance(g, tuple) and g and g[0] == "__global__"):
                raise ValueError(f"refusing to call non-global {g!r}")
            stack.append(Obj(g[1], tuple(args)))
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Obj):
                raise ValueError("BUILD on a non-object record")
            obj.state = state
            if obj.cls == "joblib.numpy_pickle.NumpyArrayWrapper":
                st = state
                dt = _dtype_from(st["dtype"])
                shape = tuple(st["shape"])
                count = int(np.prod(shape)) if shape else 1
                raw = stream.read(count * dt.itemsize)
                arr = np.frombuffer(raw, dtype=dt, count=count).reshape(
                    shape, order=st.get("order", "C")).copy()
                stack[-1] = arr
        else:
            raise ValueError(f"pickle opcode {name} is not in the safe subset")
    if len(stack) != 1:
        raise ValueError("malformed pickle stream")
    return stack[0]


@dataclass
class MinMaxParams:
    """Fitted sklearn ``MinMaxScaler`` state (``transform(X) = X * scale_ + min_``)."""

    scale_: np.ndarray
    min_: np.ndarray
    data_min_: np.ndarray
    data_max_: np.ndarray
    feature_range: tuple = (0, 1)

    def transform(self, x: np.ndarray) -> np.ndarray:
        x = np.array(x, dtype=np.float64, copy=True)
        x *= self.scale_
        x += self.min_
        return x


def load_minmax_scaler(path: str) -> MinMaxParams:
    obj = safe_load(path)
    if not (isinstance(obj, Obj) and obj.cls.endswith("MinMaxScaler")):
        raise ValueError(f"{path}: not a MinMaxScaler record ({getattr(obj, 'cls', obj)!r})")
    st = obj.state
    return MinMaxParams(
        np.asarray(st["scale_"], np.float64),
        np.asarray(st["min_"], np.float64),
        np.asarray(st["data_min_"], np.float64),
        np.asarray(st["data_max_"], np.float64),
        tuple(st.get("feature_range", (0, 1))),
    )
