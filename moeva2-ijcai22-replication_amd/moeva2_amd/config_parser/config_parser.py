"""Experiment configuration for the MoEvA2 driver.

Behaviour contract (src/config_parser/config_parser.py:70-114, pinned by
tests/test_driver_cpu.py), implemented independently:

* sources: ``-c FILE`` (.yaml/.yml/.json), ``-j JSON`` (inline object) and
  ``-p a.b.c=value``; each flag may repeat;
* merge order: every ``-c`` in command-line order, then every ``-j``, then every ``-p``
  (the reference walks its argparse namespace in flag-definition order); a later source
  overrides an earlier one leaf by leaf, nested mappings are merged, lists and scalars are
  replaced (mergedeep ``Strategy.REPLACE``);
* ``-p`` values: a token that looks like a plain decimal number is typed the way YAML 1.1
  types it (so ``42`` -> int, ``0.2`` -> float, but ``1e-3`` stays the string "1e-3");
  anything else is kept as a string;
* the config hash is the md5 hex digest of ``json.dumps(config, sort_keys=True)``, which
  names the driver's output files (metrics_*, x_attacks_*, ...).
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys
from typing import Dict, Iterable, List, Optional, Tuple

import yaml

_NUMBER = re.compile(r"[-+]?[0-9]*\.?[0-9]+(e[-+]?[0-9]+)?")
_FLAGS = ("-c", "-j", "-p")  # merge order of the three sources


def value_parser(token: str):
    """Type a ``-p`` value: plain decimal numbers as YAML reads them, else the string."""
    if not _NUMBER.fullmatch(token):
        return str(token)
    return yaml.safe_load(token)


def _read_file(path: str) -> dict:
    ext = os.path.splitext(path)[1].lower()
    with open(path, "r") as fh:
        if ext in (".yaml", ".yml"):
            return yaml.safe_load(fh) or {}
        if ext == ".json":
            return json.load(fh)
    raise ValueError(f"config file {path!r}: expected .yaml, .yml or .json")


def _dotted(assignment: str) -> dict:
    """``a.b=v`` -> {"a": {"b": typed(v)}}."""
    if "=" not in assignment:
        raise ValueError(f"-p {assignment!r}: expected key.sub=value")
    key, raw = assignment.split("=", 1)
    node = value_parser(raw)
    for part in reversed(key.split(".")):
        node = {part: node}
    return node


_LOADERS = {"-c": _read_file, "-j": lambda s: json.loads(s), "-p": _dotted}


def merge_parameters(base: dict, update: dict) -> dict:
    """Merge ``update`` into ``base`` in place: mappings recurse, other values replace."""
    stack: List[Tuple[dict, dict]] = [(base, update)]
    while stack:
        dst, src = stack.pop()
        for k, v in src.items():
            if isinstance(v, dict) and isinstance(dst.get(k), dict):
                stack.append((dst[k], v))
            else:
                dst[k] = v
    return base


def _collect(argv: Iterable[str]) -> Dict[str, List[str]]:
    """Group the values of -c/-j/-p in command-line order (``-c x`` and ``-c=x`` forms)."""
    got: Dict[str, List[str]] = {f: [] for f in _FLAGS}
    it = iter(argv)
    for tok in it:
        flag, eq, inline = tok.partition("=")
        if flag in got and eq:
            got[flag].append(inline)
        elif tok in got:
            try:
                got[tok].append(next(it))
            except StopIteration:
                raise SystemExit(f"error: argument {tok}: expected one argument")
        elif tok in ("-h", "--help"):
            print("usage: [-c FILE]... [-j JSON]... [-p key1.key2=value]...")
            raise SystemExit(0)
        else:
            raise SystemExit(f"error: unrecognized arguments: {tok}")
    return got


def get_config(argv: Optional[Iterable[str]] = None) -> dict:
    """Merged configuration of a driver command line (default: ``sys.argv[1:]``)."""
    sources = _collect(sys.argv[1:] if argv is None else argv)
    config: dict = {}
    for flag in _FLAGS:
        for value in sources[flag]:
            merge_parameters(config, _LOADERS[flag](value))
    return config


def get_dict_hash(dictionary: dict) -> str:
    return hashlib.md5(json.dumps(dictionary, sort_keys=True).encode("utf-8")).hexdigest()


def get_config_hash(config: Optional[dict] = None, argv=None) -> str:
    return get_dict_hash(get_config(argv) if config is None else config)


def save_config(pre_path: str, config: dict) -> None:
    with open(f"{pre_path}{get_dict_hash(config)}.yaml", "w") as fh:
        yaml.safe_dump(config, fh)
