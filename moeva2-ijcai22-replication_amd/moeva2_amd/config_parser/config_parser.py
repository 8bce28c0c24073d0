"""Experiment configuration (mirror of src/config_parser/config_parser.py).

Same command line as the reference drivers: ``-c FILE`` (yaml/json, repeatable), ``-j JSON``
(inline json), ``-p key1.key2=value``; later sources override earlier ones key by key
(mergedeep ``Strategy.REPLACE``, restated here since mergedeep is not a dependency).
The config hash is the md5 of the sorted-key JSON dump (``get_dict_hash``), so output
file names match the reference's for the same configuration.
"""
import abc
import argparse
import hashlib
import json
import os
import re

import yaml


def value_parser(value):
    """config_parser.py:11-16: numbers through yaml, everything else stays a string."""
    special_key = "SPECIAL_KEY"
    if re.match("^[-+]?[0-9]*\\.?[0-9]+(e[-+]?[0-9]+)?$", value) is None:
        return str(value)
    return yaml.safe_load(f"{special_key}: {value}")[special_key]


def merge_parameters(a, b):
    """Deep merge of b into a (dicts merged recursively, anything else replaced)."""
    for k, v in b.items():
        if isinstance(v, dict) and isinstance(a.get(k), dict):
            merge_parameters(a[k], v)
        else:
            a[k] = v
    return a


class Parser(abc.ABC, metaclass=abc.ABCMeta):
    def do(self, parameter_value: str):
        return self._do(parameter_value)

    @abc.abstractmethod
    def _do(self, parameter_value: str) -> dict:
        raise NotImplementedError


class ConfigFileParser(Parser):
    def __init__(self):
        self.file_parsers = {".yaml": yaml.safe_load, ".yml": yaml.safe_load, ".json": json.load}

    def _do(self, parameter_value: str) -> dict:
        extension = os.path.splitext(parameter_value)[1]
        with open(parameter_value, "r") as f:
            return self.file_parsers[extension](f)


class StrParser(Parser):
    @staticmethod
    def key_value_to_dict(key, value):
        splits = key.split(".", maxsplit=1)
        if len(splits) == 1:
            return {splits[0]: value}
        return {splits[0]: StrParser.key_value_to_dict(splits[1], value)}

    def _do(self, parameter_value: str) -> dict:
        key, value = str(parameter_value).split("=", maxsplit=1)
        return StrParser.key_value_to_dict(key, value_parser(value))


class InlineJsonParser(Parser):
    def _do(self, parameter_value: str) -> dict:
        return json.loads(str(parameter_value))


def get_config(argv=None):
    parser = argparse.ArgumentParser()
    actions = {
        parser.add_argument("-c", help="Provide config file in yaml or json.",
                            action="append").dest: ConfigFileParser(),
        parser.add_argument("-j", help="Inline json.", action="append").dest: InlineJsonParser(),
        parser.add_argument("-p", help="Provide extra parameters on the form key1.key2=value.",
                            action="append").dest: StrParser(),
    }
    args = vars(parser.parse_args(argv))
    current = {}
    for key in args:  # argparse order: -c files, then -j, then -p (as the reference)
        if args[key] is not None:
            for value in args[key]:
                merge_parameters(current, actions[key].do(value))
    return current


def get_dict_hash(dictionary):
    return hashlib.md5(json.dumps(dictionary, sort_keys=True).encode("utf-8")).hexdigest()


def get_config_hash(config=None, argv=None):
    return get_dict_hash(get_config(argv) if config is None else config)


def save_config(pre_path, config):
    with open(f"{pre_path}{get_dict_hash(config)}.yaml", "w") as f:
        yaml.safe_dump(config, f)
