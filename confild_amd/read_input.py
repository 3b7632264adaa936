"""YAML -> attribute object (basicutility/ReadInput.py:19-48)."""
from __future__ import annotations

import yaml


def read_yaml(filename: str) -> dict:
    with open(filename, "r") as f:
        return yaml.safe_load(f)


class basic_input:
    defaults = {}

    def __init__(self, input_file: str):
        self.yamlpath = input_file
        for key, value in read_yaml(input_file).items():
            setattr(self, key, value)
        for key, value in self.__class__.defaults.items():
            if not hasattr(self, key):
                setattr(self, key, value)

    @classmethod
    def update_defaults(cls, new_defaults: dict):
        cls.defaults.update(new_defaults)
