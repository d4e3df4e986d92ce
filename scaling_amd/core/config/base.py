"""Frozen pydantic configuration base.

Behavioural parity with the reference ``BaseConfig`` (``src/scaling/core/config/base.py:10-152``):
``extra="forbid"``, frozen models, JSON-subset YAML loading with recursive overrides, JSON-safe
``as_dict`` and a commented template generator.  Implementation is independent: serialization walks
the dumped structure directly instead of relying on torch's private pytree helpers.
"""
from __future__ import annotations

import json
from enum import Enum
from pathlib import Path
from typing import Any, Optional, TypeVar, Union

import yaml
from pydantic import BaseModel, ConfigDict

TBaseConfig = TypeVar("TBaseConfig", bound="BaseConfig")


def overwrite_recursive(d: dict, d_new: dict) -> None:
    """Deep-merge ``d_new`` into ``d`` in place (dict values merge, everything else replaces)."""
    for key, value in list(d_new.items()):
        if isinstance(value, dict):
            if not isinstance(d.get(key), dict):
                d[key] = {}
            overwrite_recursive(d[key], value)
        else:
            d[key] = value


def _jsonable(x: Any) -> Any:
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_jsonable(v) for v in x) if isinstance(x, list) else [_jsonable(v) for v in x]
    if isinstance(x, Path):
        return str(x)
    if isinstance(x, Enum):
        return x.value
    return x


class BaseConfig(BaseModel):
    """Base config: immutable, strict (unknown keys rejected) and JSON serializable."""

    model_config = ConfigDict(extra="forbid", frozen=True, protected_namespaces=())

    def as_dict(self) -> dict[Any, Any]:
        return _jsonable(self.model_dump())

    @classmethod
    def from_dict(cls: type[TBaseConfig], d: dict, overwrite_values: Optional[dict] = None) -> TBaseConfig:
        if overwrite_values is not None:
            overwrite_recursive(d, overwrite_values)
        return cls(**d)

    def as_str(self) -> str:
        return json.dumps(self.as_dict())

    @classmethod
    def from_str(cls: type[TBaseConfig], s: str) -> TBaseConfig:
        return cls.from_dict(json.loads(s))

    @classmethod
    def from_yaml(
        cls: type[TBaseConfig], yml_filename: Union[str, Path], overwrite_values: Optional[dict] = None
    ) -> TBaseConfig:
        with open(yml_filename, encoding="utf-8") as f:
            config_dict = yaml.load(f, Loader=yaml.SafeLoader)
        if overwrite_values is not None:
            overwrite_recursive(config_dict, overwrite_values)
        return cls.from_dict(config_dict)

    def save(self, out_file: Path, indent: int = 4) -> None:
        with open(out_file, "w", encoding="UTF-8") as f:
            json.dump(self.as_dict(), f, indent=indent)

    @classmethod
    def get_template_str(cls, indent: int = 4, level: int = 1) -> str:
        """YAML (JSON-subset) template of this config with field descriptions as comments."""

        def comment(text: Optional[str], lvl: int) -> str:
            if text is None or not text.strip():
                return ""
            pad = " " * indent * lvl
            return pad + "# " + text.strip().replace("\n", "\n" + pad + "# ") + "\n"

        fields = cls.model_fields
        names = list(cls.model_json_schema(by_alias=False)["properties"].keys())
        out = ["{\n", comment(cls.__name__, level), comment(cls.__doc__, level)]
        for i, name in enumerate(names):
            info = fields[name]
            out.append(" " * level * indent + "\n")
            out.append(comment(info.description, level))
            out.append(" " * level * indent + f'"{name}": ')
            default = info.default
            if isinstance(default, BaseConfig):
                out.append(default.get_template_str(indent=indent, level=level + 1))
            elif isinstance(default, Enum):
                out.append(json.dumps(default.value))
            elif default is not None:
                try:
                    out.append(json.dumps(_jsonable(default)))
                except TypeError:
                    out.append("null")
            if i != len(names) - 1:
                out.append(",")
            out.append("\n")
        out.append(" " * (level - 1) * indent + "}")
        return "".join(out)

    @classmethod
    def save_template(cls, out_file: Path, indent: int = 4) -> None:
        with open(out_file, "w", encoding="UTF-8") as f:
            f.write(cls.get_template_str(indent=indent))
