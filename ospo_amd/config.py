"""Config system mirroring ospo/utils/common.py:10-24,90-108 without OmegaConf.

``build_config(cfg_path)`` = YAML load + ``key.sub=value`` CLI dotlist merge ->
``AttrDict`` (attribute AND key access, nested).  ``save_config`` writes the
config as JSON text into ``{save_path}/config.yaml`` exactly like the
reference (common.py:102-108) -- that file is what ospo/inference.py reads
back through ``get_lora_config`` (ospo/utils/model.py:74-89).

Reference quirks the entry point tolerates: ``use_peft`` and
``use_lora`` are aliases; empty ``val_steps``/``max_training_steps``/... get
usable defaults instead of raising TypeError.
"""
from __future__ import annotations

import ast
import json
import os
import sys
from typing import Any, List, Optional

import yaml


class AttrDict(dict):
    """dict with attribute access (ospo/utils/common.py:10-24)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @classmethod
    def from_nested_dicts(cls, data):
        if not isinstance(data, dict):
            return data
        return cls({k: cls.from_nested_dicts(v) for k, v in data.items()})


def _parse_value(v: str) -> Any:
    if v.lower() in ("null", "none", "~", ""):
        return None
    if v.lower() in ("true", "false"):
        return v.lower() == "true"
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def merge_dotlist(cfg: dict, dotlist: List[str]) -> dict:
    """OmegaConf.from_cli semantics for ``a.b.c=value`` tokens."""
    for tok in dotlist:
        if "=" not in tok:
            continue
        key, val = tok.split("=", 1)
        key = key.lstrip("-")
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            if not isinstance(node.get(p), dict):
                node[p] = {}
            node = node[p]
        node[parts[-1]] = _parse_value(val)
    return cfg


def build_config(cfg_path: Optional[str] = None, argv: Optional[List[str]] = None) -> AttrDict:
    if cfg_path is None:
        raise ValueError("No cfg_path given.")
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f) or {}
    argv = sys.argv[1:] if argv is None else argv
    cfg = merge_dotlist(cfg, [a for a in argv if "=" in a and not a.startswith("--cfg_path")])
    # use_peft (configs/step5.yaml:13) and use_lora (model.py:48, utils/train.py:19) are the same switch
    if "use_lora" not in cfg and "use_peft" in cfg:
        cfg["use_lora"] = cfg["use_peft"]
    if "use_peft" not in cfg and "use_lora" in cfg:
        cfg["use_peft"] = cfg["use_lora"]
    return AttrDict.from_nested_dicts(cfg)


def save_config(save_path: str, config: dict) -> str:
    os.makedirs(save_path, exist_ok=True)
    p = os.path.join(save_path, "config.yaml")
    with open(p, "w") as f:
        json.dump(config, f, indent=4)
    return p


def get(cfg, path: str, default=None):
    node = cfg
    for p in path.split("."):
        if not isinstance(node, dict) or p not in node or node[p] is None:
            return default
        node = node[p]
    return node
