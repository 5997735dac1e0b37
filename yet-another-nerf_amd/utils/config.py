"""Config files with attribute access (yml / json / py), the subset of the reference's MMCV-style Config
(yanerf/utils/config.py:35-600) that the hot path's callers use: attribute-accessible nested dicts
(NeRFPipeline reads `ray_sampler.image_height` and `renderer.bg_color` by attribute, nerf_pipeline.py:43-59),
`_base_` inheritance, the `{{ fileDirname }}` substitution used by py configs, and `merge_from_dict`
(`--cfg_options a.b=c`)."""
from __future__ import annotations

import copy
import json
import os
import runpy
import tempfile
from pathlib import Path
from typing import Any

import yaml


class ConfigDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = _wrap(v)

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(f"'ConfigDict' has no attribute '{name}'")

    def __setattr__(self, name, value):
        self[name] = _wrap(value)

    def __setitem__(self, key, value):
        super().__setitem__(key, _wrap(value))

    def __deepcopy__(self, memo):
        return ConfigDict({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def copy(self):
        return ConfigDict(self)

    def to_dict(self):
        return _unwrap(self)


def _wrap(v):
    if isinstance(v, ConfigDict):
        return v
    if isinstance(v, dict):
        return ConfigDict(v)
    if isinstance(v, list):
        return [_wrap(e) for e in v]
    if isinstance(v, tuple):
        return tuple(_wrap(e) for e in v)
    return v


def _unwrap(v):
    if isinstance(v, dict):
        return {k: _unwrap(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_unwrap(e) for e in v]
    if isinstance(v, tuple):
        return tuple(_unwrap(e) for e in v)
    return v


def _merge(base: dict, new: dict) -> dict:
    out = dict(base)
    for k, v in new.items():
        if isinstance(v, dict) and not v.pop("_delete_", False) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = v
    return out


class Config:
    def __init__(self, cfg_dict: Any = None, filename: str = None):
        object.__setattr__(self, "_cfg_dict", ConfigDict(cfg_dict or {}))
        object.__setattr__(self, "_filename", filename)

    @property
    def filename(self):
        return self._filename

    @staticmethod
    def _file2dict(filename: str) -> dict:
        filename = os.path.abspath(os.path.expanduser(filename))
        suffix = Path(filename).suffix
        text = Path(filename).read_text()
        text = text.replace("{{ fileDirname }}", os.path.dirname(filename)).replace(
            "{{ fileBasename }}", os.path.basename(filename))
        if suffix in (".yml", ".yaml"):
            d = yaml.safe_load(text) or {}
        elif suffix == ".json":
            d = json.loads(text)
        elif suffix == ".py":
            with tempfile.TemporaryDirectory() as td:
                tmp = Path(td) / "cfg_tmp.py"
                tmp.write_text(text)
                ns = runpy.run_path(str(tmp))
            d = {k: v for k, v in ns.items() if not k.startswith("__") and not callable(v) and not isinstance(
                v, type(os))}
            d = {k: (v.to_dict() if isinstance(v, (Config,)) else v) for k, v in d.items()}
        else:
            raise IOError(f"unsupported config type {suffix}")
        d = _unwrap(d)
        base = d.pop("_base_", None)
        if base is not None:
            bases = base if isinstance(base, list) else [base]
            merged = {}
            for b in bases:
                merged = _merge(merged, Config._file2dict(os.path.join(os.path.dirname(filename), b)))
            d = _merge(merged, d)
        return d

    @staticmethod
    def fromfile(filename: str) -> "Config":
        return Config(Config._file2dict(filename), filename=filename)

    def to_dict(self):
        return self._cfg_dict.to_dict()

    def merge_from_dict(self, options: dict) -> None:
        d = self._cfg_dict
        for full_key, v in options.items():
            keys = full_key.split(".")
            cur = d
            for k in keys[:-1]:
                cur = cur.setdefault(k, ConfigDict())
            cur[keys[-1]] = v

    @property
    def pretty_text(self) -> str:
        return yaml.safe_dump(self.to_dict(), sort_keys=False)

    def __getattr__(self, name):
        return getattr(self._cfg_dict, name)

    def __getitem__(self, name):
        return self._cfg_dict[name]

    def __setattr__(self, name, value):
        self._cfg_dict[name] = value

    def __contains__(self, name):
        return name in self._cfg_dict

    def __repr__(self):
        return f"Config (path: {self._filename}): {self._cfg_dict}"
