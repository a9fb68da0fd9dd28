"""Spark-ML ``Params``: typed params with defaults, fluent ``setX``/``getX`` accessors,
``explainParams``, ``extractParamMap`` and uid generation (``Identifiable.randomUID``)."""
from __future__ import annotations

import copy as _copy
import itertools
import os
from typing import Any, Callable, Dict, Optional

__all__ = ["Param", "Params", "random_uid", "param_accessors"]


# Spark's Identifiable.randomUID takes 12 hex digits of a random UUID; uids only need to be
# distinct, so a per-process random base plus a counter gives the same form without an
# os.urandom call per estimator (two per rebuilt lab action)
_UID_BASE = int.from_bytes(os.urandom(6), "little")
_uid_seq = itertools.count()


def random_uid(prefix: str) -> str:
    return f"{prefix}_{(_UID_BASE + 0x9E3779B97F4A * next(_uid_seq)) & 0xFFFFFFFFFFFF:012x}"


class Param:
    def __init__(self, name: str, doc: str, default: Any = None, validator: Optional[Callable] = None,
                 has_default: bool = True, converter: Optional[Callable] = None):
        self.name, self.doc, self.default = name, doc, default
        self.validator = validator
        self.has_default = has_default
        self.converter = converter

    def __repr__(self):
        return f"Param({self.name})"


class Params:
    _params: Dict[str, Param] = {}
    uid_prefix = "params"

    def __init__(self, uid: Optional[str] = None):
        self.uid = uid or random_uid(self.uid_prefix)
        self._paramMap: Dict[str, Any] = {}

    # ---- core ------------------------------------------------------------------------------
    @classmethod
    def params_list(cls):
        cached = cls.__dict__.get("_params_cache")
        if cached is not None:
            return cached
        out = {}
        for k in reversed(cls.__mro__):
            out.update(getattr(k, "_params", {}) or {})
        cls._params_cache = out
        return out

    def _param(self, name) -> Param:
        p = self.params_list().get(name)
        if p is None:
            raise KeyError(f"Param {name} does not exist.")
        return p

    def set(self, name, value):
        p = self._param(name)
        if p.converter is not None and value is not None:
            value = p.converter(value)
        if p.validator is not None and not p.validator(value):
            raise ValueError(f"{type(self).__name__}_{self.uid} parameter {name} given invalid value {value}.")
        self._paramMap[name] = value
        return self

    _set = set

    def clear(self, name):
        self._paramMap.pop(name, None)
        return self

    def isSet(self, name):
        return name in self._paramMap

    def hasDefault(self, name):
        return self._param(name).has_default

    def isDefined(self, name):
        return self.isSet(name) or self.hasDefault(name)

    def getOrDefault(self, name):
        if name in self._paramMap:
            return self._paramMap[name]
        p = self._param(name)
        if not p.has_default:
            raise KeyError(f"Failed to find a default value for {name}")
        return p.default

    def extractParamMap(self):
        return {n: self.getOrDefault(n) for n in self.params_list() if self.isDefined(n)}

    def explainParam(self, name):
        p = self._param(name)
        parts = []
        if p.has_default:
            parts.append(f"default: {p.default}")
        if name in self._paramMap:
            parts.append(f"current: {self._paramMap[name]}")
        return f"{name}: {p.doc} ({', '.join(parts) if parts else 'undefined'})"

    def explainParams(self):
        return "\n".join(self.explainParam(n) for n in sorted(self.params_list()))

    def copy(self, extra=None):
        c = _copy.copy(self)
        c._paramMap = dict(self._paramMap)
        for k, v in (extra or {}).items():
            c.set(k, v)
        return c

    def copyValues(self, to: "Params"):
        for k, v in self._paramMap.items():
            if k in to.params_list():
                to._paramMap[k] = v
        return to

    @property
    def params(self):
        return list(self.params_list().values())


def param_accessors(cls):
    """Class decorator: add ``setX``/``getX`` for every declared param."""
    for name in cls.params_list():
        cap = name[0].upper() + name[1:]
        if not hasattr(cls, "set" + cap):
            setattr(cls, "set" + cap, (lambda n: lambda self, v: self.set(n, v))(name))
        if not hasattr(cls, "get" + cap):
            setattr(cls, "get" + cap, (lambda n: lambda self: self.getOrDefault(n))(name))
    return cls
