"""Declarative model base for the PyTorchJob SDK.

The reference SDK's models are swagger-codegen classes (sdk/python/kubeflow/pytorchjob/
models/*.py): ``swagger_types`` + ``attribute_map`` class tables, one property per
field, required fields that raise ``ValueError`` when set to None, ``to_dict``
(snake_case keys), ``to_str``/``__repr__``/``__eq__``.  Here a field table drives all of
that, so each model is a few lines and every model behaves identically.
"""
from __future__ import annotations

import pprint
from typing import Any, Dict, List, Tuple


class Model:
    # (attribute name, JSON key, type string) -- type strings use swagger notation:
    # 'str', 'int', 'V1Foo', 'list[V1Foo]', 'dict(str, V1Foo)', 'object'
    _fields: List[Tuple[str, str, str]] = []
    _required: Tuple[str, ...] = ()

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        cls.swagger_types = {a: t for a, _, t in cls._fields}
        cls.attribute_map = {a: j for a, j, _ in cls._fields}
        for attr, _, _ in cls._fields:
            setattr(cls, attr, _make_property(attr, attr in cls._required, cls.__name__))

    def __init__(self, **kwargs):
        unknown = set(kwargs) - set(self.swagger_types)
        if unknown:
            raise TypeError(f"{type(self).__name__}() got unexpected arguments {sorted(unknown)}")
        self.discriminator = None
        for attr in self.swagger_types:
            object.__setattr__(self, "_" + attr, None)
        for attr in self.swagger_types:
            val = kwargs.get(attr)
            if val is not None or attr in self._required:
                setattr(self, attr, val)

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for attr in self.swagger_types:
            out[attr] = _to_dict(getattr(self, attr))
        return out

    def to_str(self) -> str:
        return pprint.pformat(self.to_dict())

    def __repr__(self) -> str:
        return self.to_str()

    def __eq__(self, other) -> bool:
        return isinstance(other, type(self)) and self.__dict__ == other.__dict__

    def __ne__(self, other) -> bool:
        return not self == other


def _make_property(attr: str, required: bool, owner: str):
    key = "_" + attr

    def getter(self):
        return getattr(self, key)

    def setter(self, value):
        if required and value is None:
            raise ValueError(f"Invalid value for `{attr}`, must not be `None`")
        object.__setattr__(self, key, value)

    return property(getter, setter, doc=f"{owner}.{attr}")


def _to_dict(v):
    if isinstance(v, list):
        return [_to_dict(x) for x in v]
    if isinstance(v, dict):
        return {k: _to_dict(x) for k, x in v.items()}
    if hasattr(v, "to_dict"):
        return v.to_dict()
    return v
