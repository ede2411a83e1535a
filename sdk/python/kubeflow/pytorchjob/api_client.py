"""Model <-> JSON conversion (the part of the reference's swagger ApiClient the SDK uses:
``sanitize_for_serialization`` and ``deserialize``, sdk/python/kubeflow/pytorchjob/api_client.py)."""
import datetime
import re

from kubeflow.pytorchjob import models as _models
from kubeflow.pytorchjob.models.base import Model

_PRIMITIVES = {"str": str, "int": int, "float": float, "bool": bool}


class ApiClient(object):
    def __init__(self, configuration=None):
        self.configuration = configuration

    def sanitize_for_serialization(self, obj):
        """Model/list/dict/datetime -> plain JSON-able value with camelCase keys."""
        if obj is None:
            return None
        if isinstance(obj, (str, int, float, bool)):
            return obj
        if isinstance(obj, (list, tuple)):
            return [self.sanitize_for_serialization(x) for x in obj]
        if isinstance(obj, (datetime.datetime, datetime.date)):
            return obj.isoformat()
        if isinstance(obj, dict):
            return {k: self.sanitize_for_serialization(v) for k, v in obj.items()}
        if isinstance(obj, Model):
            return {obj.attribute_map[a]: self.sanitize_for_serialization(getattr(obj, a))
                    for a in obj.swagger_types if getattr(obj, a) is not None}
        raise TypeError(f"cannot serialise {type(obj).__name__}")

    def deserialize(self, data, klass):
        """JSON value -> model tree (``klass`` a class or swagger type string)."""
        if data is None:
            return None
        if isinstance(klass, str):
            m = re.match(r"list\[(.*)\]$", klass)
            if m:
                return [self.deserialize(x, m.group(1)) for x in data]
            m = re.match(r"dict\(([^,]*), (.*)\)$", klass)
            if m:
                return {k: self.deserialize(v, m.group(2)) for k, v in data.items()}
            if klass in _PRIMITIVES:
                try:
                    return _PRIMITIVES[klass](data)
                except (TypeError, ValueError):
                    return data
            if klass in ("object", "datetime", "V1Time"):
                return data
            klass = getattr(_models, klass, None)
            if klass is None:
                return data
        if not isinstance(data, dict):
            return data
        kwargs = {}
        for attr, typ in klass.swagger_types.items():
            key = klass.attribute_map[attr]
            if key in data:
                kwargs[attr] = self.deserialize(data[key], typ)
        try:
            return klass(**kwargs)
        except ValueError:
            # server objects may omit fields the schema marks required (e.g. an empty status)
            obj = klass.__new__(klass)
            obj.discriminator = None
            for attr in klass.swagger_types:
                object.__setattr__(obj, "_" + attr, kwargs.get(attr))
            return obj
