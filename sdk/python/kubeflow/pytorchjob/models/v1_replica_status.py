from .base import Model


class V1ReplicaStatus(Model):
    _fields = [("active", "active", "int"), ("failed", "failed", "int"), ("succeeded", "succeeded", "int")]
