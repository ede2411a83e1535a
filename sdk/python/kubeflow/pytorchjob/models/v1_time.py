"""V1Time: an RFC 3339 timestamp string (reference models/v1_time.py is an empty shell)."""
from .base import Model


class V1Time(Model):
    _fields = []
