from .base import Model


class V1JobCondition(Model):
    """One job condition (Created/Running/Restarting/Succeeded/Failed)."""
    _fields = [("last_transition_time", "lastTransitionTime", "V1Time"),
               ("last_update_time", "lastUpdateTime", "V1Time"),
               ("message", "message", "str"),
               ("reason", "reason", "str"),
               ("status", "status", "str"),
               ("type", "type", "str")]
    _required = ("status", "type")
