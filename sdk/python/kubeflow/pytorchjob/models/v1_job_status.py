from .base import Model


class V1JobStatus(Model):
    _fields = [("completion_time", "completionTime", "V1Time"),
               ("conditions", "conditions", "list[V1JobCondition]"),
               ("last_reconcile_time", "lastReconcileTime", "V1Time"),
               ("replica_statuses", "replicaStatuses", "dict(str, V1ReplicaStatus)"),
               ("start_time", "startTime", "V1Time")]
    _required = ("conditions", "replica_statuses")
