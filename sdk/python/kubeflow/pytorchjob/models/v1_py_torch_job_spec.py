from .base import Model


class V1PyTorchJobSpec(Model):
    _fields = [("active_deadline_seconds", "activeDeadlineSeconds", "int"),
               ("backoff_limit", "backoffLimit", "int"),
               ("clean_pod_policy", "cleanPodPolicy", "str"),
               ("pytorch_replica_specs", "pytorchReplicaSpecs", "dict(str, V1ReplicaSpec)"),
               ("ttl_seconds_after_finished", "ttlSecondsAfterFinished", "int")]
    _required = ("pytorch_replica_specs",)
