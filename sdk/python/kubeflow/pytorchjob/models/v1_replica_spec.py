from .base import Model


class V1ReplicaSpec(Model):
    _fields = [("replicas", "replicas", "int"),
               ("restart_policy", "restartPolicy", "str"),
               ("template", "template", "V1PodTemplateSpec")]
