from .base import Model


class V1PyTorchJob(Model):
    _fields = [("api_version", "apiVersion", "str"),
               ("kind", "kind", "str"),
               ("metadata", "metadata", "V1ObjectMeta"),
               ("spec", "spec", "V1PyTorchJobSpec"),
               ("status", "status", "V1JobStatus")]
