from .base import Model


class V1PyTorchJobList(Model):
    _fields = [("api_version", "apiVersion", "str"),
               ("items", "items", "list[V1PyTorchJob]"),
               ("kind", "kind", "str"),
               ("metadata", "metadata", "V1ListMeta")]
    _required = ("items",)
