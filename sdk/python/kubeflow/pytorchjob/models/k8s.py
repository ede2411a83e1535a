"""The core/v1 model subset a PyTorchJob spec needs.

The reference SDK builds jobs from ``kubernetes.client`` models (V1ObjectMeta,
V1PodTemplateSpec, V1PodSpec, V1Container, V1ResourceRequirements, ...; see its
test/test_e2e.py).  The ``kubernetes`` package is not available here, so the same
constructors are provided with identical field names and JSON keys.  Fields that a
PyTorchJob passes through untouched (volumes, tolerations, affinity, ...) are plain
dicts/lists.
"""
from .base import Model


class V1ObjectMeta(Model):
    _fields = [("annotations", "annotations", "dict(str, str)"),
               ("creation_timestamp", "creationTimestamp", "datetime"),
               ("deletion_timestamp", "deletionTimestamp", "datetime"),
               ("generate_name", "generateName", "str"),
               ("generation", "generation", "int"),
               ("labels", "labels", "dict(str, str)"),
               ("name", "name", "str"),
               ("namespace", "namespace", "str"),
               ("owner_references", "ownerReferences", "list[object]"),
               ("resource_version", "resourceVersion", "str"),
               ("uid", "uid", "str")]


class V1ListMeta(Model):
    _fields = [("_continue", "continue", "str"), ("resource_version", "resourceVersion", "str"),
               ("self_link", "selfLink", "str")]


class V1EnvVar(Model):
    _fields = [("name", "name", "str"), ("value", "value", "str"), ("value_from", "valueFrom", "object")]
    _required = ("name",)


class V1ContainerPort(Model):
    _fields = [("container_port", "containerPort", "int"), ("host_port", "hostPort", "int"),
               ("name", "name", "str"), ("protocol", "protocol", "str")]
    _required = ("container_port",)


class V1ResourceRequirements(Model):
    _fields = [("limits", "limits", "dict(str, object)"), ("requests", "requests", "dict(str, object)")]


class V1VolumeMount(Model):
    _fields = [("mount_path", "mountPath", "str"), ("name", "name", "str"), ("read_only", "readOnly", "bool")]


class V1Container(Model):
    _fields = [("args", "args", "list[str]"),
               ("command", "command", "list[str]"),
               ("env", "env", "list[V1EnvVar]"),
               ("image", "image", "str"),
               ("image_pull_policy", "imagePullPolicy", "str"),
               ("name", "name", "str"),
               ("ports", "ports", "list[V1ContainerPort]"),
               ("resources", "resources", "V1ResourceRequirements"),
               ("volume_mounts", "volumeMounts", "list[V1VolumeMount]"),
               ("working_dir", "workingDir", "str")]
    _required = ("name",)


class V1PodSpec(Model):
    _fields = [("affinity", "affinity", "object"),
               ("containers", "containers", "list[V1Container]"),
               ("host_ipc", "hostIPC", "bool"),
               ("init_containers", "initContainers", "list[V1Container]"),
               ("node_selector", "nodeSelector", "dict(str, str)"),
               ("restart_policy", "restartPolicy", "str"),
               ("scheduler_name", "schedulerName", "str"),
               ("service_account_name", "serviceAccountName", "str"),
               ("tolerations", "tolerations", "list[object]"),
               ("volumes", "volumes", "list[object]")]
    _required = ("containers",)


class V1PodTemplateSpec(Model):
    _fields = [("metadata", "metadata", "V1ObjectMeta"), ("spec", "spec", "V1PodSpec")]


class V1DeleteOptions(Model):
    _fields = [("api_version", "apiVersion", "str"), ("kind", "kind", "str"),
               ("grace_period_seconds", "gracePeriodSeconds", "int"),
               ("propagation_policy", "propagationPolicy", "str")]
