"""SDK helpers (reference sdk/python/kubeflow/pytorchjob/utils/utils.py)."""
import os

from kubeflow.pytorchjob.constants import constants

_SA_DIR = "/var/run/secrets/kubernetes.io/"


def is_running_in_k8s():
    return os.path.isdir(_SA_DIR)


def get_current_k8s_namespace():
    with open(os.path.join(_SA_DIR, "serviceaccount", "namespace")) as f:
        return f.readline().strip()


def get_default_target_namespace():
    if not is_running_in_k8s():
        return "default"
    return get_current_k8s_namespace()


def set_pytorchjob_namespace(pytorchjob):
    """Namespace of a V1PyTorchJob (or plain dict), else the default target namespace."""
    if isinstance(pytorchjob, dict):
        ns = (pytorchjob.get("metadata") or {}).get("namespace")
    else:
        md = getattr(pytorchjob, "metadata", None)
        ns = md.get("namespace") if isinstance(md, dict) else getattr(md, "namespace", None)
    return ns or get_default_target_namespace()


def get_labels(name, master=False, replica_type=None, replica_index=None):
    """Selector labels of a job's pods (optionally only the master / a type / an index)."""
    labels = {
        constants.PYTORCHJOB_GROUP_LABEL: "kubeflow.org",
        constants.PYTORCHJOB_CONTROLLER_LABEL: "pytorch-operator",
        constants.PYTORCHJOB_NAME_LABEL: name,
    }
    if master:
        labels[constants.PYTORCHJOB_ROLE_LABEL] = "master"
    if replica_type:
        labels[constants.PYTORCHJOB_TYPE_LABEL] = str.lower(replica_type)
    if replica_index is not None:
        # the reference drops index 0 (`if replica_index:`); 0 is a valid index here
        labels[constants.PYTORCHJOB_INDEX_LABEL] = str(replica_index)
    return labels


def to_selector(labels):
    return ",".join("{0}={1}".format(k, v) for k, v in labels.items())
