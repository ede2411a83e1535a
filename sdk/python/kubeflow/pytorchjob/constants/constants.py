"""PyTorchJob SDK constants (reference sdk/python/kubeflow/pytorchjob/constants/constants.py)."""
import os

PYTORCHJOB_GROUP = "kubeflow.org"
PYTORCHJOB_KIND = "PyTorchJob"
PYTORCHJOB_PLURAL = "pytorchjobs"
PYTORCHJOB_VERSION = os.environ.get("PYTORCHJOB_VERSION", "v1")

PYTORCH_LOGLEVEL = os.environ.get("PYTORCHJOB_LOGLEVEL", "INFO").upper()

# seconds to wait for a request to the API server
APISERVER_TIMEOUT = 120

# labels the operator puts on every pod/service (pkg/controller.v1/pytorch/*.go)
PYTORCHJOB_CONTROLLER_LABEL = "controller-name"
PYTORCHJOB_GROUP_LABEL = "group-name"
PYTORCHJOB_NAME_LABEL = "pytorch-job-name"
PYTORCHJOB_TYPE_LABEL = "pytorch-replica-type"
PYTORCHJOB_INDEX_LABEL = "pytorch-replica-index"
PYTORCHJOB_ROLE_LABEL = "job-role"

# MI355X: the AMD device plugin's extended resource and the collective backend name
AMD_GPU_RESOURCE = "amd.com/gpu"
RCCL_BACKEND = "nccl"  # torch.distributed's "nccl" backend is RCCL on ROCm
