"""Python SDK for the MI355X-native PyTorchJob operator.

API-compatible with the reference SDK (sdk/python/kubeflow/pytorchjob): the same
``PyTorchJobClient`` methods and V1* models, over a stdlib REST client instead of the
``kubernetes`` package.
"""
from kubeflow.pytorchjob.utils import utils  # noqa: F401
from kubeflow.pytorchjob.constants import constants  # noqa: F401

from kubeflow.pytorchjob.api_client import ApiClient  # noqa: F401
from kubeflow.pytorchjob.configuration import Configuration  # noqa: F401
from kubeflow.pytorchjob.api.py_torch_job_client import PyTorchJobClient  # noqa: F401

from kubeflow.pytorchjob.models import *  # noqa: F401,F403
