from kubeflow.pytorchjob.api.py_torch_job_client import PyTorchJobClient  # noqa: F401
