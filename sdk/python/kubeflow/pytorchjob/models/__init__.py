from kubeflow.pytorchjob.models.k8s import (V1Container, V1ContainerPort, V1DeleteOptions, V1EnvVar,  # noqa: F401
                                            V1ListMeta, V1ObjectMeta, V1PodSpec, V1PodTemplateSpec,
                                            V1ResourceRequirements, V1VolumeMount)
from kubeflow.pytorchjob.models.v1_job_condition import V1JobCondition  # noqa: F401
from kubeflow.pytorchjob.models.v1_job_status import V1JobStatus  # noqa: F401
from kubeflow.pytorchjob.models.v1_py_torch_job import V1PyTorchJob  # noqa: F401
from kubeflow.pytorchjob.models.v1_py_torch_job_list import V1PyTorchJobList  # noqa: F401
from kubeflow.pytorchjob.models.v1_py_torch_job_spec import V1PyTorchJobSpec  # noqa: F401
from kubeflow.pytorchjob.models.v1_replica_spec import V1ReplicaSpec  # noqa: F401
from kubeflow.pytorchjob.models.v1_replica_status import V1ReplicaStatus  # noqa: F401
from kubeflow.pytorchjob.models.v1_time import V1Time  # noqa: F401
