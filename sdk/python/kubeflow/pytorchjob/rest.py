"""REST transport + ApiException (kubernetes.client.rest equivalents)."""
from pytorch_operator_amd.cluster.rest import ApiException, KubeRest  # noqa: F401
