"""Client configuration (host, bearer token, TLS).  Same object the REST layer uses."""
from pytorch_operator_amd.cluster.rest import Configuration  # noqa: F401
