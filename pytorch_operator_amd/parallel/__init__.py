"""Distributed data parallelism over RCCL/xGMI (``nccl`` backend on ROCm)."""
from .dist import DistEnv, init_from_env, backend_for, is_distributed  # noqa: F401
from .ddp import FlatGradAllReduce, BucketedDDP  # noqa: F401
