"""Small dependency-free utilities (TensorBoard writer, pformat / rand_string)."""
from .misc import pformat, rand_string  # noqa: F401
