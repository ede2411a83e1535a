"""Hand-written gfx950 HIP kernels (csrc/kernels) and their Python bindings."""
from ._native import build, load, library_path, NativeLibraryError  # noqa: F401
