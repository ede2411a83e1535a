"""Small dependency-free utilities (TensorBoard writer, ...)."""
