"""Container entrypoints run inside PyTorchJob replicas (MNIST DDP worker, smoke test)."""
