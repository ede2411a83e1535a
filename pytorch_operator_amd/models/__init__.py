"""Model definitions: the reference MNIST CNN (+ its fused HIP trainer)."""
from .mnist import Net, FusedMnistTrainer, PARAM_SPECS, NUM_PARAMS, reference_init  # noqa: F401
