"""Synthetic, device-resident datasets (no network: BASELINE.json data='synthetic')."""
from .synthetic import SyntheticMnist, make_synthetic_mnist  # noqa: F401
