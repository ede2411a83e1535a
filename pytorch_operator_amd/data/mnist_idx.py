"""Reader for the MNIST IDX files (the format torchvision's ``datasets.MNIST`` downloads).

The reference worker calls ``datasets.MNIST('../data', download=True)``
(examples/mnist/mnist.py:119-131).  There is no network here and torchvision is not
installed, so the worker looks for already-present IDX files (plain or ``.gz``, flat or
in torchvision's ``MNIST/raw`` layout) and otherwise falls back to the synthetic set.
Images stay uint8: normalisation ``(x/255 - 0.1307)/0.3081`` happens inside the first
HIP kernel, so the HBM-resident dataset is 4x smaller than a float copy.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Optional, Tuple

import numpy as np
import torch

_FILES = {
    "train": ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    "test": ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}


def _open(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    with _open(path) as f:
        data = f.read()
    zero, dtype_code, ndim = struct.unpack_from(">HBB", data, 0)
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    dims = struct.unpack_from(">" + "I" * ndim, data, 4)
    off = 4 + 4 * ndim
    arr = np.frombuffer(data, dtype=np.uint8, count=int(np.prod(dims)), offset=off)
    return arr.reshape(dims)


def _find(root: str, stem: str) -> Optional[str]:
    for d in (root, os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw")):
        for suffix in ("", ".gz"):
            p = os.path.join(d, stem + suffix)
            if os.path.exists(p):
                return p
    return None


def load_mnist(root: str, split: str = "train") -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """(uint8 [n,784], int32 [n]) or None when the files are not present."""
    img_stem, lab_stem = _FILES[split]
    ip, lp = _find(root, img_stem), _find(root, lab_stem)
    if ip is None or lp is None:
        return None
    x = read_idx(ip)
    y = read_idx(lp)
    if x.shape[0] != y.shape[0] or x.shape[1:] != (28, 28):
        raise ValueError(f"unexpected MNIST shapes {x.shape} / {y.shape}")
    return (torch.from_numpy(x.reshape(-1, 784).copy()),
            torch.from_numpy(y.astype(np.int32)))


def write_idx(path: str, arr: np.ndarray) -> None:
    """Write a uint8 IDX file (used by tests to fabricate a tiny MNIST directory)."""
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    head = struct.pack(">HBB", 0, 0x08, arr.ndim) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(head + arr.tobytes())
