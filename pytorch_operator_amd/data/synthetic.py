"""A learnable synthetic stand-in for MNIST, resident in HBM.

The reference downloads MNIST (examples/mnist/mnist.py:119-131); this framework runs
without network, so it generates a dataset of the same shape and dtype: 28x28 uint8
images, int32 labels in [0,10).  Each class has a smooth random "stroke" template;
samples are the template with a random sub-pixel jitter, contrast and noise, so the
CNN must actually learn (accuracy climbs from 10% to >95% within an epoch).

The dataset stays on the device: a 60 000-image epoch is 47 MB of the 288 GB HBM3E,
and the per-epoch shuffle (``DataLoader(shuffle=True)``) is a device ``randperm``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F


@dataclass
class SyntheticMnist:
    images: torch.Tensor   # [n, 784] uint8
    labels: torch.Tensor   # [n] int32
    perm: torch.Tensor     # [n] int32 (current epoch order)
    seed: int

    @property
    def n(self) -> int:
        return self.images.shape[0]

    def reshuffle(self, epoch: int) -> None:
        g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + epoch)
        self.perm.copy_(torch.randperm(self.n, generator=g).to(torch.int32).to(self.perm.device))

    def float_images(self) -> torch.Tensor:
        """Normalised fp32 [n,1,28,28] (what ToTensor+Normalize would give)."""
        return ((self.images.float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)


def _templates(gen: torch.Generator) -> torch.Tensor:
    # 10 classes x 28x28: sums of a few random gaussian strokes, smoothed
    yy, xx = torch.meshgrid(torch.arange(28.0), torch.arange(28.0), indexing="ij")
    t = torch.zeros(10, 28, 28)
    for c in range(10):
        for _ in range(4):
            cy, cx = (torch.rand(2, generator=gen) * 16 + 6).tolist()
            sy, sx = (torch.rand(2, generator=gen) * 4 + 1.5).tolist()
            t[c] += torch.exp(-(((yy - cy) / sy) ** 2 + ((xx - cx) / sx) ** 2))
    t = t / t.amax(dim=(1, 2), keepdim=True)
    return t


def make_synthetic_mnist(n: int = 60000, seed: int = 1, device: Optional[torch.device] = None,
                         noise: float = 0.35, on_device: bool = False) -> SyntheticMnist:
    """``n`` images + labels (+ the epoch-0 permutation), moved to ``device``.

    ``on_device`` (a GPU ``device``): the same recipe drawn by one HIP kernel of this
    framework (``ops.mnist.synth_mnist``: counter-hash random numbers, bilinear warp) in ~1 ms
    instead of ~2 s of single-threaded CPU warps -- the worker's start-up path
    (harness/mnist.py).  A different random stream than the CPU recipe, so a different (equally
    learnable) dataset; every rank with the same seed draws the same one.
    """
    tmpl = _templates(torch.Generator(device="cpu").manual_seed(12345))
    if on_device and device is not None and torch.device(device).type == "cuda":
        from ..ops import mnist as K
        images, labels = K.synth_mnist(tmpl.to(device), n, seed, noise)
        ds = SyntheticMnist(images, labels, torch.empty(n, dtype=torch.int32, device=device), seed)
        ds.reshuffle(0)
        return ds
    gen = torch.Generator(device="cpu").manual_seed(seed)
    labels = torch.randint(0, 10, (n,), generator=gen)
    out = torch.empty(n, 784, dtype=torch.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        lab = labels[s:s + chunk]
        m = lab.numel()
        base = tmpl[lab].unsqueeze(1)  # [m,1,28,28]
        theta = torch.zeros(m, 2, 3)
        scale = 1.0 + (torch.rand(m, generator=gen) - 0.5) * 0.2
        theta[:, 0, 0] = scale
        theta[:, 1, 1] = scale
        theta[:, :, 2] = (torch.rand(m, 2, generator=gen) - 0.5) * 0.25
        grid = F.affine_grid(theta, (m, 1, 28, 28), align_corners=False)
        img = F.grid_sample(base, grid, align_corners=False).squeeze(1)
        img = img * (0.6 + 0.4 * torch.rand(m, 1, 1, generator=gen))
        img = img + noise * torch.rand(m, 28, 28, generator=gen) ** 3
        out[s:s + chunk] = (img.clamp(0, 1) * 255).round().to(torch.uint8).view(m, 784)
    ds = SyntheticMnist(out, labels.to(torch.int32), torch.empty(n, dtype=torch.int32), seed)
    ds.reshuffle(0)
    if device is not None:
        ds.images = ds.images.to(device)
        ds.labels = ds.labels.to(device)
        ds.perm = ds.perm.to(device)
    return ds
