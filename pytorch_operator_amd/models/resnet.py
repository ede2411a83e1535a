"""ResNet-50 for the BASELINE "ResNet-50 DDP bf16" PyTorchJob config.

Not part of the reference (its only workload is MNIST); BASELINE.json lists it as a
north-star job shape: Master=1 Worker=7, one ``amd.com/gpu`` each, bf16.  The network is
the standard torchvision-style ResNet-50 v1.5 (stride on the 3x3 conv of each
bottleneck), written out here because torchvision is not in this image.  On MI355X it
runs channels-last under bf16 autocast: convolutions go to MIOpen, the classifier GEMM to
hipBLASLt -- plain library kernels, as the MI355X guidance prescribes for non-fused work.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, layers: List[int] = (3, 4, 6, 3), num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.inplanes = width
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(width, layers[0])
        self.layer2 = self._make(width * 2, layers[1], stride=2)
        self.layer3 = self._make(width * 4, layers[2], stride=2)
        self.layer4 = self._make(width * 8, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(width * 8 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():  # zero-init the last BN of each block (standard trick)
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.bn3.weight)

    def _make(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        down = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * Bottleneck.expansion))
        layers = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * Bottleneck.expansion
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Same topology family, small enough for CPU tests."""
    return ResNet((1, 1, 1, 1), num_classes, width=8)
