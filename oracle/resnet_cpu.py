"""Plain PyTorch fp32 (CPU) restatement of torchvision ``resnet50`` minus ``fc`` -- ORACLE.

Test infrastructure only (see ``oracle/__init__.py``).

The reference's ``PretrainedBackboneDetector(backbone_name='resnet50')`` builds
``getattr(torchvision.models, 'resnet50')(pretrained=...)`` and keeps
``nn.Sequential(*list(backbone.children())[:-1])`` with ``feature_dim = backbone.fc.in_features``
(``src/pretrained_detector.py:37-40``); ``EnsembleDetector`` (``:146-218``) uses it as the
second member of the app's default ensemble (``ENSEMBLE_BACKBONES``, ``app.py:661,1597``).
torchvision is not installed here, so this restates its published architecture:

    conv1 7x7/2 pad 3 (3->64, no bias), bn1, relu, maxpool 3x3/2 pad 1,
    layer1..4 = 3, 4, 6, 3 Bottleneck blocks (planes 64, 128, 256, 512; expansion 4),
    avgpool AdaptiveAvgPool2d((1, 1)) -> (N, 2048, 1, 1)

Bottleneck ("ResNet v1.5", torchvision): conv1 1x1 -> bn1 -> relu -> conv2 3x3 (the block's
stride) -> bn2 -> relu -> conv3 1x1 (planes*4) -> bn3; identity = downsample(x) =
Sequential(conv 1x1/stride, bn) on the first block of each layer; out = relu(out + identity).
BatchNorm eps 1e-5, momentum 0.1.  Module names match torchvision, so the state_dict keys of
``children()[:-1]`` are ``0.weight`` (conv1), ``1.*`` (bn1), ``4.0.conv1.weight`` ... ``7.2.bn3.*``.
Parameter count: 23,508,032 (torchvision resnet50's 25,557,032 minus fc 2048*1000+1000).
Parity of the trunk numerics against torchvision itself is unpinned (not importable here).
"""
from __future__ import annotations

import torch
import torch.nn as nn

LAYERS = (3, 4, 6, 3)
PLANES = (64, 128, 256, 512)
EXPANSION = 4
FEATURE_DIM = 2048


class Bottleneck(nn.Module):
    expansion = EXPANSION

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * EXPANSION, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * EXPANSION)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


def make_layer(inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * EXPANSION:
        downsample = nn.Sequential(nn.Conv2d(inplanes, planes * EXPANSION, 1, stride=stride, bias=False),
                                   nn.BatchNorm2d(planes * EXPANSION))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * EXPANSION, planes))
    return nn.Sequential(*layers)


def resnet50_children():
    """The modules of ``torchvision.models.resnet50().children()`` without ``fc``, in order."""
    mods = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1)]
    inplanes = 64
    for i, (planes, blocks) in enumerate(zip(PLANES, LAYERS)):
        mods.append(make_layer(inplanes, planes, blocks, 1 if i == 0 else 2))
        inplanes = planes * EXPANSION
    mods.append(nn.AdaptiveAvgPool2d((1, 1)))
    return mods


class ResNet50TrunkCPU(nn.Sequential):
    """``nn.Sequential(*list(resnet50().children())[:-1])``: (N,3,H,W) -> (N,2048,1,1)."""

    def __init__(self):
        super().__init__(*resnet50_children())


def resnet_features(trunk: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """The detector's use of the trunk: features.view(N, -1) (pretrained_detector.py:116-118)."""
    return trunk(x).reshape(x.shape[0], -1)
