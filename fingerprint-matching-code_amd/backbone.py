"""ResNet-18 image backbone of ``Net`` (``src/model/feature_extractor.py:7-75``, ``ResNet18_final``).

The reference splits torchvision's resnet18 into ``node_layers`` (conv1 .. layer3, stride 16,
256 channels), ``edge_layers`` (layer4, stride 32, 512 channels) and ``final_layers``
(AdaptiveMaxPool2d(1)).  The convolutions are plain library convolutions (MIOpen through
``torch.nn.Conv2d``, channels_last), as SURVEY §8f rank 2 plans; what follows the backbone —
channel L2-normalisation, bilinear ``feature_align`` of both maps at the keypoints, the
[U || F] concatenation and the global max-pool — is one HIP kernel set
(``csrc/frontend.hip``, ``fpm_feature_align_fwd``).

Module and parameter names follow torchvision's ``resnet18`` inside those ``nn.Sequential``s
(``node_layers.0.weight`` = conv1, ``node_layers.4.0.conv1.weight`` = layer1[0].conv1, ...,
``edge_layers.0.1.bn2.running_var``), so a reference checkpoint's backbone loads by name.
There is no network: weights are a seeded random init in torchvision's scheme (Kaiming-normal
fan_out convs, BN weight 1 / bias 0), not ImageNet.
"""
import math

import torch
import torch.nn as nn


class BasicBlock(nn.Module):
    """torchvision ``BasicBlock`` (expansion 1)."""

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


def _layer(inplanes, planes, stride):
    ds = None
    if stride != 1 or inplanes != planes:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    return nn.Sequential(BasicBlock(inplanes, planes, stride, ds), BasicBlock(planes, planes))


def build_resnet18_split(seed=0):
    """(node_layers, edge_layers, final_layers) with torchvision's layout and a seeded init."""
    gen = torch.Generator().manual_seed(int(seed))
    node_layers = nn.Sequential(
        nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
        nn.MaxPool2d(3, 2, 1),
        _layer(64, 64, 1), _layer(64, 128, 2), _layer(128, 256, 2))
    edge_layers = nn.Sequential(_layer(256, 512, 2))
    final_layers = nn.Sequential(nn.AdaptiveMaxPool2d((1, 1)))
    for m in list(node_layers.modules()) + list(edge_layers.modules()):
        if isinstance(m, nn.Conv2d):
            fan_out = m.out_channels * m.kernel_size[0] * m.kernel_size[1]
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=gen) * math.sqrt(2.0 / fan_out))
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
    return node_layers, edge_layers, final_layers


def backbone_state_dict(seed=0):
    """State dict (reference names) of the seeded backbone, e.g. for oracle comparisons."""
    nl, el, fl = build_resnet18_split(seed)
    sd = {}
    for pre, mod in (("node_layers", nl), ("edge_layers", el)):
        for k, v in mod.state_dict().items():
            sd[pre + "." + k] = v
    return sd
