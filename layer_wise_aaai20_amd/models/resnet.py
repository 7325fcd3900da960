"""ImageNet ResNet family (v1, stride on the 3x3 conv), parameter-name compatible with
``IMAGENET/training/resnet.py`` / torchvision so checkpoints load unchanged.

``bn0=True`` applies the large-batch init of ``init_dist_weights`` (``resnet.py:154-160``): the last
BN gamma of every residual block starts at zero and the classifier at N(0, 0.01).

MI355X notes: models are meant to run ``channels_last`` in bf16 autocast (NHWC is the layout the
MFMA implicit-GEMM convolutions want); the residual join ``out += identity; relu`` goes through the
fused HIP kernel of :mod:`layer_wise_aaai20_amd.ops.nn` when ``fused=True``.
"""
from __future__ import annotations

import torch
from torch import nn

__all__ = ["ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50", "resnet101",
           "resnet152", "init_dist_weights"]


def conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes: int = 1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def init_dist_weights(model: nn.Module) -> None:
    """Goyal et al. large-batch init (``resnet.py:154-160``)."""
    for m in model.modules():
        if isinstance(m, BasicBlock):
            m.bn2.weight = nn.Parameter(torch.zeros_like(m.bn2.weight))
        if isinstance(m, Bottleneck):
            m.bn3.weight = nn.Parameter(torch.zeros_like(m.bn3.weight))
        if isinstance(m, nn.Linear):
            m.weight.data.normal_(0, 0.01)


def _make(block, layers, bn0=False, pretrained=False, **kw):
    if pretrained:
        raise RuntimeError("pretrained weights need network access; not available offline")
    m = ResNet(block, layers, **kw)
    if bn0:
        init_dist_weights(m)
    return m


def resnet18(pretrained=False, bn0=False, **kw):
    return _make(BasicBlock, [2, 2, 2, 2], bn0, pretrained, **kw)


def resnet34(pretrained=False, bn0=False, **kw):
    return _make(BasicBlock, [3, 4, 6, 3], bn0, pretrained, **kw)


def resnet50(pretrained=False, bn0=False, **kw):
    return _make(Bottleneck, [3, 4, 6, 3], bn0, pretrained, **kw)


def resnet101(pretrained=False, bn0=False, **kw):
    return _make(Bottleneck, [3, 4, 23, 3], bn0, pretrained, **kw)


def resnet152(pretrained=False, bn0=False, **kw):
    return _make(Bottleneck, [3, 8, 36, 3], bn0, pretrained, **kw)
