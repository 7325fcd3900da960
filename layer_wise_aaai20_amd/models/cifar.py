"""CIFAR-10 models of the reference: ResNet-9 (DAWNBench / myrtle.ai net), AlexNet in two flavours
and VGG-16. Parameter names and shapes match the reference definitions, so state_dicts and the
per-layer message list that drives layer-wise compression are identical.

* ``resnet9`` / ``alexnet`` graph builders — ``CIFAR10/dawn.py:22-87``
* ``AlexNet`` (classic nn.Module, ``--network Alexnet1``) — ``CIFAR10/alexnet.py:11-57``
* ``VGG`` / ``vgg16`` (VGG-D without BN, AdaptiveAvgPool 7x7) — ``CIFAR10/vgg16.py:10-94``
"""
from __future__ import annotations


import torch
from torch import nn

from .graph import (Add, Correct, Flatten, Identity, Mul, Network, batch_norm, rel_path, union)


# ----------------------------------------------------------------------------- graph builders
def conv_bn(c_in, c_out, bn_weight_init=1.0, stride=1, **kw):
    return {
        "conv": nn.Conv2d(c_in, c_out, kernel_size=3, stride=stride, padding=1, bias=False),
        "bn": batch_norm(c_out, bn_weight_init=bn_weight_init, **kw),
        "relu": nn.ReLU(True),
    }


def conv_bn_stride(c_in, c_out, bn_weight_init=1.0, **kw):
    return conv_bn(c_in, c_out, bn_weight_init, stride=2, **kw)


def residual(c, **kw):
    return {
        "in": Identity(),
        "res1": conv_bn(c, c, **kw),
        "res2": conv_bn(c, c, **kw),
        "add": (Add(), [rel_path("in"), rel_path("res2", "relu")]),
    }


def basic_resnet9(channels, weight, pool, **kw):
    net = {"prep": conv_bn(3, channels["prep"], **kw)}
    prev = channels["prep"]
    for name in ("layer1", "layer2", "layer3"):
        net[name] = dict(conv_bn(prev, channels[name], **kw), pool=pool)
        prev = channels[name]
    net.update(pool=nn.MaxPool2d(4), flatten=Flatten(),
               linear=nn.Linear(prev, 10, bias=False), classifier=Mul(weight))
    return net


def basic_alexnet(channels, weight, pool, **kw):
    net = {
        "prep": dict(conv_bn_stride(3, channels["prep"], **kw), pool=pool),
        "layer1": dict(conv_bn(channels["prep"], channels["layer1"], **kw), pool=pool),
        "layer2": conv_bn(channels["layer1"], channels["layer2"], **kw),
        "layer3": conv_bn(channels["layer2"], channels["layer3"], **kw),
        "layer4": dict(conv_bn(channels["layer3"], channels["layer4"], **kw), pool=pool),
    }
    net.update(pool=nn.MaxPool2d(2), flatten=Flatten(),
               linear=nn.Linear(channels["layer4"], 10, bias=False), classifier=Mul(weight))
    return net


def resnet9(channels=None, weight=0.125, pool=None, extra_layers=(),
            res_layers=("layer1", "layer3"), **kw):
    channels = channels or {"prep": 64, "layer1": 128, "layer2": 256, "layer3": 512}
    pool = pool if pool is not None else nn.MaxPool2d(2)
    n = basic_resnet9(channels, weight, pool, **kw)
    for layer in res_layers:
        n[layer]["residual"] = residual(channels[layer], **kw)
    for layer in extra_layers:
        n[layer]["extra"] = conv_bn(channels[layer], channels[layer], **kw)
    return n


def alexnet(channels=None, weight=0.125, pool=None, extra_layers=(), **kw):
    channels = channels or {"prep": 64, "layer1": 192, "layer2": 384, "layer3": 256, "layer4": 256}
    pool = pool if pool is not None else nn.MaxPool2d(2)
    return basic_alexnet(channels, weight, pool, **kw)


def make_losses():
    return {
        "loss": (nn.CrossEntropyLoss(reduction="none"), [("classifier",), ("target",)]),
        "correct": (Correct(), [("classifier",), ("target",)]),
    }


losses = make_losses()


# ----------------------------------------------------------------------------- nn.Module models
class _DictLossMixin:
    """forward(dict(input, target)) -> {'loss': per-sample CE, 'correct': bool} like the graph
    networks, so ``run_batches`` treats every CIFAR model alike."""

    def _heads(self):
        self.loss = (nn.CrossEntropyLoss(reduction="none"), Correct())

    def _out(self, logits, target):
        return {"loss": self.loss[0](logits, target), "correct": self.loss[1](logits, target),
                "classifier": logits}


class AlexNet(nn.Module, _DictLossMixin):
    # (out_channels, stride, pool_after) — indices reproduce features.{0,3,6,8,10}
    SPEC = ((64, 2, True), (192, 1, True), (384, 1, False), (256, 1, False), (256, 1, True))

    def __init__(self, num_classes: int = 10):
        super().__init__()
        layers, c = [], 3
        for out, stride, pool in self.SPEC:
            layers += [nn.Conv2d(c, out, kernel_size=3, stride=stride, padding=1),
                       nn.ReLU(inplace=True)]
            if pool:
                layers.append(nn.MaxPool2d(kernel_size=2))
            c = out
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(256 * 2 * 2, 4096), nn.ReLU(inplace=True),
            nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes))
        self._heads()

    def forward(self, batch):
        x = self.features(batch["input"])
        x = self.classifier(x.reshape(x.size(0), 256 * 2 * 2))
        return self._out(x, batch["target"])


VGG_CFGS = {
    "A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "B": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512,
          512, 512, "M"],
}
cfgs = VGG_CFGS


def make_layers(cfg, batch_norm: bool = False) -> nn.Sequential:
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        layers.append(nn.Conv2d(c, v, kernel_size=3, padding=1))
        if batch_norm:
            layers.append(nn.BatchNorm2d(v))
        layers.append(nn.ReLU(inplace=True))
        c = v
    return nn.Sequential(*layers)


_VGG_FOLD = True          # (False, tests only: the pool + full-width GEMMs)


def _pair_size(s):
    return (s, s) if isinstance(s, int) else tuple(s)


class VGG(nn.Module, _DictLossMixin):
    def __init__(self, features: nn.Module, num_classes: int = 10, init_weights: bool = True):
        super().__init__()
        self.features = features
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(True), nn.Dropout(),
            nn.Linear(4096, num_classes))
        self._heads()
        if init_weights:
            for m in self.modules():
                if isinstance(m, nn.Conv2d):
                    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                    if m.bias is not None:
                        nn.init.zeros_(m.bias)
                elif isinstance(m, nn.BatchNorm2d):
                    nn.init.ones_(m.weight)
                    nn.init.zeros_(m.bias)
                elif isinstance(m, nn.Linear):
                    nn.init.normal_(m.weight, 0, 0.01)
                    nn.init.zeros_(m.bias)

    def forward(self, batch):
        x = self.features(batch["input"])
        fc1 = self.classifier[0]
        oh, ow = _pair_size(self.avgpool.output_size)
        if (x.is_cuda and x.shape[-2:] == (1, 1) and hasattr(fc1, "fuse_relu") and
                fc1.in_features == x.shape[1] * oh * ow and _VGG_FOLD):
            # 32x32 CIFAR images leave a 1x1 map, which the 7x7 adaptive pool only replicates:
            # fc1 runs on the folded weight (ops/gemm.py replicated_linear, exactly the same
            # layer).
            from ..ops.gemm import replicated_linear
            x = replicated_linear(torch.flatten(x, 1), fc1, oh * ow)
            x = self.classifier[1:](x)
        else:
            x = self.avgpool(x)
            x = self.classifier(torch.flatten(x, 1))
        return self._out(x, batch["target"])


def vgg(cfg: str = "D", batch_norm: bool = False, **kw) -> VGG:
    return VGG(make_layers(VGG_CFGS[cfg], batch_norm=batch_norm), **kw)


def vgg16(**kw) -> VGG:
    """VGG-16 (config D, no BN). Built on demand (the reference instantiates it at import time,
    ``vgg16.py:94``)."""
    return vgg("D", False, **kw)


NETWORKS = {
    "resnet9": lambda: Network(union(resnet9(), make_losses())),
    "alexnet": lambda: Network(union(alexnet(), make_losses())),
    "alexnet1": AlexNet,
    "vgg16": vgg16,
}
# reference spellings (dawn.py:115-122; D6: the default 'resnet9' matched no branch)
NETWORK_ALIASES = {"Resent9": "resnet9", "ResNet9": "resnet9", "Resnet9": "resnet9",
                   "Alexnet": "alexnet", "AlexNet": "alexnet", "Alexnet1": "alexnet1",
                   "AlexNet1": "alexnet1", "VGG16": "vgg16", "vgg": "vgg16"}


def build_network(name: str) -> nn.Module:
    key = NETWORK_ALIASES.get(name, name)
    if key not in NETWORKS:
        raise ValueError(f"unknown network {name!r}; expected one of {sorted(NETWORKS)} or "
                         f"{sorted(NETWORK_ALIASES)}")
    return NETWORKS[key]()
