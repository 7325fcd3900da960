"""``CIFAR10.vgg16`` (reference ``CIFAR10/vgg16.py``). ``vgg16model`` is built lazily on first
access instead of at import time (the reference allocates 134 M parameters on import)."""
from layer_wise_aaai20_amd.models.cifar import VGG, cfgs, make_layers, vgg, vgg16  # noqa


def _vgg(arch, cfg, batch_norm, pretrained=False, progress=True, **kwargs):
    if pretrained:
        raise RuntimeError("pretrained weights need network access; not available offline")
    return vgg(cfg, batch_norm, **kwargs)


def __getattr__(name):
    if name == "vgg16model":
        m = vgg16()
        globals()["vgg16model"] = m
        return m
    raise AttributeError(name)
