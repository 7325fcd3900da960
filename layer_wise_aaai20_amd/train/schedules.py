"""Progressive-resizing ImageNet schedules of the reference launcher (``IMAGENET/train.py:57-155``),
keyed by machine count. Each phase dict uses the reference keys: ``ep`` (epoch or (start, end)),
``sz`` image size, ``bs`` per-GPU batch, ``lr`` (value or (start, end) linear ramp), ``trndir``,
``min_scale``, ``rect_val``, ``keep_dl`` (change batch size, keep loader).

The reference launcher pickles the schedule into ``--phases`` but the worker ignores it (SURVEY.md
D14); here ``train_imagenet_nv.py --phases <name|json>`` honours it.
"""
from __future__ import annotations

import copy


def _one(lr=1.0):
    s224, s288 = 224 / 512, 128 / 512
    return [
        dict(ep=0, sz=128, bs=512, trndir="-sz/160"),
        dict(ep=(0, 5), lr=(lr, 2 * lr)),
        dict(ep=5, lr=lr),
        dict(ep=14, sz=224, bs=224, lr=lr * s224),
        dict(ep=16, lr=lr / 10 * s224),
        dict(ep=27, lr=lr / 100 * s224),
        dict(ep=32, sz=288, bs=128, min_scale=0.5, rect_val=True, lr=lr / 100 * s288),
        dict(ep=(33, 35), lr=lr / 1000 * s288),
    ]


def _two_or_four(lr):
    bs = [256, 224, 128]
    sc = [b / bs[0] for b in bs]
    return [
        dict(ep=0, sz=128, bs=bs[0], trndir="-sz/160"),
        dict(ep=(0, 6), lr=(lr, 2 * lr)),
        dict(ep=6, sz=128, bs=2 * bs[0], keep_dl=True),
        dict(ep=6, lr=2 * lr),
        dict(ep=(11, 13), lr=(2 * lr, lr)),
        dict(ep=13, sz=224, bs=bs[1], trndir="-sz/352", min_scale=0.087),
        dict(ep=13, lr=lr * sc[1]),
        dict(ep=(16, 23), lr=(lr * sc[1], lr / 10 * sc[1])),
        dict(ep=(23, 28), lr=(lr / 10 * sc[1], lr / 100 * sc[1])),
        dict(ep=28, sz=288, bs=bs[2], min_scale=0.5, rect_val=True),
        dict(ep=(28, 30), lr=(lr / 100 * sc[2], lr / 1000 * sc[2])),
    ]


def _eight(lr=0.235 * 8):
    s224 = 224 / 128
    return [
        dict(ep=0, sz=128, bs=128, trndir="-sz/160"),
        dict(ep=(0, 6), lr=(lr, 2 * lr)),
        dict(ep=6, bs=256, keep_dl=True, lr=2 * lr),
        dict(ep=(11, 14), lr=(2 * lr, lr)),
        dict(ep=14, sz=224, bs=128, trndir="-sz/352", min_scale=0.087, lr=lr),
        dict(ep=17, bs=224, keep_dl=True),
        dict(ep=(17, 23), lr=(lr, lr / 10 * s224)),
        dict(ep=(23, 29), lr=(lr / 10 * s224, lr / 100 * s224)),
        dict(ep=29, sz=288, bs=128, min_scale=0.5, rect_val=True),
        dict(ep=(29, 35), lr=(lr / 100, lr / 1000)),
    ]


def _sixteen(lr=0.235 * 8):
    return [
        dict(ep=0, sz=128, bs=64, trndir="-sz/160"),
        dict(ep=(0, 6), lr=(lr, 2 * lr)),
        dict(ep=6, bs=128, keep_dl=True),
        dict(ep=6, lr=2 * lr),
        dict(ep=16, sz=224, bs=64),
        dict(ep=16, lr=lr),
        dict(ep=19, bs=192, keep_dl=True),
        dict(ep=19, lr=2 * lr / (10 / 1.5)),
        dict(ep=31, lr=2 * lr / (100 / 1.5)),
        dict(ep=37, sz=288, bs=128, min_scale=0.5, rect_val=True),
        dict(ep=37, lr=2 * lr / 100),
        dict(ep=(38, 50), lr=2 * lr / 1000),
    ]


def _smoke():
    return [
        dict(ep=0, sz=64, bs=32),
        dict(ep=(0, 1), lr=(0.1, 0.2)),
        dict(ep=1, sz=96, bs=16, lr=0.05),
        dict(ep=2, sz=112, bs=8, rect_val=True, lr=0.01),
        dict(ep=(2, 3), lr=0.001),
    ]


_BUILDERS = {
    1: _one, 2: lambda: _two_or_four(0.75 * 2), 4: lambda: _two_or_four(0.50 * 4), 8: _eight,
    16: _sixteen,
}
NAMES = {"one_machine": 1, "two_machines": 2, "four_machines": 4, "eight_machines": 8,
         "sixteen_machines": 16}


def schedule(key) -> list:
    """``schedule(1)`` / ``schedule('one_machine')`` / ``schedule('smoke')`` → fresh phase list."""
    if key == "smoke":
        return _smoke()
    if isinstance(key, str):
        key = NAMES[key]
    return copy.deepcopy(_BUILDERS[int(key)]())


schedules = {k: schedule(k) for k in _BUILDERS}
