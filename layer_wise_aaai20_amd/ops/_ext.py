"""Loader for the in-tree HIP extension (``layer_wise_aaai20_amd/_lwaaai_C.so``).

Policy: GPU tensors ALWAYS go through the HIP kernels. If the library is missing or fails to load
while a GPU is present, we try to build it in-tree once and otherwise raise — there is no silent
eager-PyTorch fallback for GPU tensors. CPU tensors (the gloo test path) use the pure-torch
implementations that mirror the kernels.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO_PATH = os.environ.get("LWAAAI_SO") or os.path.join(_PKG, "_lwaaai_C.so")
_lock = threading.Lock()
_loaded = False


class ExtensionMissing(RuntimeError):
    pass


def load(build_if_missing: bool = True):
    """Load (building first if needed) and return ``torch.ops.lwaaai``."""
    global _loaded
    if _loaded:
        return torch.ops.lwaaai
    with _lock:
        if _loaded:
            return torch.ops.lwaaai
        if not os.path.exists(SO_PATH) and build_if_missing:
            from ..csrc import build as _b
            _b.build(verbose=False)
        if not os.path.exists(SO_PATH):
            raise ExtensionMissing(
                f"{SO_PATH} not found; run `python -m layer_wise_aaai20_amd.csrc.build`")
        torch.ops.load_library(SO_PATH)
        _loaded = True
    return torch.ops.lwaaai


def ops_for(t: torch.Tensor):
    """Return torch.ops.lwaaai for GPU tensors (loud failure if unavailable), None for CPU."""
    if t.device.type == "cpu":
        return None
    return load()


def is_loaded() -> bool:
    return _loaded
