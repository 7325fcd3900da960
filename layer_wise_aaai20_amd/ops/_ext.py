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
# the same kernels built for fp16 (csrc/elem16.h, registered as torch.ops.lwaaai16)
SO16_PATH = os.environ.get("LWAAAI_SO16") or os.path.join(_PKG, "_lwaaai16_C.so")
_lock = threading.Lock()
_loaded = False
_loaded16 = False
_HALF = False


class ExtensionMissing(RuntimeError):
    pass


def _load_main(build_if_missing: bool = True):
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


def _load_half(build_if_missing: bool = True):
    global _loaded16
    if _loaded16:
        return torch.ops.lwaaai16
    _load_main(build_if_missing)              # the communicator and the shared state live there
    with _lock:
        if _loaded16:
            return torch.ops.lwaaai16
        if not os.path.exists(SO16_PATH) and build_if_missing:
            from ..csrc import build as _b
            _b.build(verbose=False)
        if not os.path.exists(SO16_PATH):
            raise ExtensionMissing(
                f"{SO16_PATH} not found; run `python -m layer_wise_aaai20_amd.csrc.build`")
        torch.ops.load_library(SO16_PATH)
        _loaded16 = True
    return torch.ops.lwaaai16


def load(build_if_missing: bool = True):
    """The kernel ops of the current precision: ``torch.ops.lwaaai`` (bf16 activations), or
    ``torch.ops.lwaaai16`` (the fp16 build of the same kernels) after ``set_half(True)``."""
    return _load_half(build_if_missing) if _HALF else _load_main(build_if_missing)


def load_main(build_if_missing: bool = True):
    """``torch.ops.lwaaai`` whatever the precision: the native communicator (csrc/rccl.cpp) is
    only built there, so its handles stay valid across ``set_half`` switches."""
    return _load_main(build_if_missing)


def set_half(on: bool) -> None:
    """Run the fused path's 16-bit tensors as fp16 (the reference's ``--fp16`` recipe on the MFMA
    kernels: v_mfma_f32_16x16x32_f16, fp32 accumulation, static loss scale in the SGD kernel)
    instead of bf16. Process-wide: set it before building a model."""
    global _HALF
    _HALF = bool(on)


def half() -> bool:
    return _HALF


def h16() -> torch.dtype:
    """The 16-bit element type of activations / weight mirrors on the fused path."""
    return torch.float16 if _HALF else torch.bfloat16


def ops_for(t: torch.Tensor):
    """Return torch.ops.lwaaai for GPU tensors (loud failure if unavailable), None for CPU."""
    if t.device.type == "cpu":
        return None
    return load()


def is_loaded() -> bool:
    return _loaded or _loaded16


# Deferred split-K reduces (csrc/gemm.hip splitk_flush; ops/block.py turns them on around a
# block's arena weight gradients). _DEFER holds a tensor on the deferring device while on.
_DEFER = [None]


def set_splitk_defer(t: torch.Tensor, on: bool) -> None:
    load().splitk_defer(t, on)
    _DEFER[0] = t if on else None


def splitk_discard(dev: torch.Tensor) -> int:
    """Drop the queued split-K reduces and their slabs without launching anything (a step that
    failed between a deferred weight-gradient GEMM and the engine's flush: the capture that fell
    back to eager, a backward that raised). Returns how many were dropped."""
    _DEFER[0] = None
    if not is_loaded():
        return 0
    return int(load().splitk_discard(dev))


def splitk_pending() -> int:
    """Split-K reduces queued and not yet flushed (0 between steps)."""
    if not is_loaded():
        return 0
    return int(load().splitk_pending())


class splitk_paused:
    """Reduce split-K outputs right away inside this scope (the tuner's timing runs: a
    deferred reduce would neither be timed nor target a real gradient)."""

    def __enter__(self):
        self.t = _DEFER[0]
        if self.t is not None:
            set_splitk_defer(self.t, False)
        return self

    def __exit__(self, *exc):
        if self.t is not None:
            set_splitk_defer(self.t, True)
        return False
