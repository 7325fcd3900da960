"""The bf16 / fp16 builds of the kernel library and the precision switch (ops/_ext.py), checked
on the host: both libraries load (no GPU needed to register ops), the fp16 one registers the same
kernel ops under torch.ops.lwaaai16 but not the communicator, and set_half routes load() and h16().
The numerics of the fp16 kernels are pinned on the GPU by tests/test_fp16_gpu.py."""
import os

import pytest
import torch

from layer_wise_aaai20_amd.csrc import build as B
from layer_wise_aaai20_amd.ops import _ext


def _libs_built():
    return os.path.exists(_ext.SO_PATH) and os.path.exists(_ext.SO16_PATH)


def test_precision_switch_routes_dtype():
    assert _ext.h16() == torch.bfloat16 and not _ext.half()
    try:
        _ext.set_half(True)
        assert _ext.h16() == torch.float16 and _ext.half()
    finally:
        _ext.set_half(False)
    assert _ext.h16() == torch.bfloat16


def test_fp16_build_flags_and_sources():
    assert "-DLW_FP16" in B.FLAGS16 and "-DLW_OPS_NS=lwaaai16" in B.FLAGS16
    assert B.OUT16.endswith("_lwaaai16_C.so")
    # the same kernel sources, without the communicator (one RCCL state per process)
    srcs = [os.path.basename(s) for s in B.sources()]
    assert "rccl.cpp" in srcs and "gemm_core.h" not in srcs
    assert B._digest(B.sources()) != B._digest(B.sources(), B.FLAGS16)


@pytest.mark.skipif(not _libs_built(), reason="kernel libraries not built")
def test_both_libraries_register_their_ops():
    main = _ext.load_main(build_if_missing=False)
    try:
        _ext.set_half(True)
        half = _ext.load(build_if_missing=False)
    finally:
        _ext.set_half(False)
    assert half is torch.ops.lwaaai16 and main is torch.ops.lwaaai
    assert _ext.load(build_if_missing=False) is torch.ops.lwaaai
    for op in ("gemm_ex", "conv3_tap", "conv3_tap_wgrad", "bn_bwd", "normalize_u8"):
        assert hasattr(main, op) and hasattr(half, op), op
    assert hasattr(main, "rccl_init")
    with pytest.raises((AttributeError, RuntimeError)):
        getattr(half, "rccl_init")
