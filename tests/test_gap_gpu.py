"""Global average pool kernels (csrc/nn.hip k_gap_fwd / k_gap_bwd) against fp32 torch
``flatten(AdaptiveAvgPool2d(1)(x), 1)`` and its gradient (ResNet head,
``IMAGENET/training/resnet.py:141-142``)."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(256, 2048, 7, 7), (3, 512, 4, 4), (5, 64, 1, 1)])
@pytest.mark.parametrize("dy_dtype", [torch.bfloat16, torch.float32])
def test_gap_matches_torch(shape, dy_dtype):
    from layer_wise_aaai20_amd.ops.nn import global_avg_pool, _GlobalAvgPoolFn
    from layer_wise_aaai20_amd.ops._ext import load
    load()
    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = global_avg_pool(x, nn.AdaptiveAvgPool2d(1))
    assert y.grad_fn is not None and "_GlobalAvgPoolFn" in type(y.grad_fn).__name__
    xr = x.detach().float().requires_grad_(True)
    yr = torch.flatten(nn.AdaptiveAvgPool2d(1)(xr), 1)
    torch.testing.assert_close(y.float(), yr, atol=1e-2, rtol=1e-2)
    dy = torch.randn(y.shape, device="cuda", dtype=dy_dtype)
    (dx,) = torch.autograd.grad(y, x, dy.to(y.dtype) if dy_dtype == torch.bfloat16 else dy.to(y.dtype))
    (dxr,) = torch.autograd.grad(yr, xr, dy.to(y.dtype).float())
    assert dx.is_contiguous(memory_format=torch.channels_last) and dx.dtype == torch.bfloat16
    torch.testing.assert_close(dx.float(), dxr, atol=1e-3, rtol=1e-2)


def test_gap_bwd_fp32_dy_direct():
    from layer_wise_aaai20_amd.ops._ext import load
    lib = load()
    dy = torch.randn(4, 64, device="cuda")
    dx = lib.gap_bwd(dy, 3, 5)
    ref = (dy / 15).view(4, 64, 1, 1).expand(4, 64, 3, 5).to(torch.bfloat16)
    assert dx.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(dx, ref)
