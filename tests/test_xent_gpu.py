"""Fused softmax cross-entropy + top-1/top-5 kernel (csrc/nn.hip k_xent) vs fp32 torch."""
import pytest
import torch
import torch.nn.functional as F

from layer_wise_aaai20_amd.ops.nn import FusedCrossEntropyLoss, fused_cross_entropy


def _ref_correct(logits, target):
    top = logits.topk(min(5, logits.shape[1]), 1).indices
    ok = top.eq(target.view(-1, 1))
    return torch.stack([ok[:, 0].float(), ok.any(1).float()], 1)


def test_xent_cpu_fallback():
    torch.manual_seed(0)
    x = torch.randn(16, 10, requires_grad=True)
    t = torch.randint(0, 10, (16,))
    loss, corr = fused_cross_entropy(x, t)
    torch.testing.assert_close(loss, F.cross_entropy(x, t))
    torch.testing.assert_close(corr, _ref_correct(x, t))


@pytest.mark.gpu
@pytest.mark.parametrize("B,C", [(256, 1000), (512, 10), (7, 3000), (64, 2048), (33, 5)])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_xent_matches_torch(B, C, reduction):
    torch.manual_seed(B + C)
    x = (torch.randn(B, C, device="cuda") * 3).requires_grad_()
    t = torch.randint(0, C, (B,), device="cuda")
    loss, corr = fused_cross_entropy(x, t, reduction=reduction)
    xr = x.detach().clone().requires_grad_()
    lr = F.cross_entropy(xr, t, reduction=reduction)
    torch.testing.assert_close(loss, lr, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(corr, _ref_correct(xr.detach(), t))
    g = torch.randn_like(lr)
    loss.backward(g)
    lr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-5, rtol=1e-4)


@pytest.mark.gpu
def test_xent_ignore_index_and_module():
    torch.manual_seed(3)
    x = torch.randn(64, 100, device="cuda", requires_grad=True)
    t = torch.randint(0, 100, (64,), device="cuda")
    t[::7] = -100
    crit = FusedCrossEntropyLoss()
    loss = crit(x, t)
    xr = x.detach().clone().requires_grad_()
    lr = F.cross_entropy(xr, t)
    torch.testing.assert_close(loss, lr, atol=1e-5, rtol=1e-5)
    loss.backward()
    lr.backward()
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-6, rtol=1e-4)
    assert crit.last_correct.shape == (64, 2)
    assert float(crit.last_correct[::7].sum()) == 0.0
