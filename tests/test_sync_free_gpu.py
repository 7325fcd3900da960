"""The compressed-gradient step never synchronises the host with the GPU: every method's
compress / exchange / decode path runs under ``torch.cuda.set_sync_debug_mode("error")`` (which
raises on any blocking device→host copy or synchronize). The threshold methods' data-dependent
counts go over the reference's dense wire by default for exactly this reason (a count exchange
would have to read the agreed capacity on the host in the middle of backward)."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP

pytestmark = pytest.mark.gpu

METHODS = [("Topk", {"K": 0.01}), ("Randomk", {"K": 0.05}), ("Thresholdv", {"V": 1e-3}),
           ("AdaptiveThreshold", {}), ("TernGrad", {}), ("RandomDithering", {"qstates": 255}),
           ("none", {})]


def _net():
    return nn.Sequential(nn.Conv2d(16, 32, 3, padding=1), nn.ReLU(), nn.Conv2d(32, 32, 3),
                         nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 16))


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("method,kw", METHODS, ids=[m for m, _ in METHODS])
def test_step_is_sync_free(method, kw, mode):
    torch.manual_seed(0)
    m = _net().cuda()
    ddp = CompressedDDP(m, compress=mode, method=method, error_feedback=method != "none",
                        bucket_cap_mb=0.01, flat_params=True, **kw)
    x = torch.randn(8, 16, 12, 12, device="cuda")
    y = torch.randint(0, 16, (8,), device="cuda")
    F.cross_entropy(ddp(x), y).backward()          # first step: allocations, workspaces
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(2):
            F.cross_entropy(ddp(x), y).backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())
