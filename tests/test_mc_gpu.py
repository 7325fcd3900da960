"""Momentum correction (DGC) fused into the compressor kernels:

* the per-bucket prologue g' = g + wd·p/grad_scale, u = mc·u + g', g = u runs inside the first
  pass of the Top-K chain for layer-wise buckets (csrc/compress.hip McArgs in k_hist pass 0 /
  k_small_select; one kernel, csrc/optim.hip k_mc_prep, otherwise) and the momentum factor
  masking (u = 0 at the sent coordinates of tensors not sent whole) inside the select kernels
  (k_small_select / k_write) — the decoded gradient, the residual and the velocity equal the CPU
  mirror (parallel/engine.py, codecs.py) bit for bit, step after step;
* the engine's step issues no ATen elementwise kernel for it (the four ATen passes it replaces:
  u.mul_().add_(), g.copy_(u), u.mul_(e != 0));
* codecs without a selection (QSGD) mask with k_mc_mask, equal to u·[e != 0].

Reference EF: ``IMAGENET/training/sparsified_ddp.py:409-413``."""
import pytest
import torch
from torch import nn

from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine

pytestmark = pytest.mark.gpu


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(16, 64, 3), nn.BatchNorm2d(64), nn.ReLU(), nn.Flatten(),
                         nn.Linear(64 * 6 * 6, 300), nn.ReLU(), nn.Linear(300, 10))


def _pair(mode, method, kw, wd):
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    engines = []
    for dev in ("cpu", "cuda"):
        net = _net().to(dev)
        eng = GradSyncEngine(list(net.named_parameters()), mode=mode, method=method,
                             error_feedback=True, momentum_correction=0.9, flat_params=True,
                             **kw)
        if wd:
            params = list(net.parameters())
            opt = FlatSGD([{"params": params[:2], "weight_decay": 0.0},
                           {"params": params[2:], "weight_decay": 5e-3}], eng.arena, lr=0.1,
                          grad_scale=0.25)
            eng.set_mc_weight_decay(opt)
        engines.append(eng)
    return engines


CASES = [("layerwise", "Topk", {"K": 0.01}),
         ("layerwise", "Topk", {"K": 0.01, "dense_below": 300}),
         ("entiremodel", "Topk", {"K": 0.001}),
         ("layerwise", "Randomk", {"K": 0.05})]


@pytest.mark.parametrize("wd", [False, True])
@pytest.mark.parametrize("mode,method,kw", CASES, ids=[f"{c[1]}-{c[0]}-{len(c[2])}" for c in CASES])
def test_fused_mc_matches_cpu_mirror_bitwise(mode, method, kw, wd):
    ec, eg = _pair(mode, method, kw, wd)
    assert ec.arena.numel == eg.arena.numel
    torch.manual_seed(1)
    for step in range(4):
        g = torch.zeros(ec.arena.numel)
        for s in ec.arena.segments:
            g[s.offset:s.offset + s.numel] = torch.randn(s.numel)
        for eng in (ec, eg):
            eng.arena.grad.copy_(g.to(eng.arena.grad.device))
            eng.sync_now()
        torch.cuda.synchronize()
        for name, a, b in (("grad", ec.arena.grad, eg.arena.grad), ("ef", ec.ef, eg.ef),
                           ("mom", ec.mom, eg.mom)):
            assert torch.equal(a, b.cpu()), (step, name, (a - b.cpu()).abs().max().item())


def test_fused_mc_issues_no_aten_elementwise_kernels():
    from torch.profiler import ProfilerActivity, profile
    net = _net().cuda()
    eng = GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.01,
                         error_feedback=True, momentum_correction=0.9, flat_params=True,
                         dense_below=300, overlap_compress=False)
    eng.arena.grad.normal_()
    eng.sync_now()                                   # (first call: tables, workspaces)
    torch.cuda.synchronize()
    eng.arena.grad.normal_()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        eng.sync_now()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    # the velocity update runs inside the first select pass (McArgs) — no k_mc_prep launch
    assert any("McArgs" in n for n in names), names
    assert not any("k_mc_prep" in n for n in names), names
    # what the fused path replaces: u.mul_(mc).add_(g), g.copy_(u), u.mul_(e != 0)
    bad = ("Mul", "mul", "Add", "add", "compare", "copy", "NE", "ne_kernel")
    aten = [n for n in names if "at::native" in n and any(k in n for k in bad)]
    assert not aten, aten


def test_mc_mask_kernel_for_codecs_without_selection():
    from layer_wise_aaai20_amd.ops._ext import load
    lib = load()
    torch.manual_seed(3)
    u = torch.randn(10007, device="cuda")
    e = torch.randn(10007, device="cuda")
    e[torch.rand(10007, device="cuda") < 0.3] = 0
    ref = u * (e != 0)
    lib.mc_mask(u, e)
    assert torch.equal(u, ref)
