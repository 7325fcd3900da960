"""Diagnostic: relative errors of the block-fused and per-layer-fused bottleneck paths against
the fp32 PyTorch bottleneck (forward output, input gradient, every parameter gradient)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from layer_wise_aaai20_amd.models.resnet import Bottleneck, conv1x1  # noqa: E402
from layer_wise_aaai20_amd.ops.nn import fuse_resnet  # noqa: E402

CL = torch.channels_last


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def make(inplanes, planes, stride, down):
    ds = None
    if down:
        ds = torch.nn.Sequential(conv1x1(inplanes, planes * 4, stride),
                                 torch.nn.BatchNorm2d(planes * 4))
    m = Bottleneck(inplanes, planes, stride, ds)
    for bn in [m.bn1, m.bn2, m.bn3] + ([ds[1]] if down else []):
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.normal_(0, 0.2)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16).float()
    return m


for cfg in [(256, 64, 1, False), (64, 64, 1, True), (256, 128, 2, True)]:
    torch.manual_seed(0)
    ref = make(*cfg).cuda().to(memory_format=CL)
    x = torch.randn(8, cfg[0], 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(8, cfg[1] * 4, 14 // cfg[2], 14 // cfg[2], device="cuda")
    xf = x.float().requires_grad_()
    yr = ref(xf)
    yr.backward(g)
    res = {}
    for name, blockmode in (("block", True), ("layer", False)):
        m = copy.deepcopy(ref)
        for p in m.parameters():
            p.grad = None
        fuse_resnet(m, block=blockmode)
        xb = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xb)
        y.backward(g.to(y.dtype))
        errs = {"y": rel(y, yr), "dx": rel(xb.grad, xf.grad)}
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            errs[n] = rel(p.grad, q.grad)
        res[name] = errs
    print(cfg)
    for k in res["block"]:
        print(f"  {k:24s} block {res['block'][k]:.4f}  layer {res['layer'][k]:.4f}")

# ---- whole ResNet-50: per-parameter errors of both bf16 paths against fp32
from layer_wise_aaai20_amd.models.resnet import resnet50  # noqa: E402
from layer_wise_aaai20_amd.ops.nn import share_bn_counters  # noqa: E402

for bs, hw in ((4, 64), (16, 96)):
    torch.manual_seed(2)
    ref = resnet50().cuda()
    for p in ref.parameters():
        p.data = p.data.to(torch.bfloat16).float()
    mods = {"block": copy.deepcopy(ref), "layer": copy.deepcopy(ref)}
    ref = ref.to(memory_format=CL)
    x = torch.randn(bs, 3, hw, hw, device="cuda").to(torch.bfloat16).float().contiguous(memory_format=CL)
    t = torch.randint(0, 1000, (bs,), device="cuda")
    torch.nn.functional.cross_entropy(ref(x), t).backward()
    errs = {}
    for name, m in mods.items():
        fuse_resnet(m, block=name == "block")
        m.to(memory_format=CL)
        share_bn_counters(m)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x)
        torch.nn.functional.cross_entropy(out.float(), t).backward()
        errs[name] = {n: rel(p.grad, q.grad) for (n, p), q in zip(m.named_parameters(), ref.parameters())}
    print(f"resnet50 bs{bs} {hw}px: worst 12 params by block error")
    for n in sorted(errs["block"], key=lambda k: -errs["block"][k])[:12]:
        print(f"  {n:36s} block {errs['block'][n]:.4f}  layer {errs['layer'][n]:.4f}")
