#!/usr/bin/env python
"""Per-shape roofline check of the fused BN kernels on the ResNet-50 (bs 256) BN layer shapes.

For each unique (C, H, residual, relu) configuration it times forward (reduce + finalize + apply)
and backward (reduce + finalize + apply) with HIP events and reports achieved HBM bandwidth from the
minimum bytes each pass must move (bf16)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from layer_wise_aaai20_amd.models.resnet import resnet50  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402


def layer_shapes(batch):
    m = resnet50()
    shapes = {}

    def hook(mod, inp, out):
        shapes[mod] = (out.shape[1], out.shape[2], out.shape[3])
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.register_forward_hook(hook)
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    # Bottleneck bn3 carries the residual; downsample BNs have no ReLU
    cfg = {}
    for n, mod in m.named_modules():
        if not isinstance(mod, torch.nn.BatchNorm2d):
            continue
        c, h, w = shapes[mod]
        res = n.endswith("bn3")
        relu = not n.endswith("downsample.1")
        key = (c, h, w, res, relu)
        cfg[key] = cfg.get(key, 0) + 1
    return cfg


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    lib = load()
    dev = torch.device("cuda")
    tot_f = tot_b = 0.0
    print(f"{'C':>5} {'HxW':>7} res relu  n  fwd_ms  fwd_GB/s  bwd_ms  bwd_GB/s")
    for (c, h, w, res, relu), cnt in sorted(layer_shapes(args.batch).items()):
        x = torch.randn(args.batch, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        wgt = torch.rand(c, device=dev) + 0.5
        b = torch.randn(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        y, mean, invstd, ss = lib.bn_fwd(x, r, wgt, b, rm, rv, True, 0.1, 1e-5, relu)
        dy = torch.randn_like(x)
        keep_y = relu and res
        tf = timeit(lambda: lib.bn_fwd(x, r, wgt, b, rm, rv, True, 0.1, 1e-5, relu), args.iters)
        tb = timeit(lambda: lib.bn_bwd(dy, x, y if keep_y else None, wgt, mean, invstd,
                                       None if keep_y else ss, True, relu, res), args.iters)
        e = x.numel() * 2
        fbytes = e * (3 + (1 if res else 0))                      # read x twice, write y, (+res)
        bbytes = e * (5 + (2 if keep_y else 0) + (1 if res else 0))  # x,dy twice + dx (+y twice, +dres)
        tot_f += tf * cnt
        tot_b += tb * cnt
        print(f"{c:5d} {h:3d}x{w:<3d} {int(res):3d} {int(relu):4d} {cnt:2d} {tf:7.3f} "
              f"{fbytes / tf / 1e6:9.0f} {tb:7.3f} {bbytes / tb / 1e6:9.0f}")
    print(f"total per step: fwd {tot_f:.3f} ms  bwd {tot_b:.3f} ms")


if __name__ == "__main__":
    main()
