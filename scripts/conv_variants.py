#!/usr/bin/env python
"""Time the conv / GEMM kernel variants of one ResNet-50 shape (plain, BN prologue, stats
epilogue, both) so the cost of each fusion is visible; also a short loop for PMC runs.
usage: python scripts/conv_variants.py [--shape 128,128,28,3,1,1] [--batch 256] [--tile N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402

CL = torch.channels_last


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="128,128,28,3,1,1")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma list of variant names")
    args = ap.parse_args()
    C, Co, H, k, s, p = (int(v) for v in args.shape.split(","))
    N = args.batch
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(Co, C, k, k, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
    Ho = CV.out_size(H, k, s, p)
    dy = torch.randn(N, Co, Ho, Ho, device="cuda").bfloat16().contiguous(memory_format=CL)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda")
    flops = 2.0 * N * Ho * Ho * Co * C * k * k
    wp = CV.pack_fwd_weight(w)
    var = {
        "fwd": lambda: CV.conv_fwd(x, w, s, p, wpack=wp),
        "fwd+stats": lambda: CV.conv_fwd(x, w, s, p, stats=True, wpack=wp),
        "fwd+pro": lambda: CV.conv_fwd(x, w, s, p, pro=(sc, sh), wpack=wp),
        "fwd+pro+stats": lambda: CV.conv_fwd(x, w, s, p, pro=(sc, sh), stats=True, wpack=wp),
        "dgrad": lambda: CV.conv_dgrad(dy, w, (H, H), s, p),
        "wgrad": lambda: CV.conv_wgrad(dy, x, tuple(w.shape), s, p),
        "wgrad+pro": lambda: CV.conv_wgrad(dy, x, tuple(w.shape), s, p, pro=(sc, sh)),
    }
    only = set(filter(None, args.only.split(",")))
    for name, fn in var.items():
        if only and name not in only:
            continue
        t = timeit(fn, args.iters)
        print(f"{args.shape:22s} {name:14s} {t:8.3f} ms {flops / t / 1e9:7.0f} TF/s", flush=True)
    print("tuner:", {str(k_[0]) + ('p' if k_[-2] else '') + ('s' if k_[-1] else ''): v
                     for k_, v in CV.TUNER.best.items()})


if __name__ == "__main__":
    main()
