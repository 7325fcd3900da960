#!/usr/bin/env python
"""Tap-reuse 3x3/1 convolution (csrc/conv3tap.hip) against the tuned implicit-GEMM path
(ops/conv.py with the tap candidate switched off) on the stride-1 3x3 shapes of ResNet-50 @224
(batch 256) and of the CIFAR nets (batch 512): forward (+ column statistics) and data gradient,
µs and TFLOP/s. usage: python scripts/conv_tap_bench.py [--batch 256]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

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
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--cifar-batch", type=int, default=512)
    args = ap.parse_args()
    lib = load()
    shapes = [("r50", args.batch, 64, 64, 56), ("r50", args.batch, 128, 128, 28),
              ("r50", args.batch, 256, 256, 14), ("r50", args.batch, 512, 512, 7),
              ("cifar", args.cifar_batch, 64, 128, 32), ("cifar", args.cifar_batch, 128, 128, 16),
              ("cifar", args.cifar_batch, 256, 512, 8), ("cifar", args.cifar_batch, 512, 512, 4)]
    print(f"{'shape':28s} {'pass':5s} {'tap us':>8s} {'TF/s':>6s} {'gemm us':>8s} {'TF/s':>6s}")
    for tag, N, C, Co, H in shapes:
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(Co, C, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(N, Co, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        flops = 2.0 * N * H * H * Co * C * 9
        op, _, _ = CV.pack_fwd_weight(w)
        wf = CV.tap_dgrad_weight(w)
        t_f = timeit(lambda: lib.conv3_tap(x, op, Co, True))
        t_d = timeit(lambda: lib.conv3_tap(dy, wf, C, False))
        dw = torch.zeros(Co, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        t_w = timeit(lambda: lib.conv3_tap_wgrad(dy, x, dw, True))
        CV.CONV3_TAP_ON = False
        try:
            g_f = timeit(lambda: CV.conv_fwd(x, w, 1, 1, wpack=(op, 9 * C, 3), stats=True))
            g_d = timeit(lambda: CV.conv_dgrad(dy, w, (H, H), 1, 1))
            g_w = timeit(lambda: CV.conv_wgrad(dy, x, tuple(w.shape), 1, 1, out=dw))
        finally:
            CV.CONV3_TAP_ON = True
        name = f"{tag} x({N},{C},{H},{H})->{Co}"
        print(f"{name:28s} {'fwd':5s} {t_f:8.1f} {flops / t_f / 1e6:6.0f} {g_f:8.1f} "
              f"{flops / g_f / 1e6:6.0f}", flush=True)
        print(f"{name:28s} {'dgrad':5s} {t_d:8.1f} {flops / t_d / 1e6:6.0f} {g_d:8.1f} "
              f"{flops / g_d / 1e6:6.0f}", flush=True)
        print(f"{name:28s} {'wgrad':5s} {t_w:8.1f} {flops / t_w / 1e6:6.0f} {g_w:8.1f} "
              f"{flops / g_w / 1e6:6.0f}", flush=True)


if __name__ == "__main__":
    main()
