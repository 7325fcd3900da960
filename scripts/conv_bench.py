#!/usr/bin/env python
"""Per-shape timing of the MFMA implicit-GEMM convs (ops/conv.py) against MIOpen (torch conv,
channels_last bf16) for the ResNet-50 @224 bs256 convolutions: forward, data gradient and weight
gradient, ms and TFLOP/s. usage: python scripts/conv_bench.py [--batch 256] [--only fwd,dgrad]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402

CL = torch.channels_last


def shapes(n):
    # (Cin, Cout, H, k, stride, pad, count in ResNet-50)
    return [(3, 64, 224, 7, 2, 3, 1), (64, 64, 56, 3, 1, 1, 3), (128, 128, 56, 3, 2, 1, 1),
            (128, 128, 28, 3, 1, 1, 3), (256, 256, 28, 3, 2, 1, 1), (256, 256, 14, 3, 1, 1, 5),
            (512, 512, 14, 3, 2, 1, 1), (512, 512, 7, 3, 1, 1, 2)]


def timeit(fn, iters=10):
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
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    N = args.batch
    tot = {"ours": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0]}
    print(f"{'shape':34s} {'pass':6s} {'ours ms':>8s} {'TF/s':>6s} {'miopen':>8s} {'TF/s':>6s}")
    for (C, Co, H, k, s, p, cnt) in shapes(N):
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(Co, C, k, k, device="cuda") * 0.05).bfloat16() \
            .contiguous(memory_format=CL)
        Ho = CV.out_size(H, k, s, p)
        dy = torch.randn(N, Co, Ho, Ho, device="cuda").bfloat16().contiguous(memory_format=CL)
        flops = 2.0 * N * Ho * Ho * Co * C * k * k
        wp = CV.pack_fwd_weight(w)
        ours = [
            lambda: CV.conv_fwd(x, w, s, p, wpack=wp),
            (lambda: CV.conv_dgrad(dy, w, (H, H), s, p)) if C % 8 == 0 else None,
            lambda: CV.conv_wgrad(dy, x, tuple(w.shape), s, p),
        ]
        ref = [
            lambda: torch.ops.aten.convolution(x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1),
            (lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1],
                                                         False, [0, 0], 1, [True, False, False]))
            if C % 8 == 0 else None,
            lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1],
                                                        False, [0, 0], 1, [False, True, False]),
        ]
        for i, name in enumerate(("fwd", "dgrad", "wgrad")):
            if ours[i] is None:
                continue
            to = timeit(ours[i])
            tr = timeit(ref[i])
            tot["ours"][i] += to * cnt
            tot["miopen"][i] += tr * cnt
            print(f"{str((C, Co, H, k, s)):34s} {name:6s} {to:8.3f} {flops / to / 1e9:6.0f} "
                  f"{tr:8.3f} {flops / tr / 1e9:6.0f}", flush=True)
    for i, name in enumerate(("fwd", "dgrad", "wgrad")):
        print(f"ResNet-50 total {name:6s}: ours {tot['ours'][i]:.3f} ms   "
              f"MIOpen {tot['miopen'][i]:.3f} ms")
    print("tuner picks:", {k[0] + str(k[1:4]): v for k, v in CV.TUNER.best.items()})


if __name__ == "__main__":
    main()
