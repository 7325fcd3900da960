#!/usr/bin/env python
"""Weight-resident 3x3 conv (csrc/conv3tap.hip k_conv3_res, C = Co = 64) against the tap kernel
and the shipped tuner's pick: forward (+ statistics) and data gradient, µs. Shapes: ResNet-50
stage 1 (batch 256, 56 px) and the CIFAR 64->64 convs (batch 512, 32 px).
usage: python scripts/conv3_res_bench.py"""
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
    lib = load()
    print(f"{'shape':22s} {'pass':5s} {'res us':>8s} {'tap us':>8s} {'tuned us':>9s} {'floor us':>9s}")
    for N, H in ((256, 56), (512, 32), (256, 28)):
        x = torch.randn(N, 64, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(N, 64, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        op, _, _ = CV.pack_fwd_weight(w)
        wf = CV.tap_dgrad_weight(w)
        floor = max(2.0 * N * H * H * 64 * 576 / 2.3e15, 2 * x.numel() * 2 / 6.3e12) * 1e6
        for name, a, wt, st in (("fwd", x, op, True), ("dgrad", dy, wf, False)):
            r = timeit(lambda: lib.conv3_res(a, wt, st))
            t = timeit(lambda: lib.conv3_tap(a, wt, 64, st))
            if name == "fwd":
                g = timeit(lambda: CV.conv_fwd(x, w, 1, 1, wpack=(op, 576, 3), stats=True))
            else:
                g = timeit(lambda: CV.conv_dgrad(dy, w, (H, H), 1, 1))
            print(f"({N},64,{H},{H})->64".ljust(22), f"{name:5s} {r:8.1f} {t:8.1f} {g:9.1f} {floor:9.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
