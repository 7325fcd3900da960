"""Time the direct LDS-patch convolutions against the implicit-GEMM tiles on their ResNet-50
shapes (bs 256). usage: python scripts/direct_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402

CL = torch.channels_last
dev = torch.device("cuda", 0)


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


x = torch.randn(256, 64, 56, 56, device=dev).bfloat16().contiguous(memory_format=CL)
w = torch.randn(64, 64, 3, 3, device=dev).bfloat16().contiguous(memory_format=CL)
dy = torch.randn(256, 64, 56, 56, device=dev).bfloat16().contiguous(memory_format=CL)
fl = 2 * 256 * 56 * 56 * 64 * 576
for t in (2, 3, 5, CV.CONV3_DIRECT):
    CV.TUNER.pick = lambda key, run, cands, default, t=t: t
    us = timeit(lambda: CV.conv_fwd(x, w, 1, 1, stats=True))
    print(f"conv3 fwd tile {t}: {us:.1f} us {fl / us / 1e6:.0f} TF/s", flush=True)
for c in (("nkc", 3), ("kc", 3), ("direct", CV.CONV3_DIRECT)):
    CV.TUNER.pick = lambda key, run, cands, default, c=c: c
    us = timeit(lambda: CV.conv_dgrad(dy, w, (56, 56), 1, 1))
    print(f"conv3 dgrad {c}: {us:.1f} us {fl / us / 1e6:.0f} TF/s", flush=True)
xs = torch.randn(256, 4, 224, 224, device=dev).bfloat16().contiguous(memory_format=CL)
ws = torch.randn(64, 3, 7, 7, device=dev).bfloat16().contiguous(memory_format=CL)
for t in (3, 5, CV.STEM_DIRECT):
    CV.TUNER.pick = lambda key, run, cands, default, t=t: t
    us = timeit(lambda: CV.conv_fwd(xs, ws, 2, 3, stats=True))
    print(f"stem fwd tile {t}: {us:.1f} us", flush=True)
