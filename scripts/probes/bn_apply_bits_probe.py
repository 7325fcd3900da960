"""Time k_bn_apply with residual (+ ReLU bitmap) on ResNet-50 layer1/layer3 shapes: is the
1-byte-per-thread bitmap store what holds the residual apply below the 2-read/1-write rate the
backward apply reaches?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

lib = load()


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


for M, C in ((256 * 56 * 56, 256), (256 * 14 * 14, 1024)):
    x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    r = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    ss = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")])
    bits = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
    gb = M * C * 2 / 1e9
    t_bits = timeit(lambda: lib.bn_apply(x, ss, r, None, True, bits))
    t_nob = timeit(lambda: lib.bn_apply(x, ss, r, None, True))
    t_nores = timeit(lambda: lib.bn_apply(x, ss, None, None, True))
    print(f"M={M} C={C}: res+bits {t_bits:.1f} us ({3 * gb / t_bits * 1e3:.2f} TB/s)  "
          f"res {t_nob:.1f} us ({3 * gb / t_nob * 1e3:.2f} TB/s)  "
          f"no-res {t_nores:.1f} us ({2 * gb / t_nores * 1e3:.2f} TB/s)", flush=True)
