#!/usr/bin/env python
"""Per-shape timing of the Linear layers of the reference models on the hand-written MFMA GEMM
(ops/gemm.py linear_fwd / linear_dgrad / linear_wgrad) against the vendor BLAS that torch calls
for the same bf16 GEMM (hipBLASLt via torch.matmul / F.linear) — the evidence that dropping the
BLAS path from the models cost nothing. Prints one row per (shape, pass): µs ours, µs BLAS, ratio.

Shapes: ResNet-50 fc (IMAGENET/training/resnet.py:110, batch 256), CIFAR AlexNet classic and
VGG-16 classifiers (CIFAR10/alexnet.py:29-37, CIFAR10/vgg16.py:23-31, batch 512)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

SHAPES = [("resnet50.fc", 256, 2048, 1000), ("alexnet.fc1", 512, 1024, 4096),
          ("alexnet.fc2", 512, 4096, 4096), ("alexnet.fc3", 512, 4096, 10),
          ("vgg16.fc1", 512, 25088, 4096), ("vgg16.fc2", 512, 4096, 4096),
          ("vgg16.fc3", 512, 4096, 10)]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1e3 * s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    print(f"{'layer':14s} {'pass':6s} {'M':>5s} {'K':>6s} {'N':>5s} {'ours_us':>9s} {'blas_us':>9s} {'ratio':>6s}")
    for name, M, K, N in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        b = torch.randn(N, device="cuda")
        dy = torch.randn(M, N, device="cuda").bfloat16()
        Np = -(-N // 8) * 8                    # MFMALinear pads odd N (ops/gemm.py)
        wp = torch.cat([w, w.new_zeros(Np - N, K)]) if Np != N else w
        bp = torch.cat([b, b.new_zeros(Np - N)]) if Np != N else b
        dyp = torch.cat([dy, dy.new_zeros(M, Np - N)], 1) if Np != N else dy
        rows = [("fwd", lambda: G.linear_fwd(x, wp, bp), lambda: F.linear(x, w, b.bfloat16())),
                ("dgrad", lambda: G.linear_dgrad(dyp, wp), lambda: dy @ w),
                ("wgrad", lambda: G.linear_wgrad(dyp, x), lambda: dy.t() @ x)]
        for pas, ours, blas in rows:
            t0, t1 = timeit(ours), timeit(blas)
            print(f"{name:14s} {pas:6s} {M:5d} {K:6d} {N:5d} {t0:9.1f} {t1:9.1f} {t0 / t1:6.2f}")


if __name__ == "__main__":
    main()
