"""Comparison table only (not a dispatch path): the ResNet-50 (bs 256) 1x1-convolution GEMMs on
the hand-written MFMA kernels, through the same tuned entry the fused bottleneck calls
(ops/block.py gemm / gemm_dgrad, every candidate tile timed, the best kept), against hipBLASLt
through torch.mm on the same operand layouts (no transpose copies: .t() views).

  forward   y[M, co]  = x[M, ci] · W[co, ci]ᵀ        (both K-contiguous)
  dgrad     dx[M, ci] = dy[M, co] · W[co, ci]         (W as stored, or the tuner's Wᵀ pack)
  wgrad     dW[co, ci] = dy[M, co]ᵀ · x[M, ci]        (ours: split-K, fp32 slabs + fixed-order
                                                       reduce into an fp32 gradient; hipBLASLt: bf16
                                                       output, i.e. fewer bytes written)

Prints one line per (shape, direction): µs ours / hipBLASLt, the ratio and TF/s, then the
per-step totals weighted by how often each shape occurs. usage: python scripts/vendor_1x1_table.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops import block as blk  # noqa: E402

B = 256
SHAPES = [  # (H, Cin, Cout, calls per step)
    (56, 64, 64, 1), (56, 64, 256, 4), (56, 256, 64, 2), (56, 256, 128, 1), (28, 128, 512, 5),
    (28, 512, 128, 3), (28, 512, 256, 1), (14, 256, 1024, 7), (14, 1024, 256, 5),
    (14, 1024, 512, 1), (7, 512, 2048, 4), (7, 2048, 512, 2)]


def timeit(fn, reps=5, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / n * 1e3)
    return statistics.median(out)


def main():
    dev = "cuda"
    tot = {"ours": 0.0, "blas": 0.0}
    worst = []
    print(f"{'shape':28s} {'dir':6s} {'ours us':>9s} {'hipBLASLt':>9s} {'ratio':>6s} "
          f"{'ours TF':>8s} {'blas TF':>8s}")
    for H, ci, co, cnt in SHAPES:
        M = B * H * H
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, ci, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(M, co, device=dev, generator=g).to(torch.bfloat16)
        W = torch.randn(co, ci, device=dev, generator=g).to(torch.bfloat16)
        dW = torch.zeros(co, ci, device=dev)
        flops = 2.0 * M * ci * co
        cases = {
            "fwd": (lambda: blk.gemm(x, ci, True, W, ci, True, M, co, ci),
                    lambda: torch.mm(x, W.t())),
            "dgrad": (lambda: blk.gemm_dgrad(dy, co, W, M, ci, co),
                      lambda: torch.mm(dy, W)),
            "wgrad": (lambda: blk.gemm(dy, co, False, x, ci, False, co, ci, M, out_bf16=False,
                                       out=dW, accumulate=True, split_k=True),
                      lambda: torch.mm(dy.t(), x)),
        }
        for d, (ours, blas) in cases.items():
            to, tb = timeit(ours), timeit(blas)
            tot["ours"] += to * cnt
            tot["blas"] += tb * cnt
            worst.append((to / tb, f"H{H} {ci}->{co} {d}"))
            print(f"H{H:3d} {ci:5d}->{co:5d} x{cnt:<2d}          {d:6s} {to:9.1f} {tb:9.1f} "
                  f"{to / tb:6.2f} {flops / to / 1e6:8.0f} {flops / tb / 1e6:8.0f}", flush=True)
    print(f"per-step totals (x calls): ours {tot['ours'] / 1e3:.3f} ms, hipBLASLt "
          f"{tot['blas'] / 1e3:.3f} ms, ratio {tot['ours'] / tot['blas']:.3f}")
    worst.sort(reverse=True)
    print("worst ratios:", ", ".join(f"{n} {r:.2f}" for r, n in worst[:5]))


if __name__ == "__main__":
    main()
