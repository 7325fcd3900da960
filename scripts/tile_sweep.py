#!/usr/bin/env python
"""Per-tile timing of the MFMA GEMM (ops/gemm.py gemm_ex with an explicit tile id) on large
square GEMMs and on the ResNet-50 / VGG GEMM shapes, in the three operand layouts a layer uses:
fwd (A, B K-contiguous), dgrad (B N-contiguous), wgrad (A M-contiguous, B N-contiguous, fp32
out). Prints TF/s per (shape, layout, tile) and the hipBLASLt time of the same product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

SHAPES = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
          ("vgg fc0", 512, 4096, 25088), ("vgg fc1", 512, 4096, 4096),
          ("r50 c3 l2", 200704, 512, 128), ("r50 c3 l3", 50176, 1024, 256),
          ("r50 c3 l4", 12544, 2048, 512), ("r50 c1 l3", 50176, 256, 1024),
          ("r50 dx l3", 50176, 1024, 256), ("r50 c1 l4", 12544, 512, 2048)]
TILES = [int(t) for t in os.environ.get("SWEEP_TILES", "1,2,3,4,5,6").split(",")]


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
    torch.manual_seed(0)
    for name, M, N, K in SHAPES:
        fl = 2.0 * M * N * K
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        wt = w.t().contiguous()          # [K][N]
        at = a.t().contiguous()          # [K][M]
        rows = [("fwd", lambda t: G.gemm_ex(a, K, True, w, K, True, M, N, K, tile=t),
                 lambda: torch.mm(a, w.t())),
                ("dgrad", lambda t: G.gemm_ex(a, K, True, wt, N, False, M, N, K, tile=t),
                 lambda: torch.mm(a, wt)),
                ("wgrad", lambda t: G.gemm_ex(at, M, False, wt, N, False, M, N, K, tile=t,
                                              out_bf16=False),
                 lambda: torch.mm(at.t(), wt))]
        for lay, ours, blas in rows:
            res = []
            for t in TILES:
                try:
                    ms = timeit(lambda: ours(t))
                    res.append(f"t{t}:{fl / ms / 1e9:5.0f}")
                except RuntimeError as e:  # noqa: PERF203
                    res.append(f"t{t}:err({str(e)[:30]})")
            bl = fl / timeit(blas) / 1e9
            print(f"{name:10s} {lay:5s} M{M:7d} N{N:5d} K{K:5d} | blas {bl:5.0f} | " + " ".join(res),
                  flush=True)
        del a, w, wt, at
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
