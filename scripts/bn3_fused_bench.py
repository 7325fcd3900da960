#!/usr/bin/env python
"""BN3 backward fused with its two GEMMs (csrc/bnfuse.hip) vs the three-pass block path at the
ResNet-50 stage-1 / stage-2 shapes (batch 256: M = 802816 rows, 256 / 64 channels; M = 200704,
512 / 128), µs per call.
The three-pass arm is bn_bwd (reduce + finalize + apply) + dW3 GEMM + da2 GEMM through the
block's tuned wrappers. usage: python scripts/bn3_fused_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import block as blk  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import h16, load  # noqa: E402


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
    for M, C, Ci in ((802816, 256, 64), (200704, 512, 128)):
        dy = torch.randn(M, C, device="cuda").to(h16())
        x = torch.randn(M, C, device="cuda").to(h16())
        a2 = torch.randn(M, Ci, device="cuda").to(h16())
        w3 = (torch.randn(C, Ci, device="cuda") / 16).to(h16())
        w3t = w3.t().contiguous()
        bits = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
        gam, mean, inv = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * .1, \
            torch.rand(C, device="cuda") + 0.5
        dgo, dbo = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        dw = torch.zeros(C, Ci, device="cuda")

        def fused():
            lib.bn3_bwd_fused(dy, x, bits, gam, mean, inv, w3t, a2, dw, dgo, dbo)

        def three():
            dc3, _, _, _ = lib.bn_bwd(dy, x, None, gam, mean, inv, None, True, True, False, bits,
                                      dgo, dbo)
            blk.gemm(dc3, C, False, a2, Ci, False, C, Ci, M, out_bf16=False, out=dw,
                     accumulate=True, split_k=True)
            blk.gemm_dgrad(dc3, C, w3, M, Ci, C)

        def reduce_only():
            lib.bn_bwd(dy, x, None, gam, mean, inv, None, True, True, False, bits, dgo, dbo)
        tf, t3, tr = timeit(fused), timeit(three), timeit(reduce_only)
        print(f"M {M} C {C} Ci {Ci}: fused {tf:.1f} us   three-pass {t3:.1f} us   "
              f"(bn_bwd alone {tr:.1f} us)", flush=True)
        del dy, x, a2, bits


if __name__ == "__main__":
    main()
