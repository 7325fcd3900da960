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

        c2 = torch.randn(M, Ci, device="cuda").to(h16())
        ss2 = torch.cat([torch.rand(Ci, device="cuda") + 0.5, torch.randn(Ci, device="cuda")])
        mean2 = torch.randn(Ci, device="cuda") * .1

        def fused_s2():
            lib.bn3_bwd_fused(dy, x, bits, gam, mean, inv, w3t, a2, dw, dgo, dbo, *(None,) * 6,
                              c2, ss2, mean2)

        def bn2_reduce():
            lib.bn_bwd(a2, c2, None, mean2, mean2, mean2, ss2, True, True, False, None)

        def three():
            dc3, _, _, _ = lib.bn_bwd(dy, x, None, gam, mean, inv, None, True, True, False, bits,
                                      dgo, dbo)
            blk.gemm(dc3, C, False, a2, Ci, False, C, Ci, M, out_bf16=False, out=dw,
                     accumulate=True, split_k=True)
            blk.gemm_dgrad(dc3, C, w3, M, Ci, C)

        def reduce_only():
            lib.bn_bwd(dy, x, None, gam, mean, inv, None, True, True, False, bits, dgo, dbo)
        tf, t3, tr = timeit(fused), timeit(three), timeit(reduce_only)
        ts2, tb2 = timeit(fused_s2), timeit(bn2_reduce)
        print(f"M {M} C {C} Ci {Ci}: fused {tf:.1f} us   three-pass {t3:.1f} us   "
              f"(bn_bwd alone {tr:.1f} us); with BN2's sums {ts2:.1f} us vs BN2's whole "
              f"backward {tb2:.1f} us", flush=True)
        del dy, x, a2, bits


def bn1():
    """BN1 (no downsample) fused with dW1 / dx vs bn_bwd + the two GEMMs."""
    lib = load()
    for M, Wd, Cin in ((802816, 64, 256), (200704, 128, 512)):
        da1 = torch.randn(M, Wd, device="cuda").to(h16())
        c1 = torch.randn(M, Wd, device="cuda").to(h16())
        x = torch.randn(M, Cin, device="cuda").to(h16())
        dy = torch.randn(M, Cin, device="cuda").to(h16())
        w1 = (torch.randn(Wd, Cin, device="cuda") / 16).to(h16())
        w1t = w1.t().contiguous()
        bits = torch.randint(0, 256, (M * Cin // 8,), dtype=torch.uint8, device="cuda")
        gam, mean, inv = torch.rand(Wd, device="cuda") + 0.5, torch.randn(Wd, device="cuda") * .1, \
            torch.rand(Wd, device="cuda") + 0.5
        ss = torch.cat([gam * inv, -mean * gam * inv]).contiguous()
        dgo, dbo = torch.zeros(Wd, device="cuda"), torch.zeros(Wd, device="cuda")
        dw = torch.zeros(Wd, Cin, device="cuda")

        def fused():
            lib.bn1_bwd_fused(da1, c1, ss, gam, mean, inv, w1t, x, dy, bits, dw, dgo, dbo)

        def three():
            dc1, _, _, _ = lib.bn_bwd(da1, c1, None, gam, mean, inv, ss, True, True, False, None,
                                      dgo, dbo)
            blk.gemm(dc1, Wd, False, x, Cin, False, Wd, Cin, M, out_bf16=False, out=dw,
                     accumulate=True, split_k=True)
            blk.gemm_dgrad(dc1, Wd, w1, M, Cin, Wd, addend=dy, addend_bits=bits)

        def reduce_only():
            lib.bn_bwd(da1, c1, None, gam, mean, inv, ss, True, True, False, None, dgo, dbo)
        tf, t3, tr = timeit(fused), timeit(three), timeit(reduce_only)
        print(f"BN1 M {M} W {Wd} Cin {Cin}: fused {tf:.1f} us   three-pass {t3:.1f} us   "
              f"(bn_bwd alone {tr:.1f} us)", flush=True)


def stem():
    """Stem backward: pool/BN apply fused into the 7x7/2 weight gradient vs the two passes."""
    from layer_wise_aaai20_amd.ops import conv as CV
    lib = load()
    N = 256
    x4 = torch.randn(N, 4, 224, 224, device="cuda").to(h16()).contiguous(
        memory_format=torch.channels_last)
    c = torch.randn(N, 64, 112, 112, device="cuda").to(h16()).contiguous(
        memory_format=torch.channels_last)
    gam, mean, inv = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * .1, \
        torch.rand(64, device="cuda") + 0.5
    ss = torch.cat([gam * inv, -mean * gam * inv]).contiguous()
    pooled, idx = lib.stem_pool_fwd(c, ss, 3, 2, 1)
    dp = torch.randn_like(pooled.float()).to(h16()).contiguous(memory_format=torch.channels_last)

    def fused():
        lib.stem_bwd_fused(dp, idx, c, ss, gam, mean, inv, 3, 2, 1, None, None, pooled, x4)

    def two():
        dc, _, _ = lib.stem_pool_bwd(dp, idx, c, ss, gam, mean, inv, 3, 2, 1, None, None, pooled)
        CV.conv_wgrad(dc, x4, (64, 3, 7, 7), 2, 3)
    print(f"stem backward: fused {timeit(fused):.1f} us   two-pass {timeit(two):.1f} us", flush=True)


if __name__ == "__main__":
    main()
    bn1()
    stem()
