#!/usr/bin/env python
"""A/B of the tiled MFMA GEMM on v_mfma_f32_16x16x32 (tiles 1..6) against its v_mfma_f32_32x32x16
twin (tile + 40, csrc/gemm_core.h k_gemm MF = 32): every ResNet-50 @224 (batch 256) 3x3
convolution pass and 1x1 GEMM shape, each tile pinned in turn, rounds interleaved in one process
(cdna_hip_programming.md §5.4 rule 24), random operands. Prints µs per (shape, pass, tile) for
both shapes and the per-pass best of each family.
usage: python scripts/mf32_ab.py [--rounds 3] [--only conv|gemm]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402
from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

CL = torch.channels_last
MF32 = 40


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


class Pin:
    """Pin ops/conv.py's tuner to one choice."""

    def __init__(self, choice):
        self.choice = choice

    def __enter__(self):
        self.old = CV.TUNER.pick
        CV.TUNER.pick = lambda key, run, cands, default: self.choice
        return self

    def __exit__(self, *a):
        CV.TUNER.pick = self.old


def conv_cases(batch):
    out = []
    for C, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        x = torch.randn(batch, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(C, C, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(batch, C, H, H, device="cuda").bfloat16().contiguous(memory_format=CL)
        dw = torch.zeros(C, C, 3, 3, device="cuda").contiguous(memory_format=CL)
        flops = 2.0 * batch * H * H * C * C * 9
        name = f"3x3 x({batch},{C},{H},{H})"
        out.append((name, "fwd", flops, (1, 2, 3, 5, 6),
                    lambda t, x=x, w=w: Pin(t), lambda x=x, w=w: CV.conv_fwd(x, w, 1, 1, stats=True)))
        out.append((name, "dgrad", flops, (1, 2, 3, 5, 6),
                    lambda t: Pin(("kc", t)), lambda dy=dy, w=w, H=H: CV.conv_dgrad(dy, w, (H, H), 1, 1)))
        pix = batch * H * H

        def wg_pin(t, C=C, pix=pix):
            bm, bn, bk = CV._TILE_DIMS[t]
            tiles = -(-C // bm) * -(-(9 * C) // bn)
            return Pin((t, CV._wgrad_splits(tiles, pix, bk)))
        out.append((name, "wgrad", flops, (1, 2, 4, 6), wg_pin,
                    lambda dy=dy, x=x, w=w, dw=dw: CV.conv_wgrad(dy, x, tuple(w.shape), 1, 1, out=dw)))
    return out


def gemm_cases():
    shapes = [(802816, 64, 256), (802816, 256, 64), (200704, 128, 512), (200704, 512, 128),
              (50176, 256, 1024), (50176, 1024, 256), (12544, 512, 2048), (12544, 2048, 512)]
    out = []
    for M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        wt = w.t().contiguous()
        g = torch.randn(M, N, device="cuda").bfloat16()
        fl = 2.0 * M * N * K
        name = f"1x1 M{M} N{N} K{K}"
        out.append((name, "fwd", fl, (1, 2, 3, 5, 6), lambda t: t,
                    lambda t, a=a, w=w, M=M, N=N, K=K: G.gemm_ex(a, K, True, w, K, True, M, N, K,
                                                                 tile=t, stats=True)))
        out.append((name, "dgrad", fl, (1, 2, 3, 5, 6), lambda t: t,
                    lambda t, a=a, wt=wt, M=M, N=N, K=K: G.gemm_ex(a, K, True, wt, N, False, M, N,
                                                                   K, tile=t)))
        out.append((name, "wgrad", fl, (1, 2, 4, 6), lambda t: t,
                    lambda t, g=g, a=a, M=M, N=N, K=K: G.gemm_ex(g, N, False, a, K, False, N, K,
                                                                 M, splits=max(1, 512 // max(1, (-(-N // 128)) * (-(-K // 128)))),
                                                                 out_bf16=False, tile=t)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    cases = []
    if a.only in ("", "conv"):
        cases += [(n, p, f, ts, pin, fn, "conv") for n, p, f, ts, pin, fn in conv_cases(a.batch)]
    if a.only in ("", "gemm"):
        cases += [(n, p, f, ts, pin, fn, "gemm") for n, p, f, ts, pin, fn in gemm_cases()]
    print(f"{'shape':28s} {'pass':5s} " + "  ".join(f"t{t}/t{t + MF32}" for t in (1, 2, 3, 4, 5, 6))
          + "   best16 best32 (us)", flush=True)
    tot16 = tot32 = 0.0
    for name, pas, fl, tiles, pin, fn, kind in cases:
        res = {}
        for _ in range(a.rounds):
            for t in tiles:
                for tt in (t, t + MF32):
                    try:
                        if kind == "conv":
                            with pin(tt):
                                us = timeit(fn)
                        else:
                            us = timeit(lambda: fn(tt))
                    except RuntimeError as e:          # noqa: PERF203
                        print(f"  {name} {pas} t{tt}: {str(e)[:60]}", flush=True)
                        us = float("inf")
                    res[tt] = min(res.get(tt, float("inf")), us)
        b16 = min(res[t] for t in tiles)
        b32 = min(res[t + MF32] for t in tiles)
        tot16 += b16
        tot32 += b32
        cells = "  ".join(f"{res.get(t, 0):6.1f}/{res.get(t + MF32, 0):6.1f}" if t in tiles else
                          f"{'-':>13s}" for t in (1, 2, 3, 4, 5, 6))
        print(f"{name:28s} {pas:5s} {cells}   {b16:6.1f} {b32:6.1f}  "
              f"({fl / b16 / 1e6:5.0f} / {fl / b32 / 1e6:5.0f} TF/s)", flush=True)
    print(f"sum of per-pass bests: mfma16 {tot16:.1f} us, mfma32 {tot32:.1f} us")


if __name__ == "__main__":
    main()
