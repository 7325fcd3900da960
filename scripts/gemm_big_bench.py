#!/usr/bin/env python
"""Forward-layout (A [M][K], B [N][K]) GEMM throughput: the 256x256x64 8-wave LDS-DMA kernel
(tile 21, csrc/gemm_big.hip) vs the 128x128x64 4-wave tile (tile 2) vs hipBLASLt (torch.mm), each
of ours at its best split-K count. Prints one JSON line per shape (TFLOP/s)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

SHAPES = [("sq8192", 8192, 8192, 8192), ("sq4096", 4096, 4096, 4096),
          ("sq16384x8192", 16384, 16384, 8192),
          ("vgg fc0 b512", 512, 4096, 25088), ("vgg fc1 b512", 512, 4096, 4096),
          # ResNet-50 at batch 256: 1x1 forward convs (M = pixels, N = out, K = in channels);
          # the c1 shapes are also the data-gradient GEMMs of the c3 convs with Wᵀ as B
          ("r50 l1 c1", 802816, 64, 256), ("r50 l1 c3", 802816, 256, 64),
          ("r50 l2 c1", 200704, 128, 512), ("r50 l2 c3", 200704, 512, 128),
          ("r50 l3 c1", 50176, 256, 1024), ("r50 l3 c3", 50176, 1024, 256),
          ("r50 l4 c1", 12544, 512, 2048), ("r50 l4 c3", 12544, 2048, 512)]
SPLITS = (1, 2, 4, 8)


def timeit(fn, iters):
    """Device time per call: the calls are captured into one HIP graph and replayed, so host
    launch overhead (allocations, binding) does not hide small kernels."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    del g
    return s.elapsed_time(e) / iters


WGRAD = [("wg l1 c3", 256, 64, 802816), ("wg l2 c3", 512, 128, 200704),
         ("wg l3 c3", 1024, 256, 50176), ("wg l4 c3", 2048, 512, 12544),
         ("wg l2 c1", 128, 512, 200704), ("wg l3 c1", 256, 1024, 50176),
         ("wg l4 c1", 512, 2048, 12544)]
DIMS = {2: (128, 128), 21: (256, 256), 22: (256, 128)}


def wgrad_rows():
    """Weight-gradient layout (both operands MN-contiguous: dY [pix][Co], X [pix][C]), fp32
    accumulated into the output as the engine does, each tile at the split counts around the
    engine's heuristic (ops/block.py _splits)."""
    for name, M, N, K in WGRAD:
        fl = 2.0 * M * N * K
        iters = max(3, min(50, int(2e13 / fl)))
        dy = torch.randn(K, M, device="cuda").bfloat16()
        x = torch.randn(K, N, device="cuda").bfloat16()
        out = torch.zeros(M, N, device="cuda")
        row = {"shape": name, "M": M, "N": N, "K": K}
        ref = None
        for t, (bm, bn) in DIMS.items():
            tiles = -(-M // bm) * -(-N // bn)
            s0 = max(1, min(512 // tiles, K // 256))
            best = None
            for sp in sorted({max(1, s0 // 2), s0, s0 * 2}):
                ms = timeit(lambda: G.load().gemm_ex(dy, M, False, x, N, False, M, N, K, None,
                                                     False, sp, False, t, None, None, True, False,
                                                     out, None, True, 0, None), iters)
                if best is None or ms < best[0]:
                    best = (ms, sp)
            row[f"t{t}_tflops"] = round(fl / best[0] / 1e9, 1)
            row[f"t{t}_splits"] = best[1]
            c, _ = G.gemm_ex(dy, M, False, x, N, False, M, N, K, splits=4, out_bf16=False, tile=t)
            if ref is None:
                ref = c
            else:
                row[f"t{t}_eq_t2"] = bool(torch.equal(c, ref))
        row["blas_tflops"] = round(fl / timeit(lambda: torch.mm(dy.t(), x), iters) / 1e9, 1)
        print(json.dumps(row), flush=True)
        del dy, x, out, ref
        torch.cuda.empty_cache()


def main():
    only = os.environ.get("ONLY")
    torch.manual_seed(0)
    for name, M, N, K in SHAPES:
        if only and only not in name:
            continue
        fl = 2.0 * M * N * K
        iters = max(3, min(50, int(2e13 / fl)))
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        row = {"shape": name, "M": M, "N": N, "K": K}
        ref = None
        for t in (2, 21, 22, 23, 24):     # 23 / 24: the persistent big tiles (never split)
            best = None
            for sp in SPLITS:
                if sp > 1 and (K // sp < 256 or t in (23, 24)):
                    continue
                ms = timeit(lambda: G.gemm_ex(a, K, True, w, K, True, M, N, K, splits=sp, tile=t),
                            iters)
                if best is None or ms < best[0]:
                    best = (ms, sp)
            row[f"t{t}_tflops"] = round(fl / best[0] / 1e9, 1)
            row[f"t{t}_splits"] = best[1]
            if name.startswith("r50"):      # conv forward: BN statistics in the epilogue
                ms = timeit(lambda: G.gemm_ex(a, K, True, w, K, True, M, N, K, tile=t, stats=True),
                            iters)
                row[f"t{t}_stats_tflops"] = round(fl / ms / 1e9, 1)
            c, _ = G.gemm_ex(a, K, True, w, K, True, M, N, K, splits=1, tile=t)
            if ref is None:
                ref = c
            else:
                row[f"t{t}_eq_t2"] = bool(torch.equal(c, ref))
        if name.startswith("r50"):
            # data-gradient layout: B = W as stored for the forward ([K][N] here, N-contiguous)
            wt = w.t().contiguous()
            ms = timeit(lambda: G.gemm_ex(a, K, True, wt, N, False, M, N, K, tile=2), iters)
            row["t2_nkc_tflops"] = round(fl / ms / 1e9, 1)
            if K in (64, 128, 256):       # streaming kernel (B panel resident in LDS)
                best = min(timeit(lambda: G.gemm_ex(a, K, True, w, K, True, M, N, K, tile=t,
                                                    stats=True), iters)
                           for t in (11, 12, 13) if not (K == 256 and t == 13))
                row["stream_stats_tflops"] = round(fl / best / 1e9, 1)
        row["blas_tflops"] = round(fl / timeit(lambda: torch.mm(a, w.t()), iters) / 1e9, 1)
        print(json.dumps(row), flush=True)
        del a, w, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    if os.environ.get("WGRAD", "1") == "1":
        wgrad_rows()
    if os.environ.get("FWD", "1") == "1":
        main()
