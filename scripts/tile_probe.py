"""Time every tile candidate on a few ResNet-50 conv / GEMM shapes (bs 256): which tile the tuner
would keep and how far each is from the others. usage: python scripts/tile_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import block as blk  # noqa: E402
from layer_wise_aaai20_amd.ops import conv as CV  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

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


def conv_fwd(N, C, Co, H, k, s, p):
    x = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=CL)
    w = torch.randn(Co, C, k, k, device=dev).bfloat16().contiguous(memory_format=CL)
    Ho = (H + 2 * p - k) // s + 1
    fl = 2 * N * Ho * Ho * Co * C * k * k
    res = {}
    for t in CV.ROW_TILES + CV.BIG_TILES:
        CV.TUNER.pick = lambda key, run, cands, default, t=t: t
        res[t] = timeit(lambda: CV.conv_fwd(x, w, s, p, stats=True))
    print(f"conv-fwd {N, C, Co, H, k, s}: " + "  ".join(
        f"{t}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for t, v in res.items()), flush=True)


def conv_dgrad(N, C, Co, H, k, s, p):
    w = torch.randn(Co, C, k, k, device=dev).bfloat16().contiguous(memory_format=CL)
    Ho = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Co, Ho, Ho, device=dev).bfloat16().contiguous(memory_format=CL)
    fl = 2 * N * Ho * Ho * Co * C * k * k
    res = {}
    for lay in ("nkc", "kc"):
        for t in CV.ROW_TILES + (CV.BIG_TILES if lay == "kc" and s == 1 else ()):
            CV.TUNER.pick = lambda key, run, cands, default, c=(lay, t): c
            res[(lay, t)] = timeit(lambda: CV.conv_dgrad(dy, w, (H, H), s, p))
    print(f"conv-dgrad {N, C, Co, H, k, s}: " + "  ".join(
        f"{t[0]}{t[1]}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for t, v in res.items()), flush=True)


def gemm_fwd(M, N, K):
    lib = load()
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    res = {}
    for t in blk.TILES + blk.BIG + (11, 12, 13):
        try:
            res[t] = timeit(lambda: lib.gemm_ex(a, K, True, b, K, True, M, N, K, None, False, 1,
                                                True, t, None, None, True, True, None, None,
                                                False, 0, None, None, None, None, None))
        except RuntimeError:
            pass
    fl = 2 * M * N * K
    print(f"gemm-fwd+stats M{M} N{N} K{K}: " + "  ".join(
        f"{t}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for t, v in res.items()), flush=True)


for shp in [(256, 256, 256, 14, 3, 1, 1), (256, 512, 512, 7, 3, 1, 1), (256, 128, 128, 28, 3, 1, 1),
            (256, 64, 64, 56, 3, 1, 1)]:
    conv_fwd(*shp)
    conv_dgrad(*shp)
for m, n, k in [(50176, 256, 1024), (50176, 1024, 256), (12544, 512, 2048), (12544, 2048, 512),
                (200704, 128, 512), (200704, 512, 128)]:
    gemm_fwd(m, n, k)
