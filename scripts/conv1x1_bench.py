"""1x1 NHWC convolutions of ResNet-50 (bs 256): MIOpen (torch conv2d / convolution_backward,
find mode) vs the hand-written MFMA GEMM (each tile shape) for forward, data-gradient and
weight-gradient. Prints ms and the better of the two per direction."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = "cuda"
B = int(os.environ.get("BATCH", 256))
shapes = [  # (H, Cin, Cout, count per step)
    (56, 64, 64, 1), (56, 64, 256, 4), (56, 256, 64, 2), (56, 256, 128, 1), (28, 128, 512, 5),
    (28, 512, 128, 3), (28, 512, 256, 1), (14, 256, 1024, 7), (14, 1024, 256, 5),
    (14, 1024, 512, 1), (7, 512, 2048, 4), (7, 2048, 512, 2)]


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def splits_for(tiles, K):
    return max(1, min(512 // max(tiles, 1), K // 1024))


tot = {"miopen": 0.0, "best_lw": 0.0, "best": 0.0}
for H, ci, co, cnt in shapes:
    x = torch.randn(B, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(co, ci, 1, 1, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, co, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = B * H * H
    x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
    dy2 = dy.permute(0, 2, 3, 1).reshape(M, co)
    w2 = w.reshape(co, ci)
    flops = 2 * M * ci * co
    mi = {
        "fwd": bench(lambda: F.conv2d(x, w)),
        "dgrad": bench(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])),
        "wgrad": bench(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])),
    }
    lw = {"fwd": {}, "dgrad": {}, "wgrad": {}}
    for t in ("128x128x32", "128x128x64", "256x64x32", "64x256x32", "256x64x64", "64x64x64"):
        lw["fwd"][t] = bench(lambda: G.gemm_ex(x2, ci, True, w2, ci, True, M, co, ci, tile=t))
        lw["dgrad"][t] = bench(lambda: G.gemm_ex(dy2, co, True, w2, ci, False, M, ci, co, tile=t))
        bm, bn = (int(v) for v in t.split("x")[:2])
        tiles = -(-co // bm) * -(-ci // bn)
        for wgs in (512, 1024, 2048):
            sp = max(1, min(wgs // tiles, M // 512))
            lw["wgrad"][f"{t}/s{sp}"] = bench(lambda: G.gemm_ex(
                dy2, co, False, x2, ci, False, co, ci, M, splits=sp, out_bf16=False, tile=t))
    line = f"H{H:3d} {ci:5d}->{co:5d} x{cnt}"
    for d in ("fwd", "dgrad", "wgrad"):
        bt, bv = min(lw[d].items(), key=lambda kv: kv[1])
        tot["miopen"] += mi[d] * cnt
        tot["best_lw"] += bv * cnt
        tot["best"] += min(bv, mi[d]) * cnt
        line += f" | {d} mi {mi[d]:.3f} lw {bv:.3f} ({bt}) {flops / bv / 1e9:5.0f}TF"
    print(line, flush=True)
print({k: round(v, 3) for k, v in tot.items()})
