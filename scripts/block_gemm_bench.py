"""Every MFMA GEMM call of one ResNet-50 block-fused training step (bs 256, 224 px), replayed in
isolation for every tile shape: time, achieved HBM GB/s against the minimum bytes of the call,
TFLOP/s, and the tile the run-time tuner chose. Grouped by role (fwd / dgrad / wgrad)."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops import block as blk  # noqa: E402
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402
from layer_wise_aaai20_amd.train.imagenet import build_trainer  # noqa: E402

B = int(os.environ.get("BATCH", 256))
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
calls = []
orig = blk.gemm


def rec(A, lda, a_kc, Bm, ldb, b_kc, M, N, K, **kw):
    calls.append(dict(A=A, lda=lda, a_kc=a_kc, B=Bm, ldb=ldb, b_kc=b_kc, M=M, N=N, K=K,
                      kw={k: v for k, v in kw.items() if k in ("out_bf16", "stats", "pro",
                                                               "pro_on_a", "split_k")},
                      addend=kw.get("addend") is not None))
    return orig(A, lda, a_kc, Bm, ldb, b_kc, M, N, K, **kw)


tr = build_trainer("resnet50", device=dev, compress="layerwise", method="Topk", K=0.001)
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
tgt = torch.randint(0, 1000, (B,), device=dev)
tr.step(imgs, tgt)
blk.gemm = rec
tr.step(imgs, tgt)
blk.gemm = orig
torch.cuda.synchronize()
lib = load()


def timeit(fn, n=10):
    fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


groups = collections.OrderedDict()
for c in calls:
    role = "wgrad" if c["kw"].get("split_k") else ("fwd" if c["b_kc"] else "dgrad")
    key = (role, c["M"], c["N"], c["K"], c["a_kc"], c["b_kc"], c["kw"].get("stats", False),
           c["kw"].get("pro") is not None, c["addend"])
    groups.setdefault(key, [c, 0])[1] += 1

tot = collections.defaultdict(float)
for key, (c, cnt) in groups.items():
    role, M, N, K = key[:4]
    pro = c["kw"].get("pro")
    ps, ph = (pro[0], pro[1]) if pro is not None else (None, None)
    ob = c["kw"].get("out_bf16", True)
    res = {}
    for tile in blk.TILES:
        sp = 1
        if c["kw"].get("split_k"):
            bm, bn = blk._tile_dims(tile)
            sp = blk._splits(-(-M // bm) * -(-N // bn), K)
        res[tile] = timeit(lambda: lib.gemm_ex(c["A"], c["lda"], c["a_kc"], c["B"], c["ldb"],
                                               c["b_kc"], M, N, K, None, False, sp, ob, tile, ps,
                                               ph, c["kw"].get("pro_on_a", True),
                                               c["kw"].get("stats", False), None, None, False, 0))
    best = min(res, key=res.get)
    t = res[best]
    obytes = M * N * (2 if ob else 4)
    nbytes = 2 * (M * K + N * K) + obytes + (M * N * 2 if c["addend"] else 0)
    tot[role] += t * cnt
    print(f"{role:5s} M{M:7d} N{N:5d} K{K:7d} x{cnt:2d} stats={int(key[6])} pro={int(key[7])} "
          f"add={int(key[8])}: {t * 1e3:7.1f} us  {nbytes / t / 1e6:6.0f} GB/s  "
          f"{2 * M * N * K / t / 1e9:5.0f} TF  tile {best} "
          f"(tuned {blk.TUNER.best.get(next(k for k in blk.TUNER.best if k[:3] == (M, N, K)), '?')})  "
          + " ".join(f"{k}:{v * 1e3:.0f}" for k, v in res.items()), flush=True)
print({k: round(v, 3) for k, v in tot.items()}, "total", round(sum(tot.values()), 3))
