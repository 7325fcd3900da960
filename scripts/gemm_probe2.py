"""Probe: forward 1x1-conv GEMM variants (B K- vs N-contiguous, stats epilogue on/off, prologue)
on the bandwidth-bound layer1/layer2 shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

lib = load()


def timeit(fn, n=10):
    fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


for M, N, K in ((802816, 256, 64), (200704, 512, 128), (802816, 64, 256)):
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(N, K, device="cuda").bfloat16()
    Wt = W.t().contiguous()
    sc = torch.rand(K, device="cuda") + 0.5
    sh = torch.randn(K, device="cuda")
    mb = (M * K + M * N) * 2 / 1e6
    print(f"M{M} N{N} K{K}  min {mb:.0f} MB -> {mb / 5e3 * 1e3:.0f} us at 5 TB/s")
    for name, b, ldb, bkc in (("Bkc", W, K, True), ("Bnc", Wt, N, False)):
        for stats in (False, True):
            for pro in (False, True):
                r = {}
                for t in (1, 2, 3, 4, 5, 6, 11, 12, 13):
                    try:
                        r[t] = timeit(lambda: lib.gemm_ex(A, K, True, b, ldb, bkc, M, N, K, None,
                                                          False, 1, True, t, sc if pro else None,
                                                          sh if pro else None, True, stats, None,
                                                          None, False, 0))
                    except RuntimeError:
                        pass
                print(f"  {name} stats={int(stats)} pro={int(pro)}: " +
                      " ".join(f"{t}:{v:.0f}" for t, v in r.items()), flush=True)
