"""Cost of the BN column-statistics epilogue: every forward 1x1 GEMM shape of the ResNet-50 step
(bs 256) timed with and without EPI_STATS, per tile. usage: python scripts/stats_cost_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

dev = torch.device("cuda", 0)
lib = load()


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


tot = {False: 0.0, True: 0.0}
for m, n, k, cnt in [(802816, 64, 256, 2), (802816, 64, 64, 1), (802816, 256, 64, 4),
                     (802816, 128, 256, 1), (200704, 128, 512, 3), (200704, 512, 128, 4),
                     (50176, 256, 1024, 5), (50176, 1024, 256, 6), (12544, 512, 2048, 2),
                     (12544, 2048, 512, 3), (200704, 256, 512, 1), (50176, 512, 1024, 1)]:
    a = torch.randn(m, k, device=dev).bfloat16()
    b = torch.randn(n, k, device=dev).bfloat16()
    line = []
    best = {}
    for stats in (False, True):
        res = {}
        for t in (2, 5, 21, 22, 23, 24, 12):
            try:
                res[t] = timeit(lambda: lib.gemm_ex(a, k, True, b, k, True, m, n, k, None, False,
                                                    1, True, t, None, None, True, stats, None,
                                                    None, False, 0, None, None, None, None, None))
            except RuntimeError:
                pass
        bt = min(res, key=res.get)
        best[stats] = res[bt]
        tot[stats] += res[bt] * cnt
        line.append(("stats " if stats else "plain ") +
                    " ".join(f"{t}:{v:.1f}" for t, v in res.items()) + f" best {bt}")
    print(f"M{m} N{n} K{k} x{cnt}: " + " | ".join(line) +
          f"  stats cost {best[True] - best[False]:.1f} us", flush=True)
print(f"total best plain {tot[False]:.0f} us, with stats {tot[True]:.0f} us")
