"""Compute-bound ResNet-50 GEMMs (layer3/4, bs 256): hand-written MFMA kernel (best tile) vs
hipBLASLt through torch.mm, same operand layouts (no transpose copies)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402
from layer_wise_aaai20_amd.ops.block import _splits, _tile_dims  # noqa: E402

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


def best_ours(*args, split=False, M=0, N=0, K=0):
    r = {}
    for t in (1, 2, 3, 4, 5, 6):
        sp = 1
        if split:
            bm, bn = _tile_dims(t)
            sp = _splits(-(-M // bm) * -(-N // bn), K)
        a = list(args)
        a[11] = sp
        a[13] = t
        r[t] = timeit(lambda: lib.gemm_ex(*a))
    t = min(r, key=r.get)
    return r[t], t


for M, C1, C2 in ((50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048),
                  (50176, 512, 256), (12544, 1024, 512)):
    x = torch.randn(M, C1, device="cuda").bfloat16()        # activations [M, Cin]
    w = torch.randn(C2, C1, device="cuda").bfloat16()       # weight [Cout, Cin]
    dy = torch.randn(M, C2, device="cuda").bfloat16()
    fl = 2 * M * C1 * C2 / 1e6
    # forward y = x · wᵀ
    o, t = best_ours(x, C1, True, w, C1, True, M, C2, C1, None, False, 1, True, 0, None, None,
                     True, False)
    b = timeit(lambda: torch.mm(x, w.t()))
    # data gradient dx = dy · w
    o2, t2 = best_ours(dy, C2, True, w, C1, False, M, C1, C2, None, False, 1, True, 0, None, None,
                       True, False)
    b2 = timeit(lambda: torch.mm(dy, w))
    # weight gradient dw = dyᵀ · x (fp32 out for ours)
    o3, t3 = best_ours(dy, C2, False, x, C1, False, C2, C1, M, None, False, 1, False, 0, None,
                       None, True, False, split=True, M=C2, N=C1, K=M)
    b3 = timeit(lambda: torch.mm(dy.t(), x))
    print(f"M{M} {C1}->{C2}: fwd ours {o:.0f}us ({fl / o:.0f} TF, t{t}) blas {b:.0f}us "
          f"({fl / b:.0f} TF) | dgrad ours {o2:.0f} (t{t2}) blas {b2:.0f} | wgrad ours {o3:.0f} "
          f"(t{t3}) blas {b3:.0f}", flush=True)
