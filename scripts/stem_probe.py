"""Time the ResNet-50 stem kernels at bs 256 / 224 px: the direct 7x7/2 convolution
(csrc/conv.hip k_stem_conv7; LWAAAI_STEM_TPW / LWAAAI_STEM_OCC are read by the library) and the
pool/BN backward with its statistics from the pooled side vs from the full-resolution conv output
(csrc/bn.hip k_stem_pool_reduce_out), with the largest difference between the two backwards.
usage: python scripts/stem_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

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


lib = load()
tag = (f"tpw={os.environ.get('LWAAAI_STEM_TPW', 'auto')} occ={os.environ.get('LWAAAI_STEM_OCC', '4')} "
       f"pf={os.environ.get('LWAAAI_STEM_PF', '0')}")
xs = torch.randn(256, 4, 224, 224, device=dev).bfloat16().contiguous(memory_format=CL)
ws = torch.randn(64, 3, 7, 7, device=dev).bfloat16().contiguous(memory_format=CL)
CV.TUNER.pick = lambda key, run, cands, default: CV.STEM_DIRECT
us = timeit(lambda: CV.conv_fwd(xs, ws, 2, 3, stats=True))
print(f"stem conv direct {tag}: {us:.1f} us", flush=True)

C = 64
c = torch.randn(256, C, 112, 112, device=dev).bfloat16().contiguous(memory_format=CL)
gamma = torch.rand(C, device=dev) + 0.5
beta = torch.randn(C, device=dev) * 0.3
rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
mean, invstd, ss = lib.bn_stats(c, None, gamma, beta, rm, rv, 0.1, 1e-5)
out, idx = lib.stem_pool_fwd(c, ss, 3, 2, 1)
dout = torch.randn_like(out)
res = {}
for name, pooled in (("full", None), ("pooled", out)):
    us = timeit(lambda: lib.stem_pool_bwd(dout, idx, c, ss, gamma, mean, invstd, 3, 2, 1, None,
                                          None, pooled))
    res[name] = lib.stem_pool_bwd(dout, idx, c, ss, gamma, mean, invstd, 3, 2, 1, None, None,
                                  pooled)
    print(f"stem pool bwd {name}: {us:.1f} us", flush=True)
for i, what in enumerate(("dx", "dgamma", "dbeta")):
    a, b = res["full"][i].float(), res["pooled"][i].float()
    print(f"  {what}: max |diff| {float((a - b).abs().max()):.3e} "
          f"(max |ref| {float(b.abs().max()):.3e})", flush=True)
