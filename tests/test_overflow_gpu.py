"""Device-side overflow accounting (``GradSyncEngine.read_overflow``).

* Top-K ties: the reference keeps every element ``>=`` the k-th largest (``CIFAR10/core.py:178-183``).
  The payload has a tie slack of ``max(16, ceil(m/64))`` slots per layer; ties beyond it stay in
  the error-feedback residual and are now counted, not silently dropped.
* Fixed-capacity threshold wire: hits beyond the per-segment capacity are counted and kept in
  EF. The GPU kernels match the CPU mirror bit for bit."""
import numpy as np
import pytest
import torch

from layer_wise_aaai20_amd.compress import codecs as C
from layer_wise_aaai20_amd.compress.plan import SegPlan

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [3000, 200000])          # small (one-block) and large (radix) paths
def test_topk_tie_overflow_counted(n):
    plan = SegPlan([0], [n])
    codec = C.TopkCodec(plan, 1, 0, K=0.01, error_feedback=True)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    codec.overflow = cnt
    g = torch.ones(n, device="cuda")                    # every element ties at the threshold
    ef = torch.zeros(n, device="cuda")
    codec.compress(g, ef, 0)
    torch.cuda.synchronize()
    cap = int(codec.cap[0])
    assert int(cnt.item()) == n - cap
    assert int((ef != 0).sum()) == n - cap              # the overflow stayed in the residual


@pytest.mark.parametrize("adaptive", [False, True])
def test_fixed_capacity_threshold_matches_cpu_mirror(adaptive):
    sizes = [5000, 70000, 300]
    plan = SegPlan(np.cumsum([0] + sizes[:-1]).tolist(), sizes)
    mk = lambda: C.ThresholdCodec(plan, 1, 0, V=0.5, adaptive=adaptive,          # noqa: E731
                                  error_feedback=True, max_density=0.02)
    gpu, cpu = mk(), mk()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.overflow = cnt
    torch.manual_seed(0)
    g = torch.randn(sum(sizes))
    e = torch.randn(sum(sizes)) * 0.1
    gg, eg = g.cuda(), e.cuda()
    out_g = gpu.compress(gg, eg, 0)
    out_c = cpu.compress(g.clone(), e.clone(), 0)
    torch.cuda.synchronize()
    assert torch.equal(out_g.cpu(), out_c)
    ecpu = e.clone()
    cpu2 = mk()
    cpu2.compress(g.clone(), ecpu, 0)
    assert torch.equal(eg.cpu(), ecpu)
    # overflow = hits the capacity could not carry
    x = g + e
    hits = 0
    for s, (o, n) in enumerate(zip(plan.offsets, sizes)):
        a = x[o:o + n].abs()
        thr = float(a.max()) * 0.5 if adaptive else 0.5
        hits += max(0, int(((a >= thr) & (x[o:o + n] != 0)).sum()) - int(gpu.cap[s]))
    assert int(cnt.item()) == hits
