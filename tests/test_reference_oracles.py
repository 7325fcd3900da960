"""Reference-semantics compressor oracles (SURVEY.md §2.2 edge cases)."""
import math

import pytest
import torch

from layer_wise_aaai20_amd.compress import reference as ref


def test_topk_keep_count_off_by_one():
    # n*K integral -> nK + 1 kept (kthvalue(ceil(n(1-K))) then >= thr)
    assert ref.topk_keep_count(1000, 0.001) == 2
    assert ref.topk_keep_count(1000, 0.0015) == 2
    assert ref.topk_keep_count(64, 0.001) == 1      # every layer keeps >= 1
    assert ref.topk_keep_count(10, 0.5) == 6
    assert ref.topk_keep_count(7, 1.0) == 7


@pytest.mark.parametrize("n,K", [(1000, 0.001), (1000, 0.01), (97, 0.3), (5, 0.5), (64, 0.001)])
def test_topk_matches_kthvalue_rule(n, K):
    g = torch.randn(n, generator=torch.Generator().manual_seed(n))
    out = ref.topk(g, K)
    thr = g.abs().kthvalue(math.ceil(n * (1 - K))).values
    exp = g.clone()
    exp[g.abs() < thr] = 0
    assert torch.equal(out, exp)
    assert int((out != 0).sum()) == ref.topk_keep_count(n, K)


def test_topk_ties_kept():
    g = torch.tensor([1.0, 1.0, 1.0, 0.5, 0.1])
    out = ref.topk(g, 0.2)            # keep-count 1, but three tie at the threshold
    assert int((out != 0).sum()) == 3


def test_randomk_count():
    for n, K in [(100, 0.05), (1000, 0.001), (33, 0.5)]:
        out = ref.randomk(torch.ones(n), K, torch.Generator().manual_seed(0))
        assert int(out.sum()) == ref.randomk_keep_count(n, K) == math.ceil(n * K)


def test_thresholds():
    g = torch.tensor([0.5, -2e-3, 1e-4, -1.0, 0.0])
    assert torch.equal(ref.thresholdv(g, 1e-3), torch.tensor([0.5, -2e-3, 0.0, -1.0, 0.0]))
    assert torch.equal(ref.adaptive_threshold(g), torch.tensor([0.5, 0.0, 0.0, -1.0, 0.0]))


def test_terngrad_values_and_zero_guard():
    g = torch.randn(1000)
    out = ref.terngrad(g, torch.Generator().manual_seed(1))
    s = g.abs().max()
    assert set(out.unique().tolist()) <= {-float(s), 0.0, float(s)}
    assert torch.equal(ref.terngrad(torch.zeros(5)), torch.zeros(5))   # no 0/0 NaN (D17)


def test_qsgd_unbiased_and_zero_guard():
    g = torch.randn(256, generator=torch.Generator().manual_seed(2))
    gen = torch.Generator().manual_seed(3)
    acc = torch.zeros(256)
    for _ in range(400):
        acc += ref.random_dithering(g, 4, gen)
    # level spacing ||g||/s ~ 4 -> per-sample std <= 2, std of the 400-mean <= 0.1: 5 sigma
    torch.testing.assert_close(acc / 400, g, rtol=0, atol=0.5)
    assert torch.equal(ref.random_dithering(torch.zeros(4), 255), torch.zeros(4))


def test_dispatch_guards_and_aliases():
    g = torch.randn(50)
    assert torch.equal(ref.compress(g, "Topk", K=0), g)           # falsy K = no compression
    assert torch.equal(ref.compress(g, "Thresholdv", V=None), g)
    assert torch.equal(ref.compress(g, "TopK", K=0.1), ref.topk(g, 0.1))   # README spelling
    assert ref.canonical_method("QSGD") == "RandomDithering"
    with pytest.raises(ValueError):
        ref.compress(g, "Topkk", K=0.1)                            # unknown names raise (D17)


def test_mean_over_ranks():
    a, b = torch.tensor([1.0, 0.0]), torch.tensor([0.0, 3.0])
    assert torch.equal(ref.mean_over_ranks([a, b]), torch.tensor([0.5, 1.5]))
