"""Exact layer-wise Top-K selection on real ResNet-50 gradients (the headline configuration, EF
off): for 3 training steps, every one of the 161 layers' decoded gradient equals the reference
compressor ``ref.topk`` (``kthvalue`` threshold, ``>=`` keeps every tie; ``CIFAR10/core.py:178-183``)
bit for bit. All gradients reach the arena in fp32 (the MFMA convolutions / GEMMs accumulate
their weight gradients in fp32 straight into it), so value ties at the threshold are as rare as
in the reference's fp32 path and the tie slots of the sparse payload suffice. The decode writes
the arena gradient (``fused_sgd=False``): the fused decode + SGD step never materialises it."""
import pytest
import torch

from layer_wise_aaai20_amd.compress import reference as ref

pytestmark = pytest.mark.gpu


def test_resnet50_layerwise_topk_bit_exact(monkeypatch):
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    torch.manual_seed(0)
    K = 0.001
    tr = build_trainer("resnet50", device="cuda", compress="layerwise", method="Topk", K=K,
                       bn0=False, fused_sgd=False)
    eng = tr.ddp.engine
    raw = {}
    for bi, codec in enumerate(eng.codecs):
        real = codec.compress

        def capture(g, ef, step, real=real, bi=bi):
            raw[bi] = g.detach().clone()          # the bucket's gradient before selection
            return real(g, ef, step)
        codec.compress = capture
    gen = torch.Generator(device="cuda").manual_seed(1)
    for step in range(3):
        x = torch.randint(0, 256, (32, 96, 96, 3), dtype=torch.uint8, device="cuda", generator=gen)
        t = torch.randint(0, 1000, (32,), device="cuda", generator=gen)
        tr.step(x, t)
        torch.cuda.synchronize()
        assert len(raw) == len(eng.buckets)
        checked = 0
        for b in eng.buckets:
            r = raw[b.index]
            for seg in eng.arena.segments[b.seg_lo:b.seg_hi]:
                o = seg.offset - b.start
                g_raw = r[o:o + seg.numel]
                got = eng.arena.grad[seg.offset:seg.offset + seg.numel]
                exp = ref.topk(g_raw, K)
                assert torch.equal(got, exp), (step, seg.name,
                                               int((got != exp).sum()), seg.numel)
                checked += 1
        assert checked == 161
        raw.clear()
