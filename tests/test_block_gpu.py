"""Whole-block fused bottleneck (ops/block.py) vs the plain fp32 PyTorch bottleneck.

The fused path runs bf16 activations through the MFMA GEMM (BN statistics in the epilogue, BN-apply
in the prologue), MIOpen for the 3x3 conv and the fused BN kernels; the reference is
``models.resnet.Bottleneck`` in fp32 on the same (bf16-representable) input and weights. Errors are
compared as relative L2 norms, which is what bf16 rounding through three conv+BN layers allows."""
import copy

import pytest
import torch

from layer_wise_aaai20_amd.models.resnet import Bottleneck, conv1x1, resnet50
from layer_wise_aaai20_amd.ops import block as blk
from layer_wise_aaai20_amd.ops.nn import fuse_resnet, share_bn_counters

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _make(inplanes, planes, stride, down):
    ds = None
    if down:
        ds = torch.nn.Sequential(conv1x1(inplanes, planes * 4, stride),
                                 torch.nn.BatchNorm2d(planes * 4))
    m = Bottleneck(inplanes, planes, stride, ds)
    for bn in [m.bn1, m.bn2, m.bn3] + ([ds[1]] if down else []):
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.normal_(0, 0.2)
    for p in m.parameters():     # bf16-representable weights: both paths see the same values
        p.data = p.data.to(torch.bfloat16).float()
    return m


def _run(m, x, g, block):
    fuse_resnet(m, block=block)
    xb = x.clone().requires_grad_()
    if block:
        assert blk.block_supported(m, xb)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xb)
    y.backward(g.to(y.dtype))
    return m, y, xb.grad


@pytest.mark.parametrize("inplanes,planes,stride,down", [
    (256, 64, 1, False), (64, 64, 1, True), (256, 128, 2, True), (512, 128, 1, False)])
def test_block_matches_reference(inplanes, planes, stride, down):
    """Block path vs fp32: within bf16 noise, and no worse than the per-layer fused path (whose
    error vs fp32 is dominated by bf16 rounding of the gradient and ReLU-mask flips near 0)."""
    torch.manual_seed(0)
    ref = _make(inplanes, planes, stride, down).cuda().to(memory_format=CL)
    mb, ml = copy.deepcopy(ref), copy.deepcopy(ref)
    x = torch.randn(8, inplanes, 14, 14, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=CL)
    xf = x.float().requires_grad_()
    y_ref = ref(xf)
    g = torch.randn_like(y_ref)
    y_ref.backward(g)
    mb, yb, dxb = _run(mb, x, g, True)
    ml, yl, dxl = _run(ml, x, g, False)
    assert yb.dtype == torch.bfloat16 and yb.shape == y_ref.shape
    assert _rel(yb, y_ref) < 1e-2
    pairs = [("dx", dxb, dxl, xf.grad)] + [
        (n, p.grad, q.grad, r.grad) for (n, p), q, r in
        zip(mb.named_parameters(), ml.parameters(), ref.parameters())]
    for n, b, lay, r in pairs:
        eb, el = _rel(b, r), _rel(lay, r)
        assert eb < 0.15, (n, eb)
        assert eb <= 1.1 * el + 5e-3, (n, eb, el)
    for (n, b), (_, c) in zip(mb.named_buffers(), ref.named_buffers()):
        if b.is_floating_point():
            torch.testing.assert_close(b, c, rtol=2e-2, atol=2e-2, msg=n)
        else:
            assert int(b) == int(c), n


def test_block_direct_arena_gradients():
    """With ``_lw_grad_ready`` set (CompressedDDP), weight/BN gradients are accumulated into the
    existing ``.grad`` tensors in place and each parameter is announced exactly once."""
    torch.manual_seed(1)
    m = _make(256, 64, 2, True).cuda().to(memory_format=CL)
    ref = copy.deepcopy(m)
    fuse_resnet(m)
    calls = []
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
        p._lw_grad_ready = lambda q: calls.append(id(q))
    ptrs = {id(p): p.grad.data_ptr() for p in m.parameters()}
    x = torch.randn(4, 256, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    y = m(x.clone().requires_grad_())
    y.float().sum().backward()
    assert sorted(calls) == sorted(id(p) for p in m.parameters())
    for p in m.parameters():
        assert p.grad.data_ptr() == ptrs[id(p)]
    xr = x.float().requires_grad_()
    ref(xr).sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 0.15, n


@pytest.mark.parametrize("inplanes,planes,stride,down", [(256, 64, 1, False), (64, 64, 1, True),
                                                         (512, 128, 1, False),
                                                         (256, 128, 2, True)])
def test_fused_bn3_backward_matches_three_pass_block(inplanes, planes, stride, down, monkeypatch):
    """Stage-1/2 bottlenecks (with and without downsample) with BN3's — and, without downsample,
    BN1's — backward fused into their two GEMMs (csrc/bnfuse.hip), and a2 = relu(bn2(c2)) never
    materialised, give the three-pass block's output, input and parameter gradients to bf16 /
    summation-order noise."""
    torch.manual_seed(3)
    ref = _make(inplanes, planes, stride, down).cuda().to(memory_format=CL)
    x = torch.randn(8, inplanes, 28, 28, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=CL)
    gy = torch.randn(8, 4 * planes, 28 // stride, 28 // stride, device="cuda").contiguous(
        memory_format=CL)
    outs = {}
    for fuse in (True, False):
        monkeypatch.setattr(blk, "FUSE_BNBWD", fuse)
        m, y, gx = _run(copy.deepcopy(ref), x.float(), gy, True)
        outs[fuse] = (y.float(), gx.float(), [p.grad.float() for p in m.parameters()])
    # the fused path's forward never materialises a2 (conv3 applies BN2 in its GEMM prologue,
    # possibly on another tile than the plain GEMM): the outputs agree to rounding
    assert _rel(outs[True][0], outs[False][0]) < 1e-2
    assert _rel(outs[True][1], outs[False][1]) < 2e-2
    for a, b in zip(outs[True][2], outs[False][2]):
        assert _rel(a, b) < 2e-2


def test_resnet50_block_vs_layer_path():
    """Whole ResNet-50 step. Deep BN-parameter gradients of a random-init net are chaotic in bf16
    (both fused paths sit ~100 % away from fp32 on some), so the check is statistical: the loss
    matches and the block path's per-parameter error distribution vs fp32 is no worse than the
    per-layer path's."""
    import statistics
    torch.manual_seed(2)
    ref = resnet50().cuda()
    for p in ref.parameters():
        p.data = p.data.to(torch.bfloat16).float()
    paths = {"block": copy.deepcopy(ref), "layer": copy.deepcopy(ref)}
    ref = ref.to(memory_format=CL)
    x = torch.randn(16, 3, 96, 96, device="cuda").to(torch.bfloat16).float()
    x = x.contiguous(memory_format=CL)
    t = torch.randint(0, 1000, (16,), device="cuda")
    ref_loss = torch.nn.functional.cross_entropy(ref(x), t)
    ref_loss.backward()
    errs, losses = {}, {}
    for name, m in paths.items():
        fuse_resnet(m, block=name == "block")
        m.to(memory_format=CL)
        share_bn_counters(m)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x)
        loss = torch.nn.functional.cross_entropy(out.float(), t)
        loss.backward()
        losses[name] = float(loss)
        errs[name] = [_rel(p.grad, q.grad) for p, q in zip(m.parameters(), ref.parameters())]
    assert abs(losses["block"] - float(ref_loss)) < 2e-2 * abs(float(ref_loss))
    mb, ml = statistics.median(errs["block"]), statistics.median(errs["layer"])
    assert mb <= 1.2 * ml + 0.02, (mb, ml)
    assert errs["block"][-1] < 0.05            # fc.bias: only the softmax output enters


@pytest.mark.parametrize("pooled", [True, False])
@pytest.mark.parametrize("shape", [(4, 64, 32, 32), (2, 64, 15, 17), (2, 64, 112, 112), (3, 128, 28, 28)])
def test_stem_bn_relu_pool_matches_layers(shape, pooled, monkeypatch, zero_gamma=False):
    """Fused BN+ReLU+max-pool stem vs FusedBatchNorm2d(relu) + nn.MaxPool2d, with the backward's
    statistics taken from the pooled side (csrc/bn.hip k_stem_pool_reduce_out) or from the
    full-resolution conv output."""
    from layer_wise_aaai20_amd.ops import nn as NN
    from layer_wise_aaai20_amd.ops.nn import stem_bn_relu_pool, to_fused_bn
    monkeypatch.setattr(NN, "STEM_POOLED", pooled)
    torch.manual_seed(3)
    C = shape[1]
    bn_a = torch.nn.BatchNorm2d(C).cuda()
    bn_a.weight.data.uniform_(-1.0, 1.5)          # negative gammas too
    bn_a.bias.data.normal_(0, 0.3)
    if zero_gamma:                                # scale 0: x is not recoverable from the pooled map
        bn_a.weight.data[::5] = 0.0
        bn_a.bias.data[::5] = bn_a.bias.data[::5].abs() + 0.1
    bn_b = copy.deepcopy(bn_a)
    to_fused_bn(bn_b, relu=True)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    c = torch.randn(*shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    ca, cb = c.clone().requires_grad_(), c.clone().requires_grad_()
    ya = stem_bn_relu_pool(ca, bn_a, pool)
    yb = pool(bn_b(cb))
    torch.testing.assert_close(ya.float(), yb.float(), rtol=0, atol=0)
    g = torch.randn_like(yb, dtype=torch.float32).to(torch.bfloat16)
    ya.backward(g)
    yb.backward(g)
    assert _rel(ca.grad, cb.grad) < 2e-2
    assert _rel(bn_a.weight.grad, bn_b.weight.grad) < 2e-2
    assert _rel(bn_a.bias.grad, bn_b.bias.grad) < 2e-2
    torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("shape", [(4, 64, 32, 32), (2, 64, 15, 17)])
def test_stem_pool_backward_zero_gamma(shape, monkeypatch):
    """Channels with gamma == 0 (pooled map constant): the pooled-side statistics pass gathers x
    at the argmax for them instead of inverting the affine."""
    test_stem_bn_relu_pool_matches_layers(shape, True, monkeypatch, zero_gamma=True)


@pytest.mark.parametrize("shape", [(4, 64, 32, 32), (2, 64, 112, 112)])
def test_stem_pool_backward_ill_conditioned_channels(shape, monkeypatch):
    """|gamma| ~ 1e-3 with beta ~ 0.5: recovering x - mean from the bf16 pooled value would put
    a per-channel bias into dgamma. Per channel, the pooled-side pass must agree with the
    full-resolution pass (which reads x itself). An fp32 torch reference pins the well-conditioned
    channels only: on the others bn(x) ~ beta +- 1e-3 rounds to a handful of bf16 values, so the
    bf16 forward's max-pool argmax (which both backward passes share) and fp32's pick different
    pixels and no 16-bit implementation can match it."""
    from layer_wise_aaai20_amd.ops import nn as NN
    from layer_wise_aaai20_amd.ops.nn import stem_bn_relu_pool
    torch.manual_seed(5)
    C = shape[1]
    bn0 = torch.nn.BatchNorm2d(C).cuda()
    bn0.weight.data.uniform_(0.5e-3, 2e-3)
    bn0.weight.data[1::2] *= -1
    good = torch.arange(0, C, 4)
    bn0.weight.data[good] = torch.empty(len(good), device="cuda").uniform_(0.5, 1.5)
    bn0.bias.data.uniform_(0.3, 0.7)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    c = torch.randn(*shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(shape[0], C, (shape[2] + 1) // 2, (shape[3] + 1) // 2, device="cuda")
    g = g.to(torch.bfloat16)
    res = {}
    for pooled in (True, False):
        monkeypatch.setattr(NN, "STEM_POOLED", pooled)
        bn = copy.deepcopy(bn0)
        ca = c.clone().requires_grad_()
        stem_bn_relu_pool(ca, bn, pool).backward(g)
        res[pooled] = (ca.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone())
    bnr = copy.deepcopy(bn0).float()
    cr = c.float().requires_grad_()
    pool(torch.relu(bnr(cr))).backward(g.float())
    (dxp, dgp, dbp), (dxf, dgf, dbf) = res[True], res[False]
    # pooled-side vs full-resolution: every channel (the ill-conditioned ones included)
    # (dgamma is a cancelling sum: the two passes' rounding differs by ~1e-3 of its largest
    # channel; the bias the pooled inversion would add on an ill-conditioned channel is O(1) of it)
    sc = float(dgf.abs().max())
    for ch in range(C):
        assert abs(float(dgp[ch] - dgf[ch])) < 1e-2 * sc, (ch, dgp[ch], dgf[ch])
        assert _rel(dxp[:, ch], dxf[:, ch]) < 2e-2, ch
    torch.testing.assert_close(dbp, dbf, rtol=1e-2, atol=1e-2 * dbf.abs().max())
    # both against fp32 torch on the well-conditioned channels
    for (_, dg, db) in res.values():
        ref = bnr.weight.grad[good]
        assert ((dg[good] - ref).abs() < 3e-2 * ref.abs().max() + 1e-3).all(), \
            (dg[good] - ref).abs().max()
        torch.testing.assert_close(db[good], bnr.bias.grad[good], rtol=2e-2,
                                   atol=2e-2 * db[good].abs().max())
    # (dx is not compared with fp32 elementwise: bf16 ties in a 3x3 window send a pixel's
    # gradient to a different argmax than fp32 picks; test_stem_bn_relu_pool_matches_layers
    # pins dx against the unfused bf16 layers instead)


@pytest.mark.parametrize("direct", [False, True])
def test_fused_stem_backward_matches_two_pass(direct, monkeypatch):
    """The stem backward with the pool / BN apply fused into the 7x7/2 weight gradient
    (csrc/stemfuse.hip) vs the two-pass path (k_stem_pool_bwd_s2 + implicit-GEMM wgrad): same
    forward, conv-weight and BN-parameter gradients within summation-order / bf16 noise, also
    when the gradients go straight into arena views (CompressedDDP's direct path)."""
    from layer_wise_aaai20_amd.ops import nn as NN
    torch.manual_seed(5)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda()
    conv.weight.data = conv.weight.data.to(torch.bfloat16).float()
    bn = torch.nn.BatchNorm2d(64).cuda()
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.normal_(0, 0.2)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 4, 224, 224, device="cuda").to(torch.bfloat16)
    x[:, 3] = 0
    x = x.contiguous(memory_format=CL)
    gy = torch.randn(2, 64, 56, 56, device="cuda").contiguous(memory_format=CL)
    res = {}
    for fuse in (True, False):
        monkeypatch.setattr(blk, "FUSE_BNBWD", fuse)
        c2, b2 = copy.deepcopy(conv), copy.deepcopy(bn)
        calls = []
        if direct:
            for p in (c2.weight, b2.weight, b2.bias):
                p.grad = torch.zeros_like(p) if p is not c2.weight else \
                    torch.zeros_like(p).contiguous(memory_format=CL)
                p._lw_grad_ready = lambda q: calls.append(id(q))
        y = NN.stem_conv_bn_relu_pool(x, c2, b2, pool)
        y.backward(gy.to(y.dtype))
        if direct:
            assert sorted(calls) == sorted(id(p) for p in (c2.weight, b2.weight, b2.bias))
        res[fuse] = (y.float(), c2.weight.grad.float(), b2.weight.grad.float(),
                     b2.bias.grad.float())
    assert torch.equal(res[True][0], res[False][0])
    for a, b in zip(res[True][1:], res[False][1:]):
        assert _rel(a, b) < 1e-2
