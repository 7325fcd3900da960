"""Hand-written MFMA implicit-GEMM convolutions (csrc/conv.hip) vs a plain fp32 torch reference:
forward / data gradient / weight gradient for every 3x3 / 7x7 / 5x5 shape of the reference models
(ResNet-50 bottlenecks and stem, ResNet-9, VGG-16, AlexNet; batch reduced), the fused BN-apply+ReLU
prologues, the column-statistics epilogue and in-place accumulation into a channels_last arena."""
import pytest
import torch
import torch.nn.functional as F

from layer_wise_aaai20_amd.ops import conv as CV

pytestmark = pytest.mark.gpu
CL = torch.channels_last

# (N, Cin, Cout, H, k, stride, pad): ResNet-50 @224 3x3 (batch 4), stem, CIFAR nets
SHAPES = [
    (4, 64, 64, 56, 3, 1, 1), (4, 128, 128, 56, 3, 2, 1), (4, 128, 128, 28, 3, 1, 1),
    (4, 256, 256, 28, 3, 2, 1), (4, 256, 256, 14, 3, 1, 1), (4, 512, 512, 14, 3, 2, 1),
    (4, 512, 512, 7, 3, 1, 1),
    (2, 3, 64, 224, 7, 2, 3),                                   # ResNet-50 stem
    (8, 3, 64, 32, 3, 1, 1), (8, 64, 128, 32, 3, 1, 1), (8, 128, 256, 16, 3, 1, 1),
    (8, 256, 512, 8, 3, 1, 1), (8, 512, 512, 2, 3, 1, 1),        # ResNet-9 / VGG-16
    (8, 64, 192, 8, 5, 1, 2), (8, 3, 64, 32, 11, 4, 5),          # AlexNet-style 5x5 / 11x11
    (3, 24, 40, 13, 3, 2, 0), (3, 16, 24, 9, 1, 2, 0),           # odd sizes, no padding
]


def _inputs(N, C, Co, H, k, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Co, C, k, k, device="cuda", generator=g) / (C * k * k) ** 0.5).bfloat16()
    return x.contiguous(memory_format=CL), w.contiguous(memory_format=CL)


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_fwd(shape):
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k)
    y, _ = CV.conv_fwd(x, w, s, p)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    assert y.shape == ref.shape
    _close(y, ref, 1e-2)


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] % 8 == 0],
                         ids=[str(s) for s in SHAPES if s[1] % 8 == 0])
def test_conv_dgrad(shape):
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 1)
    xf = x.float().requires_grad_()
    ref = F.conv2d(xf, w.float(), stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    dx = CV.conv_dgrad(dy.contiguous(memory_format=CL), w, (H, H), s, p)
    assert dx.shape == x.shape
    _close(dx, xf.grad, 1e-2)


@pytest.mark.parametrize("layout", ["nkc", "kc"])
@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] % 8 == 0],
                         ids=[str(s) for s in SHAPES if s[1] % 8 == 0])
def test_conv_dgrad_layouts(shape, layout, monkeypatch):
    """Both weight layouts the dgrad tuner chooses between (the transposing-read [K][C] pack and
    the K-contiguous [C][K] pack, parity classes padded to one row stride), every tile, with and
    without an in-place addend."""
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 2)
    xf = x.float().requires_grad_()
    ref = F.conv2d(xf, w.float(), stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    for tile in CV.ROW_TILES:
        monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default: (layout, tile))
        dx = CV.conv_dgrad(dy.contiguous(memory_format=CL), w, (H, H), s, p)
        _close(dx, xf.grad, 1e-2)
        rows = torch.randn(N * H * H, C, device="cuda").bfloat16()
        base = rows.clone()
        CV.conv_dgrad(dy.contiguous(memory_format=CL), w, (H, H), s, p, out=rows, addend=rows)
        got = rows.view(N, H, H, C).permute(0, 3, 1, 2).float()
        _close(got, xf.grad + base.view(N, H, H, C).permute(0, 3, 1, 2).float(), 1e-2)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_wgrad(shape):
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 2)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    dw = CV.conv_wgrad(dy.contiguous(memory_format=CL), x, tuple(w.shape), s, p)
    assert dw.shape == w.shape
    _close(dw, wf.grad, 2e-3)


def test_wgrad_accumulates_into_channels_last_arena_view():
    N, C, Co, H, k, s, p = 4, 64, 128, 28, 3, 2, 1
    x, w = _inputs(N, C, Co, H, k, 3)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    arena = torch.full((Co * C * k * k + 64,), 0.5, device="cuda")
    view = arena[32:32 + Co * C * k * k].as_strided(w.shape, (C * k * k, 1, k * C, C))
    assert view.is_contiguous(memory_format=CL)
    CV.conv_wgrad(dy.contiguous(memory_format=CL), x, tuple(w.shape), s, p, out=view)
    _close(view - 0.5, wf.grad, 2e-3)
    assert torch.all(arena[:32] == 0.5) and torch.all(arena[32 + Co * C * k * k:] == 0.5)


@pytest.mark.parametrize("shape", [(4, 64, 64, 56, 3, 1, 1), (4, 128, 128, 56, 3, 2, 1),
                                   (4, 256, 256, 14, 3, 1, 1)])
def test_bn_prologue_and_stats_epilogue(shape):
    """conv(relu(x*scale+shift)) with the affine in the staging prologue (padding stays zero),
    column statistics of the bf16 output, and the weight gradient with the same prologue."""
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 4)
    scale = torch.rand(C, device="cuda") + 0.5
    shift = torch.randn(C, device="cuda") * 0.5
    a = torch.relu(x.float() * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)).bfloat16()
    y, st = CV.conv_fwd(x, w, s, p, pro=(scale, shift), stats=True)
    ref = F.conv2d(a.float(), w.float(), stride=s, padding=p)
    _close(y, ref, 1e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, Co)
    tot = st.sum(0)
    torch.testing.assert_close(tot[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(tot[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    wf = w.float().requires_grad_()
    r2 = F.conv2d(a.float(), wf, stride=s, padding=p)
    dy = torch.randn_like(r2).bfloat16()
    r2.backward(dy.float())
    dw = CV.conv_wgrad(dy.contiguous(memory_format=CL), x, tuple(w.shape), s, p,
                       pro=(scale, shift))
    _close(dw, wf.grad, 2e-3)


def test_mfma_conv2d_module_matches_torch():
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(64, 128, 3, stride=2, padding=1, bias=True).cuda()
    m = torch.nn.Conv2d(64, 128, 3, stride=2, padding=1, bias=True).cuda()
    m.load_state_dict(ref.state_dict())
    with torch.no_grad():
        ref.weight.copy_(ref.weight.bfloat16().float())
    CV.to_mfma_conv(m)
    m = m.to(memory_format=CL)
    x = torch.randn(4, 64, 20, 20, device="cuda").bfloat16().float()
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    y = m(xa)
    yr = ref(xb)
    _close(y, yr, 1e-2)
    g = torch.randn_like(yr)
    y.float().backward(g)
    yr.backward(g.bfloat16().float())
    _close(xa.grad, xb.grad, 2e-2)
    _close(m.weight.grad, ref.weight.grad, 5e-3)
    _close(m.bias.grad, ref.bias.grad, 5e-3)


@pytest.mark.parametrize("cin,cout,hw,relu", [(64, 128, 16, True), (128, 64, 8, True),
                                              (3, 64, 32, True), (256, 256, 4, False)])
def test_conv_bias_relu_epilogue_matches_torch(cin, cout, hw, relu):
    """Conv2d + bias + ReLU with bias and ReLU in the MFMA epilogue and the fused
    mask / bias-gradient backward kernel (the VGG / AlexNet features pattern)."""
    torch.manual_seed(cin + cout)
    ref = torch.nn.Conv2d(cin, cout, 3, padding=1, bias=True).cuda()
    m = torch.nn.Conv2d(cin, cout, 3, padding=1, bias=True).cuda()
    with torch.no_grad():
        ref.bias.normal_(0, 0.5)
        ref.weight.copy_(ref.weight.bfloat16().float())
    m.load_state_dict(ref.state_dict())
    CV.to_mfma_conv(m)
    m.fuse_relu = relu
    x = torch.randn(8, cin, hw, hw, device="cuda").bfloat16().float()
    xa = x.clone().requires_grad_(cin % 8 == 0)     # (an image input needs no gradient)
    xb = x.clone().requires_grad_(cin % 8 == 0)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xa)
    yr = ref(xb)
    yr = F.relu(yr) if relu else yr
    _close(y.float(), yr, 1e-2)
    g = torch.randn_like(yr).bfloat16().float()
    y.float().backward(g)
    # the reference masks with the bf16-rounded output the fused backward sees
    yr.backward(g * (y.detach().float() > 0).float() if relu else g)
    _close(m.weight.grad, ref.weight.grad, 5e-3)
    _close(m.bias.grad, ref.bias.grad, 5e-3)
    if cin % 8 == 0:
        _close(xa.grad, xb.grad, 2e-2)


def test_fuse_convs_folds_sequential_relu():
    from layer_wise_aaai20_amd.models.cifar import vgg16
    net = CV.fuse_convs(vgg16())
    convs = [m for m in net.modules() if isinstance(m, CV.MFMAConv2d)]
    assert len(convs) == 13 and all(getattr(c, "fuse_relu", False) for c in convs)
    assert not any(isinstance(m, torch.nn.ReLU) for m in net.features.modules())
    from layer_wise_aaai20_amd.ops.nn import ReluMaxPool2d
    assert sum(isinstance(m, ReluMaxPool2d) for m in net.features.modules()) == 5


@pytest.mark.parametrize("shape,k,s,p", [((16, 64, 32, 32), 2, 2, 0), ((8, 512, 2, 2), 2, 2, 0),
                                         ((4, 64, 56, 56), 3, 2, 1)])
def test_relu_pool_matches_torch(shape, k, s, p):
    """ReluMaxPool2d (pool + the preceding ReLU's backward mask in one kernel) vs torch."""
    from layer_wise_aaai20_amd.ops.nn import ReluMaxPool2d
    torch.manual_seed(shape[1])
    a = F.relu(torch.randn(*shape, device="cuda")).bfloat16().contiguous(memory_format=CL)
    pool = torch.nn.MaxPool2d(k, s, p)
    pool.__class__ = ReluMaxPool2d
    xa = a.clone().requires_grad_()
    y = pool(xa)
    xr = a.float().requires_grad_()
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr)
    g = torch.randn_like(yr).bfloat16()
    y.backward(g)
    yr.backward(g.float())
    # torch routes a window of zeros to its first zero; the fused kernel also applies the ReLU
    # mask (x > 0), so compare on the pixels that are positive
    m = a.float() > 0
    torch.testing.assert_close(xa.grad.float() * m, xr.grad * m, atol=1e-2, rtol=1e-2)
    assert float(xa.grad.float()[~m].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(64, 32, 3, 1, 1), (48, 24, 3, 2, 1), (40, 16, 1, 2, 0),
                                   (16, 8, 7, 2, 3), (24, 16, 1, 1, 0)])
def test_pack_dgrad_kc_matches_torch(shape):
    """One-launch K-contiguous data-gradient weight pack vs the same slabs built with torch."""
    co, c, k, s, p = shape
    H = 11
    w = torch.randn(co, c, k, k, device="cuda").bfloat16().contiguous(memory_format=CL)
    classes = CV._dgrad_classes(H, H, k, k, s, s, p, p)
    packed, offs, kmax = CV.pack_dgrad_weight_kc(w, classes, s, s)
    wt = w.permute(1, 2, 3, 0)                                   # [C, R, S, Co]
    ref = torch.zeros(len(classes), c, kmax, dtype=torch.bfloat16, device="cuda")
    for i, (ch, cw, r0, s0, TR, TS, *_r) in enumerate(classes):
        slab = wt[:, r0::s][:, :TR][:, :, s0::s][:, :, :TS].reshape(c, TR * TS * co)
        ref[i, :, :slab.shape[1]] = slab
    assert offs == [i * c * kmax for i in range(len(classes))]
    assert torch.equal(packed.view(len(classes), c, kmax), ref)


BIG_SHAPES = [(4, 64, 64, 56, 3, 1, 1), (4, 128, 128, 56, 3, 2, 1), (4, 128, 128, 28, 3, 1, 1),
              (4, 256, 256, 14, 3, 1, 1), (4, 512, 512, 7, 3, 1, 1), (3, 64, 136, 9, 3, 1, 0),
              (2, 192, 64, 11, 5, 1, 2)]


@pytest.mark.parametrize("shape", BIG_SHAPES, ids=[str(s) for s in BIG_SHAPES])
def test_conv_big_tiles(shape, monkeypatch):
    """The 256x256 / 256x128 8-wave LDS-DMA tiles with the im2col row gather (gemm_big.hip GA):
    forward (+ column statistics, + bias/ReLU epilogue) and the stride-1 data gradient on the
    K-contiguous weight pack, against fp32 torch and bit-identical to the 128x128x64 DMA tile
    (same per-element MFMA accumulation order); row counts off the 256 grid, padding 0 / 1 / 2,
    N below the tile width."""
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 5)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    pick = CV.TUNER.pick
    outs = {}
    bias = torch.randn(Co, device="cuda")
    for tile in (2, 21, 22):
        monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default: tile)
        y, st = CV.conv_fwd(x, w, s, p, stats=True)
        _close(y, ref, 1e-2)
        yf = y.float().permute(0, 2, 3, 1).reshape(-1, Co)
        tot = st.sum(0)
        torch.testing.assert_close(tot[0], yf.sum(0), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(tot[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
        yb, _ = CV.conv_fwd(x, w, s, p, bias=bias, relu=True)
        _close(yb, torch.relu(ref + bias.view(1, -1, 1, 1)), 1e-2)
        outs[tile] = (y, yb)
    for tile in (21, 22):
        assert torch.equal(outs[tile][0], outs[2][0]) and torch.equal(outs[tile][1], outs[2][1])
    if s != 1:
        return
    # data gradient of conv(x2: Co -> C channels): the gathered tensor dy has C % 64 == 0 channels
    x2, w2 = _inputs(N, Co, C, H, k, 6)
    xf = x2.float().requires_grad_()
    r2 = F.conv2d(xf, w2.float(), stride=1, padding=p)
    dy = torch.randn_like(r2).bfloat16().contiguous(memory_format=CL)
    r2.backward(dy.float())
    dxs = {}
    for tile in (2, 21, 22):
        monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default: ("kc", tile))
        dxs[tile] = CV.conv_dgrad(dy, w2, (H, H), 1, p)
        _close(dxs[tile], xf.grad, 1e-2)
    assert torch.equal(dxs[21], dxs[2]) and torch.equal(dxs[22], dxs[2])
    monkeypatch.setattr(CV.TUNER, "pick", pick)


def test_conv_big_tiles_are_tuner_candidates(monkeypatch):
    """The tuner is offered the big tiles exactly where the kernel supports them."""
    seen = {}

    def spy(key, run, cands, default):
        seen[key[0]] = tuple(cands)
        return default
    monkeypatch.setattr(CV.TUNER, "pick", spy)
    x, w = _inputs(2, 64, 128, 14, 3, 7)
    CV.conv_fwd(x, w, 1, 1, stats=True)
    assert 21 in seen["f"] and 22 in seen["f"]
    CV.conv_fwd(x, w, 1, 1, pro=(torch.ones(64, device="cuda"), torch.zeros(64, device="cuda")))
    assert 21 not in seen["f"]
    dy = torch.randn(2, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=CL)
    CV.conv_dgrad(dy, w, (14, 14), 1, 1)
    assert ("kc", 21) in seen["d"] and ("nkc", 21) not in seen["d"]
    dy2 = torch.randn(2, 128, 7, 7, device="cuda").bfloat16().contiguous(memory_format=CL)
    CV.conv_dgrad(dy2, w, (14, 14), 2, 1)          # stride 2: parity classes, no big tiles
    assert all(c[1] not in (21, 22) for c in seen["d"])


@pytest.mark.parametrize("N,H", [(2, 224), (3, 112), (40, 224)])
def test_stem_direct_conv_matches_gemm_path(N, H, monkeypatch):
    """The direct 7x7/2 stem convolution from an LDS patch (csrc/conv.hip k_stem_conv7) is
    bit-identical to the implicit-GEMM 4-channel path (same k order, 32-wide MFMA steps) and its
    statistics rows (one per workgroup) fold to the column sums of the stored output. N = 40 at
    224 px gives more row tiles than two per CU, so workgroups walk several tiles (the last one a
    partial run)."""
    x, w = _inputs(N, 3, 64, H, 7, 9)
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    outs = {}
    for tile in (3, 2, CV.STEM_DIRECT):
        monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default, t=tile: t)
        y, st = CV.conv_fwd(x, w, 2, 3, stats=True)
        _close(y, ref, 1e-2)
        outs[tile] = (y, st)
    y, st = outs[CV.STEM_DIRECT]
    assert torch.equal(y, outs[3][0]) and torch.equal(y, outs[2][0])
    assert y.is_contiguous(memory_format=CL)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    tot = st.sum(0)
    torch.testing.assert_close(tot[0], yf.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(tot[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("shape", [(4, 256, 256, 14, 3, 1, 1), (4, 512, 512, 7, 3, 1, 1),
                                   (4, 128, 256, 28, 3, 2, 1), (3, 64, 136, 9, 3, 1, 0),
                                   (2, 256, 512, 14, 1, 2, 0)],
                         ids=lambda s: str(s))
@pytest.mark.parametrize("tile", [21, 22])
def test_conv_wgrad_big_tiles(shape, tile, monkeypatch):
    """Weight gradients on the 8-wave big tiles with the im2col column gather (gemm_big.hip GB):
    fp32 vs torch for 1 / 2 / 4 split-K slices, padding 0 / 1, stride 1 / 2, N = taps*C off the
    tile grid, and accumulation into a channels_last arena view."""
    N, C, Co, H, k, s, p = shape
    x, w = _inputs(N, C, Co, H, k, 11)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    for sp in (1, 2, 4):
        monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default, c=(tile, sp): c)
        dw = CV.conv_wgrad(dy.contiguous(memory_format=CL), x, tuple(w.shape), s, p)
        _close(dw, wf.grad, 2e-3)
    arena = torch.full((Co * C * k * k,), 0.25, device="cuda")
    view = arena.as_strided(w.shape, (C * k * k, 1, k * C, C))
    CV.conv_wgrad(dy.contiguous(memory_format=CL), x, tuple(w.shape), s, p, out=view)
    _close(view - 0.25, wf.grad, 2e-3)


# the tap-reuse 3x3/1 kernel (csrc/conv3tap.hip): every stride-1 3x3 shape of ResNet-50 (batch
# reduced; 28 / 14 / 7 px tiles span images), the CIFAR nets, and both channel tiles (64, 128)
TAP_SHAPES = [(3, 64, 64, 56), (3, 128, 128, 28), (3, 256, 256, 14), (5, 512, 512, 7),
              (4, 64, 128, 32), (4, 128, 256, 16), (6, 256, 512, 8), (9, 512, 512, 4),
              (2, 32, 64, 14), (4, 96, 128, 28)]


@pytest.mark.parametrize("shape", TAP_SHAPES, ids=[str(s) for s in TAP_SHAPES])
def test_conv3_tap_fwd_stats_dgrad(shape):
    """k_conv3_tap vs fp32 F.conv2d: forward (and its column statistics of the stored bf16
    values, one row per 224-pixel tile) and the data gradient through the flipped weight."""
    from layer_wise_aaai20_amd.ops._ext import load
    N, C, Co, H = shape
    lib = load()
    x, w = _inputs(N, C, Co, H, 3, 7)
    op, K, _ = CV.pack_fwd_weight(w)
    y, st = lib.conv3_tap(x, op, Co, True)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=CL)
    _close(y, ref, 1e-2)
    yb = y.float().permute(0, 2, 3, 1).reshape(-1, Co)
    assert st.shape[1:] == (2, Co)
    torch.testing.assert_close(st[:, 0].sum(0), yb.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[:, 1].sum(0), (yb * yb).sum(0), rtol=1e-4, atol=1e-2)
    # data gradient: dx = conv(dy, W') with W'[ci][r][s][co] = w[co][ci][2-r][2-s] (its output
    # channel tile needs C == 64 or C % 128 == 0)
    if not (C == 64 or C % 128 == 0):
        return
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    xf = x.float().requires_grad_()
    F.conv2d(xf, w.float(), padding=1).backward(dy.float())
    dx, _ = lib.conv3_tap(dy, CV.tap_dgrad_weight(w), C, False)
    _close(dx, xf.grad, 1e-2)


def test_conv3_tap_is_a_tuner_candidate(monkeypatch):
    """Forced through the tuner (conv_fwd / conv_dgrad), the tap kernel gives the GEMM path's
    results to bf16 rounding."""
    x, w = _inputs(2, 64, 64, 56, 3, 3)
    calls = []
    orig = CV.TUNER.pick

    def pick(key, run, cands, default):
        c = [c for c in cands if (c == CV.CONV3_TAP or (isinstance(c, tuple) and c[0] == "tap"))]
        calls.append(bool(c))
        return c[0] if c else orig(key, run, cands, default)
    monkeypatch.setattr(CV.TUNER, "pick", pick)
    y, st = CV.conv_fwd(x, w, 1, 1, stats=True)
    _close(y, F.conv2d(x.float(), w.float(), padding=1), 1e-2)
    dy = torch.randn_like(y.float()).bfloat16().contiguous(memory_format=CL)
    dx = CV.conv_dgrad(dy, w, (56, 56), 1, 1)
    xf = x.float().requires_grad_()
    F.conv2d(xf, w.float(), padding=1).backward(dy.float())
    _close(dx, xf.grad, 1e-2)
    assert calls == [True, True]


@pytest.mark.parametrize("shape", TAP_SHAPES, ids=[str(s) for s in TAP_SHAPES])
def test_conv3_tap_wgrad(shape):
    """k_conv3_tap_wgrad (+ the fixed-order split reduce) vs fp32 torch, fresh and accumulated
    into a channels_last fp32 arena view."""
    from layer_wise_aaai20_amd.ops._ext import load
    N, C, Co, H = shape
    lib = load()
    x, w = _inputs(N, C, Co, H, 3, 11)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, padding=1)
    dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=CL)
    ref.backward(dy.float())
    dw = lib.conv3_tap_wgrad(dy, x, None, False)
    assert dw.shape == (Co, C, 3, 3) and dw.is_contiguous(memory_format=CL)
    _close(dw, wf.grad, 2e-3)
    base = torch.randn(Co, C, 3, 3, device="cuda").contiguous(memory_format=CL)
    out = base.clone()
    lib.conv3_tap_wgrad(dy, x, out, True)
    _close(out - base, wf.grad, 2e-3)


@pytest.mark.parametrize("co,c", [(64, 64), (128, 128), (512, 512), (64, 32), (256, 128)])
def test_tap_dgrad_weight_pack_matches_flip(co, c):
    """tap_dgrad_weight by one pack_dgrad_kc launch walking the 3x3 window backwards equals the
    flip + transpose it replaces, bit for bit."""
    w = torch.randn(co, c, 3, 3, device="cuda").bfloat16().contiguous(memory_format=CL)
    got = CV.tap_dgrad_weight(w)
    ref = w.flip(2, 3).permute(1, 2, 3, 0).reshape(c, -1).contiguous()
    assert got.shape == ref.shape and torch.equal(got, ref)


@pytest.mark.parametrize("shape", [(64, 64, 3, 1, 1), (128, 128, 3, 2, 1), (512, 256, 3, 2, 1),
                                   (256, 64, 1, 1, 0), (64, 32, 1, 2, 0), (48, 24, 3, 2, 0)])
def test_pack_dgrad_nkc_matches_slices(shape, monkeypatch):
    """pack_dgrad_weight's one-launch [K][C] pack equals the permute / slice / cat form."""
    co, c, k, s, p = shape
    w = torch.randn(co, c, k, k, device="cuda").bfloat16().contiguous(memory_format=CL)
    H = 14
    classes = CV._dgrad_classes(H, H, k, k, s, s, p, p)
    got, go = CV.pack_dgrad_weight(w, classes, s, s)
    ref, ro = CV.pack_dgrad_weight(w.cpu(), classes, s, s)    # (CPU: the permute / slice form)
    assert go == ro and torch.equal(got.cpu(), ref)
