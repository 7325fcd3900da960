"""Fused NHWC BatchNorm(+add)(+ReLU) HIP kernels vs torch's BatchNorm (fp32 reference)."""
import pytest
import torch
import torch.nn.functional as F

from layer_wise_aaai20_amd.ops.nn import fused_batch_norm, fuse_resnet

pytestmark = pytest.mark.gpu


def _ref(x, res, w, b, rm, rv, relu):
    y = F.batch_norm(x.float(), rm, rv, w, b, True, 0.1, 1e-5)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 7), (2, 2048, 3, 3), (3, 24, 5, 5)])
def test_fused_bn_matches_torch(dtype, relu, residual, shape):
    torch.manual_seed(0)
    C = shape[1]
    x = (torch.randn(*shape, device="cuda") * 2 + 0.5).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    res = (torch.randn(*shape, device="cuda").to(dtype).contiguous(
        memory_format=torch.channels_last).requires_grad_() if residual else None)
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_()
    b = torch.randn(C, device="cuda").requires_grad_()
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    rm2, rv2 = rm.clone(), rv.clone()
    y = fused_batch_norm(x, w, b, rm, rv, True, 0.1, 1e-5, relu=relu, residual=res)
    xr = x.detach().float().requires_grad_()
    resr = res.detach().float().requires_grad_() if residual else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = _ref(xr, resr, wr, br, rm2, rv2, relu)
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-5)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    gtol = dict(rtol=3e-2, atol=5e-1) if dtype == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(w.grad, wr.grad, **gtol)
    torch.testing.assert_close(b.grad, br.grad, **gtol)
    if residual:
        torch.testing.assert_close(res.grad.float(), resr.grad, **tol)


def test_fused_bn_eval_mode():
    C = 32
    x = torch.randn(4, C, 6, 6, device="cuda").contiguous(memory_format=torch.channels_last)
    w, b = torch.rand(C, device="cuda"), torch.randn(C, device="cuda")
    rm, rv = torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5
    y = fused_batch_norm(x, w, b, rm, rv, False, 0.1, 1e-5, relu=True)
    yr = F.relu(F.batch_norm(x, rm, rv, w, b, False, 0.1, 1e-5))
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)


def test_fused_resnet18_matches_unfused():
    from layer_wise_aaai20_amd.models.resnet import resnet18
    torch.manual_seed(0)
    a = resnet18().cuda().to(memory_format=torch.channels_last)
    b = resnet18().cuda().to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    fuse_resnet(b, mfma=False)             # BN fusion only: fp32 parity
    assert set(a.state_dict()) == set(b.state_dict())
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    ya, yb = a(x), b(x)
    torch.testing.assert_close(yb, ya, rtol=1e-3, atol=1e-3)
    ya.square().mean().backward()
    yb.square().mean().backward()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pb.grad, pa.grad, rtol=2e-3, atol=2e-4, msg=n)
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(bb.float(), ba.float(), rtol=1e-4, atol=1e-5, msg=n)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_fused_resnet18_mfma_convs_close_to_torch():
    """Fused BN + every conv / the fc on the MFMA kernels (bf16 operands) vs the same model in
    fp32: the error is of the same size as torch's own bf16-autocast error."""
    from layer_wise_aaai20_amd.models.resnet import resnet18
    torch.manual_seed(0)
    r = resnet18().cuda().to(memory_format=torch.channels_last)      # fp32 reference
    a = resnet18().cuda().to(memory_format=torch.channels_last)      # torch, bf16 autocast
    b = resnet18().cuda().to(memory_format=torch.channels_last)      # fused, MFMA kernels
    a.load_state_dict(r.state_dict())
    b.load_state_dict(r.state_dict())
    fuse_resnet(b)
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    yr = r(x)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya, yb = a(x), b(x)
    ea, eb = _rel(ya, yr), _rel(yb, yr)
    assert eb < 2 * ea + 1e-2, (ea, eb)
    yr.square().mean().backward()
    ya.float().square().mean().backward()
    yb.float().square().mean().backward()
    for (n, pr), pa, pb in zip(r.named_parameters(), a.parameters(), b.parameters()):
        ga, gb = _rel(pa.grad, pr.grad), _rel(pb.grad, pr.grad)
        assert gb < 2 * ga + 2e-2, (n, ga, gb)


@pytest.mark.parametrize("shape,k", [((16, 128, 32, 32), 2), ((8, 256, 16, 16), 2),
                                     ((8, 512, 8, 8), 2), ((4, 64, 16, 16), 4)])
def test_bn_relu_pool_matches_torch(shape, k):
    """FusedBNReluPool2d (the CIFAR conv_bn -> MaxPool2d fusion) vs fp32 torch BN+ReLU+pool:
    output, input gradient, gamma/beta gradients and running statistics."""
    from layer_wise_aaai20_amd.ops.nn import FusedBNReluPool2d, to_fused_bn
    torch.manual_seed(1)
    C = shape[1]
    x = (torch.randn(*shape, device="cuda") * 1.5 + 0.3).bfloat16()
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    bn = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_()
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(bn.state_dict())
    to_fused_bn(bn, relu=True)
    bn.__class__ = FusedBNReluPool2d
    bn.fuse_pool = (k, k, 0)
    y = bn(x)
    xr = x.detach().float().requires_grad_()
    a = F.relu(ref(xr))
    # the fused kernel pools the bf16-rounded activation: round straight-through so that window
    # ties (and their first-max routing) match
    a = a + (a.detach().bfloat16().float() - a.detach())
    yr = F.max_pool2d(a, k)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = torch.randn_like(yr).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    # a window whose two maxima differ only past bf16 precision in the two BN paths routes its
    # gradient to a different pixel: allow a handful of such pixels, all others must match
    err = (x.grad.float() - xr.grad).abs()
    bad = err > 5e-2 + 5e-2 * xr.grad.abs()
    assert bad.float().mean().item() < 2e-4, f"{int(bad.sum())} mismatched gradient elements"
    for a_, b_ in ((bn.weight.grad, ref.weight.grad), (bn.bias.grad, ref.bias.grad)):
        # (a misrouted tie moves one pixel's gradient between two pixels of a channel's sums)
        assert (a_ - b_).abs().max().item() <= 2e-2 * b_.abs().max().item() + 1e-3
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-2, rtol=1e-2)


def test_graph_fusion_folds_pools():
    """fuse_graph_network folds every conv_bn -> MaxPool2d of ResNet-9 into the BN (and leaves
    the final 4x4 pool after the residual add alone)."""
    from layer_wise_aaai20_amd.models.cifar import resnet9
    from layer_wise_aaai20_amd.models.graph import Network
    from layer_wise_aaai20_amd.ops.nn import FusedBNReluPool2d, fuse_graph_network
    net = fuse_graph_network(Network(resnet9()))
    fused = [n for n, m in net.named_modules() if isinstance(m, FusedBNReluPool2d)]
    assert sorted(fused) == ["layer1_bn", "layer2_bn", "layer3_bn"]
    assert isinstance(net.pool, torch.nn.MaxPool2d)


@pytest.mark.parametrize("M,C", [(4096, 256), (3136, 512), (784, 2048), (1000, 64)])
def test_bn_bwd_dual_matches_two_single_passes(M, C):
    """bn_bwd_dual (BN3 + downsample BN sharing dy and the ReLU bitmap, one reduce and one apply
    pass) is bit-identical to two bn_bwd calls, including accumulation into dgamma/dbeta views."""
    from layer_wise_aaai20_amd.ops._ext import load
    lib = load()
    g = torch.Generator(device="cuda").manual_seed(M + C)
    mk = lambda: torch.randn(M, C, device="cuda", generator=g).bfloat16()  # noqa: E731
    dy, x, x2 = mk(), mk(), mk()
    bits = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda", generator=g)
    stats = [(torch.rand(C, device="cuda", generator=g) + 0.5,
              torch.randn(C, device="cuda", generator=g) * 0.1,
              torch.rand(C, device="cuda", generator=g) + 0.5) for _ in range(2)]
    (g1, m1, i1), (g2, m2, i2) = stats
    outs = [torch.randn(C, device="cuda", generator=g) for _ in range(4)]
    ref_outs = [o.clone() for o in outs]
    dx_a, dg_a, db_a, _ = lib.bn_bwd(dy, x, None, g1, m1, i1, None, True, True, False, bits,
                                     ref_outs[0], ref_outs[1])
    dx_b, dg_b, db_b, _ = lib.bn_bwd(dy, x2, None, g2, m2, i2, None, True, True, False, bits,
                                     ref_outs[2], ref_outs[3])
    dx, dx2, dg, db, dg2, db2 = lib.bn_bwd_dual(dy, x, x2, bits, g1, m1, i1, g2, m2, i2, *outs)
    assert torch.equal(dx, dx_a) and torch.equal(dx2, dx_b)
    for a, b in zip((dg, db, dg2, db2), ref_outs):
        assert torch.equal(a, b)
    assert dg.data_ptr() == outs[0].data_ptr()          # accumulated in place


@pytest.mark.parametrize("M,C,R", [(50176, 256, 392), (12544, 2048, 98), (802816, 64, 6272),
                                   (1000, 136, 8)])
def test_bn_stats_from_rows_one_launch(M, C, R, monkeypatch):
    """bn_stats on GEMM-epilogue statistics rows: the one-launch colsum + finalize (per-slice
    arrival tickets, last block folds) gives the batch mean / invstd / scale-shift and running
    statistics of the rows, and its tickets re-arm: repeated calls agree bit for bit."""
    from layer_wise_aaai20_amd.ops._ext import load
    lib = load()
    g = torch.Generator(device="cuda").manual_seed(C)
    rows = torch.randn(R, 2, C, device="cuda", generator=g)
    rows[:, 1] = rows[:, 1].abs() * 4 + 2
    x = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    gamma = torch.rand(C, device="cuda", generator=g) + 0.5
    beta = torch.randn(C, device="cuda", generator=g)
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    outs = [lib.bn_stats(x, rows, gamma, beta, rm, rv, 0.1, 1e-5) for _ in range(3)]
    s = rows.double().sum(0)
    mean = s[0] / M
    var = (s[1] / M - mean * mean).clamp_min(0)
    torch.testing.assert_close(outs[0][0].double(), mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(outs[0][1].double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
    sc = gamma.double() / torch.sqrt(var + 1e-5)
    torch.testing.assert_close(outs[0][2][:C].double(), sc, rtol=1e-4, atol=1e-5)
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0]))
    assert torch.isfinite(rm).all() and not torch.equal(rm, torch.zeros_like(rm))


@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("M,C,Ci", [(4096, 256, 64), (3000, 256, 64), (802816 // 16, 256, 64),
                                    (4096, 512, 128), (1000, 512, 128), (200704 // 8, 512, 128)])
def test_bn3_bwd_fused_matches_three_passes(M, C, Ci, dual):
    """bn3_bwd_fused (csrc/bnfuse.hip: BN3's apply inside one kernel with da2 = dc3·W3 and
    dW3 = dc3ᵀ·a2) vs bn_bwd / bn_bwd_dual + fp32 products of their dc3: dgamma/dbeta
    bit-identical (the same reduce + finalize), the shortcut BN's dx2 (dual) within one bf16 ulp,
    da2 within bf16 rounding, dW3 within fp32 summation-order noise, the weight gradient
    accumulated into a given view. M = 3000 / 1000 end in a partial tile; 4096 / 1000 run one
    tile group (the result added straight into the destination). BN2's backward sums, reduced
    by the same kernel from its da2 tiles (rows per tile group), match an fp64 reduction of the
    returned da2, and BN2's backward fed those rows matches the one running its own reduce.
    With a2_from_bn2 (a2 formed in the kernel from c2, as the a2-free forward needs) every output
    is bit-identical to the run given the materialised a2 = relu(bn2(c2))."""
    from layer_wise_aaai20_amd.ops._ext import h16, load
    lib = load()
    g = torch.Generator(device="cuda").manual_seed(M + C + dual)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(h16())  # noqa: E731
    dy, x, x2, a2 = mk(M, C), mk(M, C), mk(M, C), mk(M, Ci)
    w3 = (torch.randn(C, Ci, device="cuda", generator=g) / 16).to(h16())
    w3t = w3.t().contiguous()
    bits = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda", generator=g)
    st = [(torch.rand(C, device="cuda", generator=g) + 0.5,
           torch.randn(C, device="cuda", generator=g) * 0.1,
           torch.rand(C, device="cuda", generator=g) + 0.5) for _ in range(2)]
    (gam, mean, inv), (gam2, mean2, inv2) = st
    outs = [torch.randn(C, device="cuda", generator=g) for _ in range(4)]
    ref = [o.clone() for o in outs]
    if dual:
        dc3, rdx2, _, _, _, _ = lib.bn_bwd_dual(dy, x, x2, bits, gam, mean, inv, gam2, mean2, inv2,
                                                *ref)
    else:
        dc3, _, _, _ = lib.bn_bwd(dy, x, None, gam, mean, inv, None, True, True, False, bits,
                                  ref[0], ref[1])
    dw = torch.full((C, Ci), 0.25, device="cuda")
    down = (x2, gam2, mean2, inv2, outs[2], outs[3]) if dual else ()
    c2 = mk(M, Ci)
    ss2 = torch.cat([torch.rand(Ci, device="cuda", generator=g) + 0.5,
                     torch.randn(Ci, device="cuda", generator=g) * 0.3])
    mean2b = torch.randn(Ci, device="cuda", generator=g) * 0.1
    a2 = lib.bn_apply(c2, ss2, None, None, True)
    # a2 formed inside the kernel from c2: the same bits as from the materialised a2
    outs_c = [o.clone() for o in outs]
    dw_c = torch.full((C, Ci), 0.25, device="cuda")
    down_c = (x2, gam2, mean2, inv2, outs_c[2], outs_c[3]) if dual else (None,) * 6
    res_c = lib.bn3_bwd_fused(dy, x, bits, gam, mean, inv, w3t, c2, dw_c, outs_c[0], outs_c[1],
                              *down_c, c2, ss2, mean2b, True)
    down = down if dual else (None,) * 6
    da2, dwr, dg, db, dx2, dg2, db2, st2 = lib.bn3_bwd_fused(
        dy, x, bits, gam, mean, inv, w3t, a2, dw, outs[0], outs[1], *down, c2, ss2, mean2b)
    assert torch.equal(dw_c, dw) and torch.equal(res_c[0], da2) and torch.equal(res_c[7], st2)
    if dual:
        assert torch.equal(res_c[4], dx2)
    # BN2's sums from the kernel vs fp64 over the da2 it wrote
    d = da2.double() * ((c2.float() * ss2[:Ci] + ss2[Ci:]) > 0).double()
    want = torch.stack([d.sum(0), (d * (c2.double() - mean2b.double())).sum(0)])
    got = st2.double().sum(0)
    tol = 1e-4 * d.abs().sum(0).max().item() + 1e-4
    assert (got - want).abs().max().item() <= tol, ((got - want).abs().max().item(), tol)
    inv2b = torch.rand(Ci, device="cuda", generator=g) + 0.5
    gam2b = torch.rand(Ci, device="cuda", generator=g) + 0.5
    r_dc2, _, r_dg2, r_db2 = lib.bn_bwd(da2, c2, None, gam2b, mean2b, inv2b, ss2, True, True,
                                        False, None)
    f_dc2, _, f_dg2, f_db2 = lib.bn_bwd(da2, c2, None, gam2b, mean2b, inv2b, ss2, True, True,
                                        False, None, None, None, st2)
    torch.testing.assert_close(f_db2, r_db2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(f_dg2, r_dg2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(f_dc2.float(), r_dc2.float(), rtol=2e-2, atol=2e-2)
    assert torch.equal(dg, ref[0]) and torch.equal(db, ref[1])
    if dual:
        assert torch.equal(dg2, ref[2]) and torch.equal(db2, ref[3])
        ulp = (rdx2.float().abs() * 2.0 ** -7).clamp_min(1e-30)
        assert bool(((dx2.float() - rdx2.float()).abs() <= ulp).all())
    else:
        assert dx2.numel() == 0
    assert dwr.data_ptr() == dw.data_ptr()
    ref_da2 = dc3.float() @ w3.float()
    err = (da2.float() - ref_da2).abs().max().item()
    assert err <= 1e-2 * ref_da2.abs().max().item(), err
    ref_dw = dc3.float().t() @ a2.float()
    err = ((dw - 0.25) - ref_dw).abs().max().item()
    assert err <= 1e-4 * ref_dw.abs().max().item() + 1e-3, err
    # without a destination: a fresh [C, Ci] result
    _, dw2, _, _, _, _, _, _ = lib.bn3_bwd_fused(dy, x, bits, gam, mean, inv, w3t, a2, None, None,
                                              None, *((x2, gam2, mean2, inv2) if dual else ()))
    torch.testing.assert_close(dw2, dw - 0.25, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,Wd,Cin", [(4096, 64, 256), (3000, 64, 256), (802816 // 16, 64, 256),
                                      (1000, 128, 512), (200704 // 8, 128, 512)])
def test_bn1_bwd_fused_matches_three_passes(M, Wd, Cin):
    """bn1_bwd_fused (csrc/bnfuse.hip: BN1's apply, ReLU mask from c1 through the forward affine,
    inside one kernel with dx = dc1·W1 + dy·bit3 and dW1 = dc1ᵀ·x) vs bn_bwd + fp32 products of
    its dc1: dgamma/dbeta bit-identical, dx within bf16 rounding of the GEMM epilogue's
    bf16(acc) + addend, dW1 within summation-order noise, accumulated into a given view."""
    from layer_wise_aaai20_amd.ops._ext import h16, load
    lib = load()
    g = torch.Generator(device="cuda").manual_seed(M + Wd)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(h16())  # noqa: E731
    da1, c1, x, dy = mk(M, Wd), mk(M, Wd), mk(M, Cin), mk(M, Cin)
    w1 = (torch.randn(Wd, Cin, device="cuda", generator=g) / 16).to(h16())
    bits = torch.randint(0, 256, (M * Cin // 8,), dtype=torch.uint8, device="cuda", generator=g)
    gam = torch.rand(Wd, device="cuda", generator=g) + 0.5
    mean = torch.randn(Wd, device="cuda", generator=g) * 0.1
    inv = torch.rand(Wd, device="cuda", generator=g) + 0.5
    ss = torch.cat([gam * inv, -mean * gam * inv + 0.1]).contiguous()
    outs = [torch.randn(Wd, device="cuda", generator=g) for _ in range(2)]
    ref = [o.clone() for o in outs]
    dc1, _, _, _ = lib.bn_bwd(da1, c1, None, gam, mean, inv, ss, True, True, False, None, *ref)
    dw = torch.full((Wd, Cin), 0.25, device="cuda")
    dx, dwr, dg, db = lib.bn1_bwd_fused(da1, c1, ss, gam, mean, inv, w1.t().contiguous(), x, dy,
                                        bits, dw, *outs)
    assert torch.equal(dg, ref[0]) and torch.equal(db, ref[1])
    assert dwr.data_ptr() == dw.data_ptr()
    mask = ((bits.view(-1, 1) >> torch.arange(8, device="cuda")) & 1).view(M, Cin).bool()
    ref_dx = (dc1.float() @ w1.float()).to(h16()).float() + torch.where(mask, dy.float(), 0.)
    err = (dx.float() - ref_dx).abs().max().item()
    assert err <= 1e-2 * ref_dx.abs().max().item(), err
    ref_dw = dc1.float().t() @ x.float()
    err = ((dw - 0.25) - ref_dw).abs().max().item()
    assert err <= 1e-4 * ref_dw.abs().max().item() + 1e-3, err
