"""Single-process engine / arena / DDP / optimizer behaviour on CPU."""
import pytest
import torch
from torch import nn

from layer_wise_aaai20_amd.compress import reference as ref
from layer_wise_aaai20_amd.models import cifar
from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
from layer_wise_aaai20_amd.parallel import functional as F
from layer_wise_aaai20_amd.parallel.arena import GradArena, plan_buckets
from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine


def small_net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU(), nn.Flatten(),
                         nn.Linear(8 * 6 * 6, 10))


def test_arena_views_and_reverse_order():
    m = small_net().to(memory_format=torch.channels_last)
    a = GradArena(list(m.named_parameters()))
    assert [s.name for s in a.segments][0] == "4.bias"          # reverse registration order
    m(torch.randn(2, 3, 8, 8)).sum().backward()
    for s in a.segments:
        assert s.param.grad.data_ptr() == a.grad.data_ptr() + s.offset * 4
        assert s.offset % 64 == 0
    w = m[0].weight
    assert w.grad.stride() == w.stride()                         # channels_last grad view
    assert float(a.grad.abs().sum()) > 0


def test_bucket_plan_caps_and_entire_model():
    m = cifar.build_network("resnet9")
    a = GradArena(list(m.named_parameters()))
    bs = plan_buckets(a, "layerwise", 4 * 2 ** 20)
    assert bs[0].start == 0 and bs[-1].end == a.numel
    assert all(b1.end == b2.start for b1, b2 in zip(bs, bs[1:]))
    assert len(bs) > 2
    assert len(plan_buckets(a, "entiremodel", 1)) == 1


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("method,kw", [("Topk", dict(K=0.01)), ("Thresholdv", dict(V=1e-3)),
                                       ("AdaptiveThreshold", {}), ("none", {})])
def test_functional_sync_matches_oracle(mode, method, kw):
    m = cifar.build_network("resnet9")
    batch = {"input": torch.randn(4, 3, 32, 32), "target": torch.randint(0, 10, (4,))}
    m(batch)["loss"].sum().backward()
    grads = [p.grad.clone() for p in m.parameters()]
    F.compressed_comm(m, mode, 1, method, kw.get("K"), kw.get("V"), None)
    if mode == "layerwise":
        for p, g in zip(m.parameters(), grads):
            assert torch.equal(p.grad.reshape(-1), ref.compress(g.reshape(-1), method, **kw))
    else:
        # entire-model: the compressor sees the concatenation in arena (reverse) order
        flat = torch.cat([g.reshape(-1) for g in reversed(grads)])
        exp = ref.compress(flat, method, **kw)
        got = torch.cat([p.grad.reshape(-1) for p in reversed(list(m.parameters()))])
        assert torch.equal(got, exp)


def test_entire_model_starves_small_layers_layerwise_does_not():
    m = cifar.build_network("resnet9")
    m({"input": torch.randn(4, 3, 32, 32), "target": torch.randint(0, 10, (4,))})["loss"] \
        .sum().backward()
    F.layerwise_compressed_comm(m, 1, "Topk", 0.001)
    assert all(int((p.grad != 0).sum()) >= 1 for p in m.parameters())


def test_compressed_ddp_hooks_match_functional():
    torch.manual_seed(1)
    a = cifar.build_network("resnet9")
    b = cifar.build_network("resnet9")
    b.load_state_dict(a.state_dict())
    batch = {"input": torch.randn(4, 3, 32, 32), "target": torch.randint(0, 10, (4,))}
    ddp = CompressedDDP(b, compress="layerwise", method="Topk", K=0.01, bucket_cap_mb=2,
                        flat_params=False)
    a(batch)["loss"].sum().backward()
    F.layerwise_compressed_comm(a, 1, "Topk", 0.01)
    ddp(batch)["loss"].sum().backward()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad)
    assert ddp.engine.stats.steps == 1 and len(ddp.engine.buckets) > 1


def test_bucket_launch_order_is_strict():
    m = cifar.build_network("resnet9")
    eng = GradSyncEngine(m.named_parameters(), "layerwise", "Topk", K=0.01, bucket_cap_mb=1)
    launched = []
    eng._launch = lambda bi: launched.append(bi)
    nb = len(eng.buckets)
    assert nb >= 3
    # make the LAST bucket ready first: nothing may launch until bucket 0 is complete
    for b in reversed(eng.buckets):
        for s in range(b.seg_lo, b.seg_hi):
            eng.mark_ready(s)
        if b.index != 0:
            assert launched == []
    assert launched == list(range(nb))


def test_check_reduction_detects_unfinished_backward():
    m = small_net()
    ddp = CompressedDDP(m, method="Topk", K=0.1, flat_params=False)
    ddp(torch.randn(2, 3, 8, 8))
    ddp.engine._active = True
    with pytest.raises(RuntimeError):
        ddp(torch.randn(2, 3, 8, 8))


def test_flat_sgd_matches_torch_sgd_and_state_dict():
    ma, mb = small_net(), small_net()
    mb.load_state_dict(ma.state_dict())
    arena = GradArena(list(mb.named_parameters()), flat_params=True)
    bn = [mb[1].weight, mb[1].bias]
    rest = [p for p in mb.parameters() if all(p is not q for q in bn)]
    bn_a = [ma[1].weight, ma[1].bias]
    rest_a = [p for p in ma.parameters() if all(p is not q for q in bn_a)]
    oa = torch.optim.SGD([{"params": bn_a, "weight_decay": 0}, {"params": rest_a}], lr=0.05,
                         momentum=0.9, nesterov=True, weight_decay=1e-3)
    ob = FlatSGD([{"params": bn, "weight_decay": 0}, {"params": rest}], arena, lr=0.05,
                 momentum=0.9, nesterov=True, weight_decay=1e-3)
    x = torch.randn(4, 3, 8, 8)
    for _ in range(4):
        oa.zero_grad()
        ma(x).square().mean().backward()
        arena.zero_()
        mb(x).square().mean().backward()
        oa.step()
        ob.step()
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    sd = ob.state_dict()
    oc = torch.optim.SGD([{"params": bn_a, "weight_decay": 0}, {"params": rest_a}], lr=0.05,
                         momentum=0.9, nesterov=True, weight_decay=1e-3)
    oc.load_state_dict(sd)                       # FlatSGD checkpoints load into torch SGD
    for k, v in oa.state_dict()["state"].items():
        torch.testing.assert_close(sd["state"][k]["momentum_buffer"], v["momentum_buffer"],
                                   rtol=1e-5, atol=1e-6)


class _DirectLinear(torch.autograd.Function):
    """Like the fused MFMA ops (ops/block.py, ops/gemm.py): the weight gradient is written straight
    into its arena view, the op announces it with ``_lw_grad_ready`` and returns None for it —
    after which PyTorch still runs the weight's post-accumulate-grad hook."""

    @staticmethod
    def forward(ctx, x, w, written):
        ctx.save_for_backward(x, w)
        ctx.written = written
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        p = ctx.w_param
        if getattr(p, "_lw_grad_ready", None) is not None and p.grad is not None:
            p.grad.add_(dy.t() @ x)
            ctx.written.add(id(p))
            p._lw_grad_ready(p)
            return dy @ w, None, None
        return dy @ w, dy.t() @ x, None


class _DirectNet(nn.Module):
    def __init__(self, written):
        super().__init__()
        self.written = written
        self.l1, self.l2, self.l3 = (nn.Linear(16, 16, bias=False) for _ in range(3))

    def forward(self, x):
        for m in (self.l1, self.l2, self.l3):
            x = torch.relu(_DirectLinear.apply(x, m.weight, self.written))
        return x


def test_direct_arena_gradients_count_once_per_step():
    """A bucket is launched only once every one of its segments is complete, even though a
    directly-written parameter is announced twice (by the op, then by autograd's hook)."""
    written = set()
    net = _DirectNet(written)
    ddp = CompressedDDP(net, compress="layerwise", method="Topk", K=0.5, bucket_cap_mb=1.0,
                        flat_params=True)
    params = {id(m.weight): m.weight for m in (net.l1, net.l2, net.l3)}
    launched = []
    real = ddp.engine._launch

    def launch(bi):
        b = ddp.engine.buckets[bi]
        segs = ddp.engine.arena.segments[b.seg_lo:b.seg_hi]
        launched.append(all(id(s.param) in written for s in segs))
        real(bi)
    ddp.engine._launch = launch
    # route each Function call to its weight
    apply = _DirectLinear.apply

    def apply_with_param(x, w, wr):
        out = apply(x, w, wr)
        out.grad_fn.w_param = params[id(w)]
        return out
    _DirectLinear.apply = staticmethod(apply_with_param)
    try:
        for _ in range(2):
            written.clear()
            launched.clear()
            ddp(torch.randn(4, 16)).sum().backward()
            assert launched and all(launched), launched
    finally:
        _DirectLinear.apply = staticmethod(apply)


def test_dense_below_sends_small_tensors_whole():
    """``dense_below`` (opt-in EF fix): segments of at most that many elements keep every
    element; larger ones keep the reference count."""
    from layer_wise_aaai20_amd.compress.codecs import TopkCodec, RandkCodec
    from layer_wise_aaai20_amd.compress.plan import SegPlan
    plan = SegPlan([0, 64], [64, 10000])
    c = TopkCodec(plan, 1, 0, K=0.01, dense_below=4096)
    assert c.keep.tolist() == [64, ref.topk_keep_count(10000, 0.01)]
    g = torch.randn(10064)
    ef = torch.zeros(10064)
    send = c.compress(g.clone(), ef, 0)
    out = torch.zeros(10064)
    c.decompress(send, None, out)
    assert torch.equal(out[:64], g[:64])                       # small: all of it
    assert int((out[64:] != 0).sum()) == c.keep[1]
    assert float(ef[:64].abs().sum()) == 0.0
    r = RandkCodec(plan, 1, 0, K=0.01, dense_below=100)
    assert r.keep.tolist()[0] == 64


def _mc_expect(eng, u, sent):
    """Momentum factor masking: u at the sent coordinates -> 0, unless the segment went whole."""
    out = u.clone()
    for s in eng.arena.segments:
        sl = slice(s.offset, s.offset + s.numel)
        m = sent[sl] != 0
        if int(m.sum()) < s.numel:
            out[sl][m] = 0
    return out


def test_momentum_correction_accumulates_velocity_and_masks():
    """DGC momentum correction: u = m·u + g; the residual accumulates u; sent coordinates have
    their velocity zeroed; decoded + e_new == e_old + u (what was sent is exactly removed)."""
    torch.manual_seed(0)
    net = small_net()
    eng = GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.05,
                         error_feedback=True, momentum_correction=0.9)
    u_prev = torch.zeros_like(eng.arena.grad)
    for _ in range(4):
        g = torch.zeros(eng.arena.numel)
        for s in eng.arena.segments:
            g[s.offset:s.offset + s.numel] = torch.randn(s.numel)
        e_old = eng.ef.clone()
        eng.arena.grad.copy_(g)
        eng.sync_now()
        u_expect = 0.9 * u_prev + g
        sent = eng.arena.grad                                     # world 1: decoded = sent
        torch.testing.assert_close(sent + eng.ef, e_old + u_expect, rtol=1e-5, atol=1e-6)
        # velocity zeroed exactly where something was sent, except in a segment sent whole
        torch.testing.assert_close(eng.mom, _mc_expect(eng, u_expect, sent), rtol=0, atol=0)
        u_prev = eng.mom.clone()
    with pytest.raises(ValueError):
        GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.05,
                       error_feedback=False, momentum_correction=0.9)


def test_lr_scaled_residual_rescales_by_lr_ratio():
    """ef_lr_scaled: before step t compresses, the residual left at step t-1 is multiplied by
    lr_{t-1} / lr_t (1 on the first step and whenever either LR is 0), so sent + e_new equals
    e_old * ratio + g."""
    torch.manual_seed(0)
    net = small_net()
    eng = GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.05,
                         error_feedback=True, ef_lr_scaled=True)
    lrs = [0.1, 0.2, 0.2, 0.05, 0.0, 0.3]
    ratios = [1.0, 0.5, 1.0, 4.0, 1.0, 1.0]
    box = {}
    eng.lr_source = lambda: box["lr"]
    for lr, r in zip(lrs, ratios):
        box["lr"] = torch.tensor([lr])
        eng.begin_step()
        assert abs(float(eng._lr_ratio) - r) < 1e-6, (lr, float(eng._lr_ratio))
        g = torch.zeros(eng.arena.numel)
        for s in eng.arena.segments:
            g[s.offset:s.offset + s.numel] = torch.randn(s.numel)
        e_old = eng.ef.clone()
        eng.arena.grad.copy_(g)
        eng.sync_now()
        torch.testing.assert_close(eng.arena.grad + eng.ef, e_old * r + g, rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.05,
                       error_feedback=False, ef_lr_scaled=True)


def test_momentum_correction_dense_segments_keep_ordinary_momentum():
    """a tensor that travels whole (dense_below) keeps u = m·u + g every step (its
    velocity is never reset), so under MC it trains with ordinary momentum; the compressed ones
    are masked where sent."""
    torch.manual_seed(1)
    net = small_net()
    eng = GradSyncEngine(list(net.named_parameters()), mode="layerwise", method="Topk", K=0.05,
                         error_feedback=True, momentum_correction=0.9, dense_below=64)
    small = [s for s in eng.arena.segments if s.numel <= 64]
    assert small, "small_net has tensors under the dense_below bound"
    u = torch.zeros(eng.arena.numel)
    for _ in range(3):
        g = torch.zeros(eng.arena.numel)
        for s in eng.arena.segments:
            g[s.offset:s.offset + s.numel] = torch.randn(s.numel)
        eng.arena.grad.copy_(g)
        eng.sync_now()
        u = 0.9 * u + g
        for s in small:
            sl = slice(s.offset, s.offset + s.numel)
            torch.testing.assert_close(eng.mom[sl], u[sl], rtol=1e-6, atol=1e-7)
            torch.testing.assert_close(eng.arena.grad[sl], u[sl], rtol=1e-6, atol=1e-7)
        u = eng.mom.clone()


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
def test_momentum_correction_folds_weight_decay_per_group(mode):
    """with MC the weight decay enters the gradient before the velocity,
    u = m·u + g + wd·p with each param group's wd (no_bn_wd groups stay at 0), and the optimizer
    then applies none (its groups are set to 0); the loss-scaled gradient gets wd·p/grad_scale."""
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    torch.manual_seed(2)
    net = small_net()
    eng = GradSyncEngine(list(net.named_parameters()), mode=mode, method="Topk", K=0.05,
                         error_feedback=True, momentum_correction=0.9, flat_params=True)
    params = [p for p in net.parameters()]
    groups = [{"params": params[:1], "weight_decay": 0.0},
              {"params": params[1:], "weight_decay": 1e-2}]
    opt = FlatSGD(groups, eng.arena, lr=0.1, momentum=0.0, weight_decay=1e-2, grad_scale=0.5)
    eng.set_mc_weight_decay(opt)
    assert all(g["weight_decay"] == 0.0 for g in opt.param_groups)
    wd = torch.zeros(eng.arena.numel)
    assert sum(s.param is params[0] for s in eng.arena.segments) == 1
    for s in eng.arena.segments:
        if s.param is not params[0]:
            wd[s.offset:s.offset + s.numel] = 1e-2
    p = eng.arena.param_buf.clone()
    g = torch.zeros(eng.arena.numel)
    for s in eng.arena.segments:                 # (layer-wise segments are padded apart)
        g[s.offset:s.offset + s.numel] = torch.randn(s.numel)
    e_old = eng.ef.clone()
    eng.arena.grad.copy_(g)
    eng.sync_now()
    u = g + wd * p / 0.5
    torch.testing.assert_close(eng.arena.grad + eng.ef, e_old + u, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(eng.mom, _mc_expect(eng, u, eng.arena.grad), rtol=1e-6, atol=1e-7)


def test_claimed_overwrite_skips_zeroing_once_whole_written():
    """engine.claim_overwrite: a segment whole-written by exactly one claim in a step is left out
    of the next begin_step's zeroing and may be overwritten; a second claim (a shared weight)
    puts it back under zeroing; a left-out segment nobody wrote is zeroed before the exchange."""
    m = small_net()
    eng = GradSyncEngine(list(m.named_parameters()), mode="layerwise", method="none")
    seg = eng.arena.segments[-1]                  # (the conv weight)
    view = eng.arena.grad_view(seg)
    eng.begin_step()
    assert eng.claim_overwrite(seg.index) is False          # nothing left unzeroed yet
    view.fill_(3.0)
    eng.begin_step()
    assert seg.index in eng._no_zero
    assert float(view.abs().min()) == 3.0                   # not zeroed: it will be overwritten
    others = [s for s in eng.arena.segments if s.index != seg.index]
    for s in others:
        eng.arena.grad_view(s).fill_(1.0)
    eng.begin_step()                                        # (no backward ran: same set)
    assert all(float(eng.arena.grad_view(s).abs().max()) == 0.0 for s in others)
    assert eng.claim_overwrite(seg.index) is True
    assert eng.claim_overwrite(seg.index) is False          # a second use accumulates
    eng.begin_step()
    assert seg.index not in eng._no_zero and float(view.abs().max()) == 0.0
    # left out but not written this step: zeroed in finish, before its bucket is exchanged
    eng._claims = [0] * len(eng.arena.segments)
    eng._claims[seg.index] = 1
    eng.begin_step()
    assert seg.index in eng._no_zero
    view.fill_(5.0)
    eng.finish()
    assert float(view.abs().max()) == 0.0


def test_fused_sgd_contract_is_enforced():
    """with the decode fused into the SGD step, a second backward before step(), or an
    LR change between backward and step(), raises instead of silently diverging."""
    import pytest as _pt
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    from layer_wise_aaai20_amd.parallel.arena import GradArena
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(10, 4)), torch.nn.Parameter(torch.randn(7))]
    arena = GradArena(list(zip(["a", "b"], ps)), flat_params=True)
    opt = FlatSGD(ps, arena, lr=0.1, momentum=0.9, nesterov=True)
    opt.exclude_segments([0])                 # as GradSyncEngine.set_fused_sgd leaves it
    opt.mark_fused_update(opt.fused_hyper())
    opt.step()                                # consumes the mark
    opt.mark_fused_update(opt.fused_hyper())
    with _pt.raises(RuntimeError, match="second backward"):
        opt.mark_fused_update(opt.fused_hyper())
    opt.param_groups[0]["lr"] = 0.05          # LR changed after backward
    with _pt.raises(RuntimeError, match="changed between backward"):
        opt.step()


def test_mc_mask_resets_whole_segments():
    """ADVICE r5 (pinned behaviour): on the k_mc_mask path (a threshold codec here) the velocity
    is zeroed wherever the residual is zero — a segment sent whole restarts its velocity every
    step, unlike Top-K's selection kernels, which keep momentum for whole segments."""
    from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine
    torch.manual_seed(0)
    ps = [("w", torch.nn.Parameter(torch.randn(64, 8))), ("b", torch.nn.Parameter(torch.randn(8)))]
    eng = GradSyncEngine(ps, mode="layerwise", method="Thresholdv", V=1e-12, error_feedback=True,
                         momentum_correction=0.9, bucket_cap_mb=1.0, flat_params=True)
    for _ in range(2):
        eng.arena.grad.copy_(torch.randn(eng.arena.numel).sign() * (1 + torch.rand(eng.arena.numel)))
        eng.sync_now()
        assert float(eng.ef.abs().max()) == 0.0        # every element above V: sent whole
        assert float(eng.mom.abs().max()) == 0.0       # ... so its velocity was reset
