"""HIP kernels vs the CPU (torch/numpy) mirror implementation and vs the reference oracles.

Selection (Top-K, Random-K, thresholds) and TernGrad packing must be bit-identical between the
GPU kernels and the CPU path; QSGD is compared to tolerance because the L2 norm is summed in a
different order.
"""
import numpy as np
import pytest
import torch

from layer_wise_aaai20_amd.compress import codecs
from layer_wise_aaai20_amd.compress import reference as ref
from layer_wise_aaai20_amd.compress.plan import SegPlan

pytestmark = pytest.mark.gpu

SIZES = [64, 3, 1000, 4096, 4097, 9408, 65536, 147456, 1000, 2359296 // 4]


def make_plan(sizes, align=64):
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + align - 1) // align * align
    return SegPlan(offs, sizes), o


def rand_grad(n, seed=0, scale=1e-2):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, generator=g) * scale


@pytest.mark.parametrize("K", [0.001, 0.01, 0.25])
@pytest.mark.parametrize("ef", [False, True])
def test_topk_gpu_matches_cpu(K, ef):
    plan, N = make_plan(SIZES)
    x = rand_grad(N, 1)
    e = rand_grad(N, 2, 1e-3) if ef else None
    cc, cg = codecs.TopkCodec(plan, 1, 0, K), codecs.TopkCodec(plan, 1, 0, K)
    xc, ec = x.clone(), (e.clone() if ef else None)
    pc = cc.compress(xc, ec, 0).clone()
    xg, eg = x.cuda(), (e.cuda() if ef else None)
    pg = cg.compress(xg, eg, 0).cpu()
    assert torch.equal(pc, pg)
    if ef:
        torch.testing.assert_close(ec, eg.cpu(), rtol=0, atol=0)
    # decoded == reference oracle on g + e
    out = torch.zeros(N, device="cuda")
    cg.decompress(pg.cuda(), None, out, world=1)
    out = out.cpu()
    base = x + e if ef else x
    for s in range(plan.S):
        o, n = int(plan.offsets[s]), int(plan.sizes[s])
        assert torch.equal(out[o:o + n], ref.topk(base[o:o + n], K)), s


def test_topk_ties_and_zeros():
    plan, N = make_plan([5000, 200, 20000])
    x = torch.zeros(N)
    x[:3000] = 1.0          # heavy ties at the threshold
    x[3000:3010] = 2.0
    x[5120:5130] = torch.arange(10).float()
    cc, cg = codecs.TopkCodec(plan, 1, 0, 0.01), codecs.TopkCodec(plan, 1, 0, 0.01)
    pc = cc.compress(x.clone(), None, 0).clone()
    pg = cg.compress(x.cuda(), None, 0).cpu()
    assert torch.equal(pc, pg)


@pytest.mark.parametrize("K", [0.001, 0.05])
@pytest.mark.parametrize("ef", [False, True])
def test_randk_gpu_matches_cpu(K, ef):
    plan, N = make_plan(SIZES)
    x = rand_grad(N, 3)
    e = rand_grad(N, 4, 1e-3) if ef else None
    cc = codecs.RandkCodec(plan, 1, 0, K, seed=77)
    cg = codecs.RandkCodec(plan, 1, 0, K, seed=77)
    ec = e.clone() if ef else None
    vc = cc.compress(x.clone(), ec, 9).clone()
    eg = e.cuda() if ef else None
    vg = cg.compress(x.cuda(), eg, 9).cpu()
    assert torch.equal(cc._idx["cpu"], cg._idx["cuda:0"].cpu())
    assert torch.equal(vc, vg)
    if ef:
        assert torch.equal(ec, eg.cpu())
    out = torch.zeros(N, device="cuda")
    cg.decompress(vg.cuda(), None, out, world=1)
    for s in range(plan.S):
        o, n = int(plan.offsets[s]), int(plan.sizes[s])
        assert int((out[o:o + n] != 0).sum()) <= ref.randomk_keep_count(n, K)


@pytest.mark.parametrize("world", [2, 8])
def test_unpack_pairs_rank_ordered(world):
    plan, N = make_plan(SIZES)
    c = codecs.TopkCodec(plan, world, 0, 0.01)
    payloads = []
    for r in range(world):
        payloads.append(codecs.TopkCodec(plan, 1, 0, 0.01).compress(rand_grad(N, 10 + r), None, 0)
                        .clone())
    gathered = torch.cat(payloads)
    oc = torch.zeros(N)
    c.unpack_pairs_cpu(gathered, world, oc, c.cap_off)
    og = torch.zeros(N, device="cuda")
    c.decompress(None, gathered.cuda(), og, world=world)
    assert torch.equal(oc, og.cpu())


def test_terngrad_bitwise():
    plan, N = make_plan(SIZES)
    x = rand_grad(N, 5)
    cc = codecs.TernGradCodec(plan, 1, 3, seed=11)
    cg = codecs.TernGradCodec(plan, 1, 3, seed=11)
    pc = cc.compress(x.clone(), None, 2).clone()
    pg = cg.compress(x.cuda(), None, 2).cpu()
    assert torch.equal(pc, pg)
    oc = torch.zeros(N)
    og = torch.zeros(N, device="cuda")
    cc.decompress(None, torch.cat([pc, pc]), oc, world=2)
    cg.decompress(None, torch.cat([pg, pg]).cuda(), og, world=2)
    torch.testing.assert_close(oc, og.cpu())


@pytest.mark.parametrize("qstates", [127, 255, 1000])
def test_qsgd_close(qstates):
    plan, N = make_plan(SIZES)
    x = rand_grad(N, 6)
    cc = codecs.QSGDCodec(plan, 1, 0, qstates, seed=5)
    cg = codecs.QSGDCodec(plan, 1, 0, qstates, seed=5)
    e_c, e_g = torch.zeros(N), torch.zeros(N, device="cuda")
    pc = cc.compress(x.clone(), e_c, 1).clone()
    pg = cg.compress(x.cuda(), e_g, 1).cpu()
    hdr = cc.hdr
    torch.testing.assert_close(pc[:plan.S].view(torch.float32), pg[:plan.S].view(torch.float32),
                               rtol=1e-5, atol=0)
    mism = (pc[hdr:] != pg[hdr:]).float().mean().item()
    assert mism < 2e-3, mism
    og = torch.zeros(N, device="cuda")
    cg.decompress(pg.cuda(), None, og, world=1)
    # EF identity on every real element: decoded + residual == input
    for s in range(plan.S):
        o, n = int(plan.offsets[s]), int(plan.sizes[s])
        torch.testing.assert_close((og + e_g)[o:o + n], x.cuda()[o:o + n], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("adaptive", [False, True])
def test_threshold_gpu_matches_cpu(adaptive):
    plan, N = make_plan(SIZES)
    x = rand_grad(N, 7)
    kw = dict(adaptive=True) if adaptive else dict(V=0.02)
    cc = codecs.ThresholdCodec(plan, 1, 0, **kw)
    cg = codecs.ThresholdCodec(plan, 1, 0, **kw)
    pc = cc.compress(x.clone(), None, 0).clone()
    pg = cg.compress(x.cuda(), None, 0).cpu()
    assert torch.equal(pc, pg)


def test_flat_sgd_matches_torch():
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    from layer_wise_aaai20_amd.parallel.arena import GradArena
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8),
                             torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 10)).cuda()
    m2 = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8),
                             torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 10)).cuda()
    m2.load_state_dict(m1.state_dict())
    arena = GradArena(list(m2.named_parameters()), flat_params=True)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-3)
    o2 = FlatSGD(m2.parameters(), arena, lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-3)
    x = torch.randn(4, 3, 8, 8, device="cuda")
    for _ in range(3):
        o1.zero_grad()
        m1(x).square().mean().backward()
        arena.zero_()
        m2(x).square().mean().backward()
        o1.step()
        o2.step()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p1, p2, rtol=1e-5, atol=1e-6)


def test_normalize_u8():
    from layer_wise_aaai20_amd.ops.nn import normalize_nhwc_u8
    x = torch.randint(0, 256, (3, 17, 13, 3), dtype=torch.uint8, device="cuda")
    mean = torch.tensor([120.0, 110.0, 100.0])
    std = torch.tensor([60.0, 61.0, 62.0])
    y = normalize_nhwc_u8(x, mean, std, torch.float32)
    ref_ = (x.permute(0, 3, 1, 2).float().cpu() - mean.view(1, 3, 1, 1)) / std.view(1, 3, 1, 1)
    torch.testing.assert_close(y.cpu(), ref_, rtol=1e-6, atol=1e-5)
    yb = normalize_nhwc_u8(x, mean, std, torch.bfloat16)
    torch.testing.assert_close(yb.float().cpu(), ref_, rtol=1e-2, atol=1e-2)
    assert yb.is_contiguous(memory_format=torch.channels_last)


def test_resnet50_step_topk_gpu():
    from layer_wise_aaai20_amd.ops import _ext
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    _ext.load()
    tr = build_trainer("resnet50", device=torch.device("cuda", 0), K=0.001)
    imgs = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, device="cuda")
    tgt = torch.randint(0, 1000, (16,), device="cuda")
    losses = [float(tr.step(imgs, tgt)) for _ in range(3)]
    assert all(np.isfinite(losses))
    st = tr.ddp.sync_stats()
    assert st.payload_bytes < st.dense_bytes * 0.01


def test_invalid_launch_raises():
    """Every binding checks hipGetLastError after its launches: a rejected launch configuration
    surfaces as a RuntimeError at the op that caused it."""
    from layer_wise_aaai20_amd.ops._ext import load
    with pytest.raises(RuntimeError, match="launch failed"):
        load().selftest_bad_launch(torch.empty(1, device="cuda"))
    torch.cuda.synchronize()            # not sticky: the device keeps working
    assert torch.ones(4, device="cuda").sum().item() == 4


@pytest.mark.parametrize("adaptive", [False, True])
@pytest.mark.parametrize("with_ef", [False, True])
def test_threshold_dense_in_place_matches_cpu(adaptive, with_ef):
    """Threshold methods on the dense wire: the GPU kernel (k_thresh_dense) and the CPU mirror
    produce the same compressed vector and residual."""
    torch.manual_seed(0)
    sizes = [5000, 64, 20000, 9000]
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).tolist()
    plan = SegPlan(offs, sizes)
    g = torch.randn(sum(sizes)) * 0.01
    ef = torch.randn(sum(sizes)) * 0.001 if with_ef else None
    c = codecs.ThresholdCodec(plan, 1, 0, V=0.005, adaptive=adaptive)
    gc, ec = g.clone(), (ef.clone() if with_ef else None)
    c.compress_dense(gc, ec)
    gg, eg = g.cuda(), (ef.cuda() if with_ef else None)
    c.compress_dense(gg, eg)
    assert torch.equal(gg.cpu(), gc)
    if with_ef:
        assert torch.equal(eg.cpu(), ec)
    assert 0 < int((gc != 0).sum()) < gc.numel()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cifar_augment_kernel_matches_torch_gathers(dtype):
    """csrc/augment.hip (random crop + flip + cutout into a channels_last batch) against the
    torch gather path of GPUBatches with the same per-epoch choices."""
    from layer_wise_aaai20_amd.data.cifar import GPUBatches
    torch.manual_seed(0)
    data = torch.randn(300, 3, 40, 40, device="cuda")
    labels = torch.randint(0, 10, (300,), device="cuda")
    outs = []
    for kern in (True, False):
        gb = GPUBatches(data, labels, 64, shuffle=True, augment=True, seed=5,
                        channels_last=True, dtype=dtype)
        gb.use_kernel = kern
        assert gb._kernel_ok() == kern
        outs.append([(b["input"], b["target"]) for b in gb])
    assert len(outs[0]) == len(outs[1]) == 5
    for (xk, tk), (xt, tt) in zip(*outs):
        assert xk.is_contiguous(memory_format=torch.channels_last) and xk.dtype == dtype
        assert torch.equal(tk, tt)
        assert torch.equal(xk, xt)


def test_cifar_augment_pad4_zero_channel():
    """pad4: the same augmented batch with a zero 4th channel (the MFMA image convolution's
    input layout, ops/conv.py _c4_input), bit for bit in its first three channels."""
    from layer_wise_aaai20_amd.data.cifar import GPUBatches
    torch.manual_seed(0)
    data = torch.randn(200, 3, 40, 40, device="cuda")
    labels = torch.randint(0, 10, (200,), device="cuda")
    outs = []
    for pad4 in (False, True):
        gb = GPUBatches(data, labels, 64, shuffle=True, augment=True, seed=3,
                        channels_last=True, dtype=torch.bfloat16, pad4=pad4)
        outs.append([b["input"] for b in gb])
    for x3, x4 in zip(*outs):
        assert x4.shape[1] == 4 and x4.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(x4[:, :3], x3)
        assert int((x4[:, 3] != 0).sum()) == 0


@pytest.mark.parametrize("M,C", [(512, 64), (1000, 2048), (512, 4096), (96, 6144)])
def test_relu_bias_bwd_matches_torch(M, C):
    """csrc/nn.hip k_relu_bias_bwd (the bias + ReLU epilogue backward, channel slices of 2048 for
    the 4096-wide classifier layers): dy·[y > 0] bit for bit and the fp32 bias gradient, also
    accumulated into a given buffer."""
    from layer_wise_aaai20_amd.ops._ext import h16, load
    torch.manual_seed(0)
    dy = torch.randn(M, C, device="cuda").to(h16())
    y = torch.randn(M, C, device="cuda").to(h16())
    dym, db = load().relu_bias_bwd(dy, y, None)
    ref = dy * (y > 0)
    assert torch.equal(dym, ref)
    exp = ref.float().sum(0)
    assert torch.allclose(db, exp, rtol=1e-5, atol=1e-3)
    acc = torch.ones(C, device="cuda")
    load().relu_bias_bwd(dy, y, acc)
    assert torch.allclose(acc, exp + 1, rtol=1e-5, atol=1e-3)


def _kc_jobs():
    """(weight, cls, sh, sw, kmax) of every pack_dgrad_kc form a step asks for: 1x1 Wᵀ, a 3x3/1
    slab, the four parity classes of a 3x3/2 and of a strided 1x1, the flipped 3x3 window."""
    from layer_wise_aaai20_amd.ops import conv as CV
    from layer_wise_aaai20_amd.ops._ext import h16
    torch.manual_seed(0)
    CL = torch.channels_last
    jobs = []
    for k, n in [(256, 64), (64, 256), (1000, 512), (24, 40)]:
        w = torch.randn(k, n, device="cuda").to(h16())
        jobs.append((w.reshape(k, n, 1, 1), [0, 0, 1, 1], 1, 1, -(-k // 8) * 8))
    for co, c, R, st, pad, hw in [(64, 64, 3, 1, 1, 56), (128, 64, 3, 2, 1, 56),
                                  (256, 128, 1, 2, 0, 28)]:
        w = torch.randn(co, c, R, R, device="cuda").to(h16()).contiguous(memory_format=CL)
        classes = CV._dgrad_classes(hw, hw, R, R, st, st, pad, pad)
        cls = []
        for (_c, _w, r0, s0, TR, TS, *_x) in classes:
            cls += [r0, s0, TR, TS]
        kmax = -(-max(TR * TS * co for (_c, _w, _r, _s, TR, TS, *_x) in classes) // 8) * 8
        jobs.append((w, cls, st, st, kmax))
        jobs.append((w, cls, st, st, 0))            # the [K][C] slabs (pack_dgrad_nkc)
        if R == 3 and st == 1:
            jobs.append((w, [2, 2, 3, 3], -1, -1, 9 * co))
    return jobs


def test_pack_kc_multi_matches_single_packs():
    """csrc/conv.hip k_pack_kc_multi (a step's data-gradient weight packs in one launch,
    ops/conv.py kc_pack) against one pack_dgrad_kc per weight, bit for bit (zero-padded rows)."""
    from layer_wise_aaai20_amd.ops import conv as CV
    from layer_wise_aaai20_amd.ops._ext import load
    jobs = _kc_jobs()
    outs, prm = [], []
    for w, cls, sh, sw, kmax in jobs:
        nc = len(cls) // 4
        c4 = cls + [0] * (16 - len(cls))
        n = (nc * w.shape[1] * kmax if kmax else
             sum(cls[4 * i + 2] * cls[4 * i + 3] for i in range(nc)) * w.shape[0] * w.shape[1])
        outs.append(torch.empty(n, dtype=w.dtype, device="cuda"))
        prm += [sh, sw, kmax, nc] + c4[0::4] + c4[1::4] + c4[2::4] + c4[3::4]
    load().pack_kc_multi([j[0] for j in jobs], outs, prm)
    for (w, cls, sh, sw, kmax), o in zip(jobs, outs):
        assert torch.equal(o, CV._pack1(load(), w, cls, sh, sw, kmax))


def test_kc_pack_step_batch_follows_weight_updates():
    """ops/conv.py kc_pack: within engine steps the second step's packs come from the batched
    launch and equal fresh packs of the weights as updated in place between the steps; outside
    a step (kc_end_step) every request packs afresh."""
    from layer_wise_aaai20_amd.ops import conv as CV
    from layer_wise_aaai20_amd.ops._ext import load
    jobs = _kc_jobs()
    try:
        for step in range(3):
            CV.kc_new_step()
            for w, cls, sh, sw, kmax in jobs:
                got = CV.kc_pack(w, cls, sh, sw, kmax)
                assert torch.equal(got, CV._pack1(load(), w, cls, sh, sw, kmax)), step
            if step >= 1:
                assert len(CV._KC["reg"]) == len(jobs)
            CV.kc_end_step()
            for w, *_ in jobs:
                w.mul_(0.5).add_(0.25)      # the optimizer's in-place update
        w, cls, sh, sw, kmax = jobs[0]
        before = dict(CV._KC["cache"])
        CV.kc_pack(w, cls, sh, sw, kmax)
        assert CV._KC["cache"].keys() == before.keys() and \
            all(CV._KC["cache"][k] is v for k, v in before.items())   # unarmed: untouched
    finally:
        CV.kc_end_step()
        CV._KC.update(reg={}, cache={}, used=set())


@pytest.mark.parametrize("method,q", [("QSGD", 127), ("QSGD", 255), ("QSGD", 4000),
                                      ("TernGrad", None)])
@pytest.mark.parametrize("align", [64, 1])
def test_dequant_shard_matches_cpu_mirror(method, q, align):
    """k_dequant_shard (quantised reduce-scatter receive side) vs the CPU mirror, bit for bit, on
    CPU-made payloads of 5 ranks: every shard's bf16 mean, and the assembled bucket image expanded
    by k_bf16_expand equals the all-gather decode rounded to bf16."""
    W = 5
    plan, N = make_plan(SIZES, align)
    cs = [codecs.make_codec(method, plan, W, r, qstates=q, wire="qrs", seed=9) for r in range(W)]
    pays = [c.compress(rand_grad(N, 40 + r), None, 3).clone() for r, c in enumerate(cs)]
    img_c = torch.zeros(cs[0].n, dtype=torch.bfloat16)
    img_g = torch.zeros(cs[0].n, dtype=torch.bfloat16, device="cuda")
    for r, c in enumerate(cs):
        r1 = torch.zeros(W * c.wpr[r], dtype=torch.int32)
        rows = r1.view(W, -1)
        for p in range(W):
            for d, x in zip(c.piece_slots(rows[p], r), c.pieces(pays[p], r)):
                d.copy_(x)
        c.reduce_shard(r1, r, img_c)
        c.reduce_shard(r1.cuda(), r, img_g)
    assert torch.equal(img_c, img_g.cpu())
    ag = codecs.make_codec(method, plan, W, 0, qstates=q, wire="sparse", seed=9)
    ref16 = torch.zeros(N)
    ag.decompress(None, torch.cat(pays), ref16, world=W)
    out = torch.zeros(N, device="cuda")
    cs[0].decompress(None, img_g, out)
    assert torch.equal(out.cpu(), ref16.to(torch.bfloat16).float())


def test_wire_wait_holds_the_stream():
    """The loopback wire model's busy kernel (k_wire_wait) lasts at least the requested time."""
    from layer_wise_aaai20_amd.ops._ext import load
    lib = load()
    dev = torch.empty(0, device="cuda")
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lib.wire_wait(dev, 50.0, 16)
    a.record()
    lib.wire_wait(dev, 300.0, 16)
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b)
    assert 0.29 <= ms < 5.0, ms


def test_splitk_discard_drops_queued_reduces():
    """split-K reduces queued by a step that never reached its flush are dropped
    (splitk_discard) instead of being added into the next step's arena."""
    from layer_wise_aaai20_amd.ops import _ext
    from layer_wise_aaai20_amd.ops.block import gemm
    lib = _ext.load()
    torch.manual_seed(0)
    M, N, K = 128, 256, 8192
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    dst = torch.zeros(M, N, device="cuda")
    _ext.set_splitk_defer(dst, True)
    try:
        gemm(a, M, False, b, N, False, M, N, K, out_bf16=False, out=dst, accumulate=True,
             split_k=True)
    finally:
        _ext.set_splitk_defer(dst, False)
    if _ext.splitk_pending() == 0:
        pytest.skip("the tuner picked an unsplit tile: nothing was deferred")
    assert _ext.splitk_discard(dst) >= 1
    assert _ext.splitk_pending() == 0
    assert int(lib.splitk_flush(dst)) == 0
    torch.cuda.synchronize()
    assert float(dst.abs().max()) == 0.0            # nothing was reduced into the target
