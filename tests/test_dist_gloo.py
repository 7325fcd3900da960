"""Multi-process (gloo, CPU) data-parallel tests — BASELINE config 1 and the DP variants."""
import pytest
import torch

from dist_utils import run_world


def _batch(rank, n=4):
    g = torch.Generator().manual_seed(100 + rank)
    return {"input": torch.randn(n, 3, 32, 32, generator=g),
            "target": torch.randint(0, 10, (n,), generator=g)}


def _raw_grads(model, batch):
    model.zero_grad()
    model(batch)["loss"].sum().backward()
    return [p.grad.detach().clone() for p in model.parameters()]


def _w_topk_layerwise(rank, world, method, kw, ef):
    import torch.distributed as dist
    from layer_wise_aaai20_amd.compress import reference as ref
    from layer_wise_aaai20_amd.models import cifar
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    torch.manual_seed(rank)                     # different init per rank: DDP must broadcast
    m = cifar.build_network("resnet9")
    ref_model = cifar.build_network("resnet9")
    ddp = CompressedDDP(m, compress="layerwise", method=method, error_feedback=ef,
                        bucket_cap_mb=4, flat_params=False, **kw)
    ref_model.load_state_dict(m.state_dict())
    b = _batch(rank)
    raw = _raw_grads(ref_model, b)
    ddp(b)["loss"].sum().backward()
    got = [p.grad.detach().clone() for p in m.parameters()]
    # oracle: mean over ranks of each rank's reference-compressed gradient
    comp = [ref.compress(g.reshape(-1), method, **kw) for g in raw]
    allc = [[torch.zeros_like(c) for _ in range(world)] for c in comp]
    for c, a in zip(comp, allc):
        dist.all_gather(a, c)
    exp = [sum(a) / world for a in allc]
    params = [p.detach().clone() for p in m.parameters()]
    return got, exp, params


@pytest.mark.parametrize("method,kw", [("Topk", {"K": 0.01}), ("none", {}),
                                       ("Thresholdv", {"V": 0.01}),
                                       ("AdaptiveThreshold", {})])
def test_layerwise_world2_matches_oracle(method, kw):
    """BASELINE config 1: ResNet-9, layer-wise Top-K k=1%, gloo, world_size=2."""
    res = run_world(_w_topk_layerwise, 2, (method, kw, False))
    (g0, e0, p0), (g1, e1, p1) = res
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)                          # replicas start identical (D16 fixed)
    for a, b, e in zip(g0, g1, e0):
        assert torch.equal(a, b)                          # every rank holds the same gradient
        torch.testing.assert_close(a.reshape(-1), e, rtol=1e-5, atol=1e-7)


def _w_entire_ef(rank, world, method, kw, steps):
    from layer_wise_aaai20_amd.models import cifar
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    torch.manual_seed(0)
    m = cifar.build_network("alexnet")
    ddp = CompressedDDP(m, compress="entiremodel", method=method, error_feedback=True,
                        flat_params=True, **kw)
    opt = FlatSGD(m.parameters(), ddp.arena, lr=0.01, momentum=0.9, nesterov=True)
    losses = []
    for s in range(steps):
        out = ddp(_batch(rank * 10 + s, 8))
        out["loss"].sum().backward()
        opt.step()
        losses.append(float(out["loss"].mean()))
    return ([p.detach().clone() for p in m.parameters()], ddp.engine.ef.clone(), losses,
            ddp.engine.stats.payload_bytes, ddp.engine.stats.dense_bytes)


@pytest.mark.parametrize("method,kw", [("Topk", {"K": 0.01}), ("RandomDithering", {"qstates": 127}),
                                       ("TernGrad", {}), ("Randomk", {"K": 0.05})])
def test_entiremodel_error_feedback_world2(method, kw):
    """BASELINE config 3 flavour: AlexNet entire-model compression + error feedback."""
    (pa, ea, la, pay, dense), (pb, eb, lb, _, _) = run_world(_w_entire_ef, 2, (method, kw, 3))
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)                          # replicas stay bit-identical
    assert not torch.equal(ea, eb)                        # residuals are per-rank state
    assert float(ea.abs().sum()) > 0
    assert pay < dense


def _w_randk_ddp(rank, world):
    from layer_wise_aaai20_amd.models import cifar
    from layer_wise_aaai20_amd.parallel.ddp import RandomKSparsifiedDDP
    torch.manual_seed(0)
    m = cifar.build_network("resnet9")
    ddp = RandomKSparsifiedDDP(m, randk=0.05, seed=1234, flat_params=False)
    ddp(_batch(rank))["loss"].sum().backward()
    nz = [(p.grad != 0) for p in m.parameters()]
    return [p.grad.clone() for p in m.parameters()], nz, ddp.engine.codecs[0].name


def test_randomk_sparsified_ddp_world2():
    (g0, nz0, name), (g1, nz1, _) = run_world(_w_randk_ddp, 2)
    assert name == "randk"
    for a, b, m0, m1 in zip(g0, g1, nz0, nz1):
        assert torch.equal(a, b) and torch.equal(m0, m1)


def _w_cifar_train(rank, world, extra=()):
    import os
    import tempfile
    from layer_wise_aaai20_amd.train.cifar_main import main
    d = tempfile.mkdtemp()
    tsv = main(["-r", str(rank), "-w", str(world), "-n", "Resent9", "-c", "layerwise",
                "--method", "Topk", "-K", "0.01", "--synthetic", "--n_train", "256",
                "--n_test", "64", "--batch_size", "64", "--epochs", "2", "--log_dir", d,
                "--device", "cpu"] + list(extra))
    return str(tsv), open(os.path.join(d, "logs.tsv")).read()


def test_cifar_entrypoint_world2():
    (t0, f0), (t1, f1) = run_world(_w_cifar_train, 2)
    assert f0.splitlines()[0] == "epoch\thours\ttop1Accuracy"
    assert len(f0.splitlines()) == 3


def _w_cifar_batches(rank, world, full):
    from layer_wise_aaai20_amd.train import cifar_main
    seen = {}
    orig = cifar_main.D.GPUBatches

    def spy(*a, **kw):
        b = orig(*a, **kw)
        if kw.get("augment"):
            seen["shard"] = kw.get("shard")
            seen["n"] = len(b)
        return b
    cifar_main.D.GPUBatches = spy
    try:
        _w_cifar_train(rank, world, ["--full_data"] if full else [])
    finally:
        cifar_main.D.GPUBatches = orig
    return seen


def test_cifar_cli_shards_by_default():
    """Each rank trains on its own 1/W shard unless --full_data."""
    s = run_world(_w_cifar_batches, 2, (False,))
    assert [x["shard"] for x in s] == [(0, 2), (1, 2)]
    assert s[0]["n"] == s[1]["n"] == 2                  # 256 / 2 ranks / bs 64
    f = run_world(_w_cifar_batches, 2, (True,))
    assert [x["shard"] for x in f] == [(0, 1), (0, 1)] and f[0]["n"] == 4


def _w_agree(rank, world):
    from layer_wise_aaai20_amd.parallel import comm
    return comm.agree(True), comm.agree(rank != 1), comm.agree(False)


def test_agree_is_collective_and():
    for r in run_world(_w_agree, 2):
        assert r == (True, False, False)


def _w_dist_predict(rank, world):
    from layer_wise_aaai20_amd.data.imagenet import DistValSampler
    from layer_wise_aaai20_amd.train.imagenet_main import distributed_predict
    from torch import nn

    class R:
        pass
    R.world, R.rank = world, rank
    smp = DistValSampler(list(range(5)), 4, distributed=True)
    shards = [len(b) for b in smp]
    torch.manual_seed(0)
    model = nn.Linear(3, 4)
    n = len(smp.shard)
    x = torch.randn(n, 3)
    t = torch.zeros(n, dtype=torch.long)
    top1, top5, loss, total = distributed_predict(R(), x, t, model, nn.CrossEntropyLoss())
    return shards, total, top5


def test_distributed_predict_uneven():
    (s0, tot0, t5), (s1, tot1, _) = run_world(_w_dist_predict, 2)
    assert s0 == [4] and s1 == [1] and tot0 == tot1 == 5
    assert t5 == 100.0


def _w_count_exchange(rank, world):
    from layer_wise_aaai20_amd.compress import codecs
    from layer_wise_aaai20_amd.compress.plan import SegPlan
    from layer_wise_aaai20_amd.parallel import comm
    plan = SegPlan([0, 128], [100, 50])
    g = torch.zeros(192)
    g[: 10 * (rank + 1)] = 1.0                             # rank-dependent counts
    c = codecs.ThresholdCodec(plan, world, rank, V=0.5, count_exchange=comm.all_reduce_max)
    send = c.compress(g, None, 0)
    recv = torch.empty(send.numel() * world, dtype=send.dtype)
    comm.all_gather(recv, send).wait()
    out = torch.zeros(192)
    c.decompress(send, recv, out)
    return out, c.cap_off.tolist()


def test_threshold_count_exchange():
    (o0, c0), (o1, c1) = run_world(_w_count_exchange, 2)
    assert c0 == c1 == [0, 20, 20]
    assert torch.equal(o0, o1)
    assert torch.equal(o0[:10], torch.ones(10)) and torch.equal(o0[10:20], torch.full((10,), .5))


def _w_qrs(rank, world, mode, method, kw, steps):
    """The quantised reduce-scatter wire (codecs.QuantRSCodec) against the code all-gather wire
    on identical replicas: same codes (same Philox streams), so every step's averaged gradient is
    the all-gather wire's fp32 mean rounded to bf16, on every rank."""
    from layer_wise_aaai20_amd.compress.codecs import QuantRSCodec
    from layer_wise_aaai20_amd.models import cifar
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    torch.manual_seed(0)
    ma, mb = cifar.build_network("resnet9"), cifar.build_network("resnet9")
    mb.load_state_dict(ma.state_dict())
    qa = CompressedDDP(ma, compress=mode, method=method, wire="qrs", bucket_cap_mb=1,
                       flat_params=False, **kw)
    ga = CompressedDDP(mb, compress=mode, method=method, wire="sparse", bucket_cap_mb=1,
                       flat_params=False, **kw)
    assert all(isinstance(c, QuantRSCodec) for c in qa.engine.codecs)
    out = []
    for s in range(steps):
        b = _batch(rank * 10 + s)
        for d in (qa, ga):
            d.module.zero_grad()
            d(b)["loss"].sum().backward()
        got = [p.grad.detach().clone() for p in ma.parameters()]
        exp = [p.grad.detach().to(torch.bfloat16).float() for p in mb.parameters()]
        out.append((got, exp))
    return out, qa.engine.stats.payload_bytes, ga.engine.stats.payload_bytes


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode,method,kw", [("entiremodel", "RandomDithering", {"qstates": 255}),
                                            ("layerwise", "TernGrad", {}),
                                            ("layerwise", "RandomDithering", {"qstates": 4000})])
def test_quantised_reduce_scatter_wire(world, mode, method, kw):
    res = run_world(_w_qrs, world, (mode, method, kw, 2))
    for steps, pay_qrs, pay_ag in res:
        for got, exp in steps:
            for a, e in zip(got, exp):
                assert torch.equal(a, e), (a - e).abs().max()
        if world > 2 and kw.get("qstates") == 255:         # QSGD-255: fewer bytes than the
            assert pay_qrs < pay_ag * (world - 1)          # code all-gather from 3 ranks on
    for s in range(2):                                    # identical on every rank
        for r in res[1:]:
            for a, b in zip(res[0][0][s][0], r[0][s][0]):
                assert torch.equal(a, b)


def _w_buffer_sync(rank, world, sync):
    from layer_wise_aaai20_amd.models import cifar
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    torch.manual_seed(0)
    m = cifar.build_network("resnet9")
    ddp = CompressedDDP(m, compress="layerwise", method="Topk", K=0.01, buffer_sync=sync,
                        flat_params=False)
    for s in range(3):
        ddp(_batch(rank * 10 + s))["loss"].sum().backward()
    bufs = lambda: [b.detach().clone() for b in m.buffers() if b.is_floating_point()]  # noqa
    before = bufs()
    ddp.sync_buffers()
    after = bufs()
    ddp.eval()
    ddp(_batch(99))
    return before, after, bufs()


def test_lazy_buffer_sync_matches_per_step_broadcast():
    """BN running statistics are broadcast where they are read (evaluation,
    checkpoints), not before every training forward. Rank 0's buffers — the ones every rank holds
    at those points — are the reference's per-forward-broadcast values exactly."""
    lazy = run_world(_w_buffer_sync, 2, ("lazy",))
    step = run_world(_w_buffer_sync, 2, ("step",))
    (b0, a0, e0), (b1, a1, e1) = lazy
    assert any(not torch.equal(x, y) for x, y in zip(b0, b1))     # rank-local during training
    for x, y in zip(a0, a1):
        assert torch.equal(x, y)                                  # synced to rank 0's
    for x, y in zip(a0, step[0][1]):
        assert torch.equal(x, y)                                  # = the reference's values
    for x, y in zip(e0, e1):
        assert torch.equal(x, y)
