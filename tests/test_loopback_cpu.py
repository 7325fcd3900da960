"""The loopback communicator (``parallel/loopback.py``) on CPU: one engine at a simulated world of
4 ranks whose 3 peers compress stored gradients with codecs built for their own ranks. Checks the
multi-rank result the real collectives must produce (``tests/test_dist_world8.py`` invariants):
one collective per bucket in bucket order, and the decoded arena equals the mean over ranks of what
each rank sent — ``g_r + e_r(before) - e_r(after)`` with error feedback, the reference compressor's
mean (``CIFAR10/core.py:175-225``) without."""
import pytest
import torch

from layer_wise_aaai20_amd.compress import reference as ref
from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine
from layer_wise_aaai20_amd.parallel.loopback import attach_loopback

W = 4
METHODS = [("none", {}), ("Topk", {"K": 0.05}), ("Randomk", {"K": 0.1}),
           ("Thresholdv", {"V": 0.5}), ("AdaptiveThreshold", {}), ("TernGrad", {}),
           ("RandomDithering", {"qstates": 127}), ("RandomDithering", {"qstates": 255})]


def _params():
    torch.manual_seed(0)
    shapes = [(16, 3, 3, 3), (16,), (32, 16, 3, 3), (32,), (10, 32), (10,)]
    return [(f"p{i}", torch.nn.Parameter(torch.randn(s))) for i, s in enumerate(shapes)]


def _grads(eng, seed):
    g = torch.Generator().manual_seed(seed)
    out = torch.zeros(eng.arena.numel)
    for s in eng.arena.segments:
        out[s.offset:s.offset + s.numel] = torch.randn(s.numel, generator=g)
    return out


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("ef", [False, True])
@pytest.mark.parametrize("method,kw", METHODS,
                         ids=[f"{m}{kw.get('qstates', '')}" for m, kw in METHODS])
def test_loopback_world4(method, kw, mode, ef):
    if method == "none" and ef:
        pytest.skip("no residual without compression")
    eng = GradSyncEngine(_params(), mode=mode, method=method, error_feedback=ef,
                         bucket_cap_mb=0.01, world_size=W, **kw)
    if mode == "layerwise":
        assert len(eng.buckets) > 1
    peers = [_grads(eng, 100 + r) for r in range(1, W)]
    lb = attach_loopback(eng, peers)
    g0 = _grads(eng, 100)
    for step in range(3):                                # residuals evolve over steps
        eng.arena.grad.copy_(g0)
        e_old = [eng.ef.clone() if ef else None] + \
            [e.clone() if e is not None else None for e in lb.sim.ef]
        lb.calls.clear()
        eng.sync_now()
        got = eng.arena.grad.clone()
        kinds = {c[0] for c in lb.calls}
        # (the quantised reduce-scatter wire: two grouped send/recv phases per bucket)
        per = 2 if kinds == {"send_recv1", "send_recv2"} else 1
        assert [c[1] for c in lb.calls] == [b for b in range(len(eng.buckets))
                                             for _ in range(per)]
        assert len(kinds) == per
        raw = [g0] + peers
        if ef:
            e_new = [eng.ef] + lb.sim.ef
            sent = sum(raw[r] + e_old[r] - e_new[r] for r in range(W)) / W
            if per == 2:                                 # bf16-rounded mean on that wire
                torch.testing.assert_close(got, sent.to(torch.bfloat16).float(),
                                           rtol=2 ** -7, atol=1e-6)
            else:
                torch.testing.assert_close(got, sent, rtol=1e-5, atol=1e-6)
            assert float(eng.ef.abs().sum()) > 0 or method == "none"
        elif method in ("none", "Topk", "Thresholdv", "AdaptiveThreshold"):
            exp = torch.zeros_like(got)
            for r in range(W):
                if mode == "entiremodel":
                    exp += ref.compress(raw[r], method, **kw)
                else:
                    for s in eng.arena.segments:
                        sl = slice(s.offset, s.offset + s.numel)
                        exp[sl] += ref.compress(raw[r][sl], method, **kw)
            torch.testing.assert_close(got, exp / W, rtol=1e-5, atol=1e-6)
        elif method == "Randomk":
            nz = got != 0                                # shared-seed support: the rank mean there
            mean = sum(raw) / W
            torch.testing.assert_close(got[nz], mean[nz], rtol=1e-5, atol=1e-6)
        else:                                            # unbiased quantisers: finite, bounded
            assert torch.isfinite(got).all()


def test_loopback_rejects_world_mismatch():
    eng = GradSyncEngine(_params(), mode="layerwise", method="Topk", K=0.1, world_size=2)
    with pytest.raises(ValueError):
        attach_loopback(eng, [_grads(eng, 1), _grads(eng, 2)])


@pytest.mark.parametrize("method,kw", [("Thresholdv", {"V": 0.5}), ("AdaptiveThreshold", {})])
@pytest.mark.parametrize("density", [1.0, 0.02])
def test_fixed_capacity_threshold_wire(method, kw, density, monkeypatch):
    """The graph-capturable sparse threshold wire (fixed per-segment capacity): with room for
    every hit it equals the exact dense-wire result; with too little room the hits that do not
    fit stay in the error-feedback residual, so decoded == mean_r(what each rank sent)."""
    res = {}
    for wire in ("dense", "sparse-capped"):
        eng = GradSyncEngine(_params(), mode="layerwise", method=method, error_feedback=True,
                             bucket_cap_mb=0.01, world_size=W, wire=wire,
                             max_density=density if wire == "sparse-capped" else None, **kw)
        if wire == "sparse-capped":
            assert all(c.graph_safe and c.name == "threshold" for c in eng.codecs)
        peers = [_grads(eng, 100 + r) for r in range(1, W)]
        lb = attach_loopback(eng, peers)
        g0 = _grads(eng, 100)
        eng.arena.grad.copy_(g0)
        e_old = [eng.ef.clone()] + [e.clone() for e in lb.sim.ef]
        eng.sync_now()
        e_new = [eng.ef] + lb.sim.ef
        sent = sum(([g0] + peers)[r] + e_old[r] - e_new[r] for r in range(W)) / W
        torch.testing.assert_close(eng.arena.grad, sent, rtol=1e-5, atol=1e-6)
        res[wire] = eng.arena.grad.clone()
    if density == 1.0:
        torch.testing.assert_close(res["sparse-capped"], res["dense"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("method,kw", [("RandomDithering", {"qstates": 255}), ("TernGrad", {}),
                                       ("RandomDithering", {"qstates": 4000})])
@pytest.mark.parametrize("world", [4, 8])
def test_loopback_quantised_reduce_scatter(method, kw, mode, world):
    """The quantised reduce-scatter wire at a simulated world of 4 / 8: the decoded arena is
    the code all-gather wire's mean rounded to bf16 (same codes: same Philox streams), the
    exchange is two grouped send/recv phases per bucket, and it moves fewer bytes than the
    all-gather of codes whenever the factory picks it."""
    from layer_wise_aaai20_amd.compress.codecs import QuantRSCodec
    engs, lbs = [], []
    for wire in ("qrs", "sparse"):
        e = GradSyncEngine(_params(), mode=mode, method=method, bucket_cap_mb=0.01,
                           world_size=world, wire=wire, **kw)
        peers = [_grads(e, 100 + r) for r in range(1, world)]
        lbs.append(attach_loopback(e, peers))
        engs.append(e)
    assert all(isinstance(c, QuantRSCodec) for c in engs[0].codecs)
    g0 = _grads(engs[0], 100)
    for step in range(2):
        for e, lb in zip(engs, lbs):
            e.arena.grad.copy_(g0)
            lb.calls.clear()
            e.sync_now()
        q, a = engs[0].arena.grad, engs[1].arena.grad
        assert torch.equal(q, a.to(torch.bfloat16).float()), (q - a).abs().max()
        assert [c[0] for c in lbs[0].calls] == ["send_recv1", "send_recv2"] * len(engs[0].buckets)
    if method == "RandomDithering" and kw["qstates"] == 255 and mode == "entiremodel":
        assert engs[0].stats.payload_bytes < engs[1].stats.payload_bytes * (world - 1)


def test_graph_overlap_modes():
    """LWAAAI_GRAPH_OVERLAP=auto is the measured winner with the wire priced in (inline, "0"),
    at any world size and with any communicator; "1" / "comm" remain selectable."""
    from layer_wise_aaai20_amd.parallel.loopback import WireModel
    e1 = GradSyncEngine(_params(), mode="layerwise", method="Topk", K=0.05)
    assert e1.graph_overlap_mode() == "0"
    e = GradSyncEngine(_params(), mode="layerwise", method="Topk", K=0.05, world_size=4)
    lb = attach_loopback(e, [_grads(e, 100 + r) for r in range(1, 4)])
    assert e.graph_overlap_mode() == "0"
    lb.wire_model = WireModel()
    e.set_graph_overlap("auto")
    assert e.graph_overlap_mode() == "0"
    e.set_graph_overlap("1")
    assert e.graph_overlap_mode() == "1"
    e.set_graph_overlap("comm")
    assert e.graph_overlap_mode() == "comm"
    with pytest.raises(ValueError):
        e.set_graph_overlap("sideways")
