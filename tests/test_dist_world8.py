"""Eight gloo ranks (CPU) through the CompressedDDP hook path — the multi-rank invariants of the
reference's DDPs (``IMAGENET/training/ddp.py:312-327,434-450``, ``sparsified_ddp.py:403-452``):

* every method x {layerwise, entiremodel} x {EF off, on}: gradients bit-identical on all ranks;
* buckets launch strictly in bucket order, and exactly one collective per bucket per step is
  issued (no double reduce);
* values: deterministic methods without EF equal the mean over ranks of the reference
  compressor (``CIFAR10/core.py:175-225``); WITH error feedback every method (the random ones
  too) satisfies decoded == mean_r(g_r - e_r), i.e. what each rank sent is exactly its
  gradient minus its new residual.
"""
import pytest
import torch

from dist_utils import run_world

METHODS = [("none", {}), ("Topk", {"K": 0.05}), ("Randomk", {"K": 0.1}),
           ("Thresholdv", {"V": 0.02}), ("AdaptiveThreshold", {}), ("TernGrad", {}),
           ("RandomDithering", {"qstates": 127})]
CONFIGS = [(m, kw, mode, ef) for m, kw in METHODS for mode in ("layerwise", "entiremodel")
           for ef in (False, True) if not (m == "none" and ef)]


def _net():
    from torch import nn
    return nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.Conv2d(8, 16, 3, stride=2),
                         nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(16, 10))


def _w_all(rank, world):
    import torch.distributed as dist
    import torch.nn.functional as F
    from layer_wise_aaai20_amd.parallel import comm, engine as E
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    calls = []
    real_ar, real_ag = comm.all_reduce, comm.all_gather

    def ar(t, pg=None):
        calls.append("all_reduce")
        return real_ar(t, pg)

    def ag(out, t, pg=None):
        calls.append("all_gather")
        return real_ag(out, t, pg)
    E.comm.all_reduce, E.comm.all_gather = ar, ag
    real_sr = comm.C10dP2P.send_recv

    def sr(self, *a, **k):
        calls.append("send_recv")           # (the quantised reduce-scatter wire: 2 per bucket)
        return real_sr(self, *a, **k)
    comm.C10dP2P.send_recv = sr
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.randn(6, 3, 12, 12, generator=g)
    y = torch.randint(0, 10, (6,), generator=g)
    results = []
    for method, kw, mode, ef in CONFIGS:
        torch.manual_seed(rank)                          # different init: DDP must broadcast
        m = _net()
        ddp = CompressedDDP(m, compress=mode, method=method, error_feedback=ef,
                            bucket_cap_mb=0.002, flat_params=False, **kw)
        ref = _net()
        ref.load_state_dict(m.state_dict())
        F.cross_entropy(ref(x), y).backward()
        raw = [p.grad.detach().clone() for p in ref.parameters()]
        launched = []
        real_launch = ddp.engine._launch

        def launch(bi, real_launch=real_launch):
            launched.append(bi)
            return real_launch(bi)
        ddp.engine._launch = launch
        calls.clear()
        F.cross_entropy(ddp(x), y).backward()
        got = [p.grad.detach().clone() for p in m.parameters()]
        eng = ddp.engine
        efs = None
        if eng.ef is not None:
            efs = [eng.ef[eng.arena.by_param[id(p)].offset:
                          eng.arena.by_param[id(p)].offset + p.numel()].view_as(p).clone()
                   for p in m.parameters()]
        # everyone's raw gradients (and residuals) for the oracle
        all_raw = []
        for t in raw:
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t.contiguous())
            all_raw.append(parts)
        all_ef = None
        if efs is not None:
            all_ef = []
            for t in efs:
                parts = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(parts, t.contiguous())
                all_ef.append(parts)
        results.append({"got": got, "launched": launched, "calls": list(calls),
                        "nbuckets": len(eng.buckets), "raw": all_raw, "ef": all_ef,
                        "payload": eng.stats.payload_bytes, "dense": eng.stats.dense_bytes})
    return results


@pytest.fixture(scope="module")
def world8():
    return run_world(_w_all, 8)


def _oracle_plain(raw_per_rank, method, kw, mode):
    from layer_wise_aaai20_amd.compress import reference as ref
    world = len(raw_per_rank[0])
    if mode == "layerwise":
        return [sum(ref.compress(r.reshape(-1), method, **kw) for r in parts).view_as(parts[0])
                / world for parts in raw_per_rank]
    # entire model: one compressor call over the concatenation in arena (reverse) order
    flat = [torch.cat([parts[r].reshape(-1) for parts in reversed(raw_per_rank)])
            for r in range(world)]
    mean = sum(ref.compress(f, method, **kw) for f in flat) / world
    out, off = [], 0
    for parts in reversed(raw_per_rank):
        n = parts[0].numel()
        out.append(mean[off:off + n].view_as(parts[0]))
        off += n
    return list(reversed(out))


@pytest.mark.parametrize("idx", range(len(CONFIGS)),
                         ids=[f"{m}-{mode}-{'ef' if ef else 'noef'}" for m, _, mode, ef in CONFIGS])
def test_world8_invariants(world8, idx):
    method, kw, mode, ef = CONFIGS[idx]
    res = [r[idx] for r in world8]
    r0 = res[0]
    for r in res[1:]:                                    # bit-identical gradients on all ranks
        for a, b in zip(r0["got"], r["got"]):
            assert torch.equal(a, b)
    # the quantised reduce-scatter wire (QSGD at world 8): two grouped send/recv phases per
    # bucket and a bf16-rounded mean
    qrs = any(c == "send_recv" for c in r0["calls"])
    for r in res:                                        # bucket order, one exchange / bucket
        assert r["launched"] == list(range(r["nbuckets"]))
        assert len(r["calls"]) == r["nbuckets"] * (2 if qrs else 1), r["calls"]
    if mode == "layerwise":
        assert r0["nbuckets"] > 1                        # the bucketing is exercised
    if ef:
        world = len(res)
        for gi, g in enumerate(r0["got"]):
            sent = sum(r0["raw"][gi][k] - r0["ef"][gi][k] for k in range(world)) / world
            if qrs:
                sent = sent.to(torch.bfloat16).float()
            torch.testing.assert_close(g, sent, rtol=1e-5 if not qrs else 2 ** -7,
                                       atol=1e-6)
        assert any(float(e.abs().sum()) > 0 for e in r0["ef"][0]) or method == "none"
    elif method in ("none", "Topk", "Thresholdv", "AdaptiveThreshold"):
        exp = _oracle_plain(r0["raw"], method, kw, mode)
        for g, e in zip(r0["got"], exp):
            torch.testing.assert_close(g, e, rtol=1e-5, atol=1e-7)
    elif method == "Randomk":
        # index-free shared-seed masks: the support is common, values are the rank mean there
        mean = [sum(parts) / len(parts) for parts in r0["raw"]]
        for g, mu in zip(r0["got"], mean):
            nz = g != 0
            torch.testing.assert_close(g[nz], mu[nz], rtol=1e-5, atol=1e-7)
    if method != "none":
        assert r0["payload"] <= r0["dense"]
