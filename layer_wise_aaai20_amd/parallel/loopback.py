"""Loopback communicator: a simulated world of W ranks on ONE GPU.

RCCL refuses two ranks on one device (``profiles/r2_rccl_share_gpu_refused.log``), so the world > 1
default path — bucket collectives on the native RCCL communicator, inline inside a captured HIP
graph, decoded at world W — cannot run on a 1-GPU box. :class:`LoopbackRccl` has the
:class:`~.comm.NativeRccl` interface and produces exactly what W real ranks would deliver:

* the W-1 peer payloads come from the SAME codec classes built for the peers' ranks (their own
  Philox tags / error-feedback residuals) compressing stored peer gradients, on the caller's
  stream, so they are captured into the step graph with everything else;
* ``all_gather(out, inp)`` writes the rank-ordered concatenation RCCL would write
  (``recv = world x send``); ``all_reduce(t)`` adds the peers' vectors in rank order.

Used by ``tests/test_loopback_gpu.py`` to check the captured world-W step against eager and
against the CPU oracle (mean over ranks of what each rank sent), the multi-rank invariant that
the reference's DDP relies on (``IMAGENET/training/ddp.py:434-477``,
``sparsified_ddp.py:454-494``).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from ..compress.codecs import make_codec
from .comm import _Done


class PeerSim:
    """The W-1 simulated peers of one engine: per-peer codecs (built for the peer's rank), peer
    error-feedback residuals and a fixed stored gradient arena per peer."""

    def __init__(self, engine, peer_grads: Sequence[torch.Tensor], rank: int = 0,
                 frozen: bool = False):
        self.engine = engine
        # frozen (timing runs, bench.py --simulate-world): each bucket's peer payloads are
        # compressed once and replayed; a step then costs this rank what it costs a real rank —
        # its own compression, the received bytes landing in memory, the W-rank decode — without
        # the W-1 peers' compressions a real node runs on the other GPUs
        self.frozen = bool(frozen)
        self._frozen = {}
        self.world = engine.world
        self.rank = rank
        self.peers = [r for r in range(self.world) if r != rank]
        if len(peer_grads) != len(self.peers):
            raise ValueError(f"need {len(self.peers)} peer gradients, got {len(peer_grads)}")
        n = engine.arena.numel
        self.grads = [g.reshape(-1)[:n].to(engine.device, torch.float32).contiguous()
                      for g in peer_grads]
        self.scratch = [torch.empty_like(g) for g in self.grads]
        self.ef = [torch.zeros_like(g) if engine.ef is not None else None for g in self.grads]
        self.codecs = []
        for r in self.peers:
            cs = []
            for plan in engine.plans:
                c = make_codec(engine.method, plan, self.world, r, **engine.codec_kw)
                c.step_t = engine._dstep
                inner = getattr(c, "inner", None)
                if inner is not None:
                    inner.step_t = engine._dstep
                cs.append(c)
            self.codecs.append(cs)
        self._ptr = None

    def bucket_of(self, t: torch.Tensor) -> int:
        """Which bucket a collective belongs to, from its buffer address (the codecs' persistent
        send buffers, or the bucket's arena slice for the in-place dense wire)."""
        if self._ptr is None:
            eng = self.engine
            m = {}
            for bi, (b, c) in enumerate(zip(eng.buckets, eng.codecs)):
                m[eng.arena.grad[b.start:b.end].data_ptr()] = bi
                inner = getattr(c, "inner", c)
                for owner in (c, inner):
                    sb = getattr(owner, "send_buffer", None)
                    try:
                        m[sb(eng.device).data_ptr()] = bi
                    except (TypeError, AttributeError):   # no fixed send buffer (dense wires)
                        pass
            self._ptr = m
        return self._ptr[t.data_ptr()]

    def bucket_of_codec(self, codec) -> int:
        for bi, c in enumerate(self.engine.codecs):
            if c is codec:
                return bi
        raise KeyError("codec is not one of the engine's")

    def payloads(self, bi: int) -> List[torch.Tensor]:
        """Every peer's payload for bucket ``bi`` this step (stream-ordered, capturable)."""
        if self.frozen and bi in self._frozen:
            return self._frozen[bi]
        b = self.engine.buckets[bi]
        out = []
        for j, r in enumerate(self.peers):
            g = self.scratch[j][b.start:b.end]
            g.copy_(self.grads[j][b.start:b.end])       # compressors fold EF into g in place
            e = self.ef[j][b.start:b.end] if self.ef[j] is not None else None
            out.append(self.codecs[j][bi].compress(g, e, self.engine.step))
        if self.frozen:
            out = [t.clone() for t in out]
            self._frozen[bi] = out
        return out


class WireModel:
    """Transfer time of a collective on a W-GPU xGMI full mesh (MI355X: 7 links per GPU, one per
    peer), charged to the simulated step as a busy kernel (``csrc/compress.hip k_wire_wait``) of
    that duration on ``cus`` workgroups, enqueued right after the loopback's in-memory delivery on
    the collective's stream — so it lands where RCCL's kernel would: inline on the compute
    stream, or beside backward on the side branch, holding CU slots as RCCL's channel
    workgroups do.

    * all-gather of P bytes per rank: every peer's P arrives over its own link, P / link;
    * all-reduce of B bytes (direct reduce-scatter + all-gather over W-1 links): 2·B / (W·link);
    * broadcast of B bytes from the root: B / link;
    * grouped send/recv: the largest per-peer message / link;
    each plus ``latency_us``."""

    def __init__(self, link_gbs: float = 100.0, latency_us: float = 15.0, cus: int = 16):
        self.link_gbs, self.latency_us, self.cus = float(link_gbs), float(latency_us), int(cus)
        self.charged_us = 0.0          # host-side sum of the modelled transfer times (per call)

    def us(self, kind: str, nbytes: int, world: int) -> float:
        per = self.link_gbs * 1e3          # bytes per microsecond
        if kind == "all_reduce":
            t = 2.0 * nbytes / (world * per)
        else:                              # all_gather payload / broadcast / largest p2p message
            t = nbytes / per
        return t + self.latency_us

    def charge(self, device, kind: str, nbytes: int, world: int) -> None:
        from ..ops._ext import load
        us = self.us(kind, nbytes, world)
        self.charged_us += us
        load().wire_wait(torch.empty(0, device=device), us, self.cus)


class LoopbackRccl:
    """:class:`~.comm.NativeRccl` stand-in for a world of ``world`` ranks on one GPU.
    ``wire_model`` (a :class:`WireModel`): each collective also pays its modelled xGMI time."""

    def __init__(self, peers: PeerSim, wire_model: "WireModel" = None):
        self.sim = peers
        self.world = peers.world
        self.rank = peers.rank
        self.calls: List[tuple] = []
        self._frozen_sum = {}
        self._frozen_cat = {}
        self._qrs_step = {}
        self.wire_model = wire_model

    def _wire(self, t: torch.Tensor, kind: str, nbytes: int) -> None:
        if self.wire_model is not None and t.is_cuda:
            self.wire_model.charge(t.device, kind, nbytes, self.world)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        bi = self.sim.bucket_of(inp)
        self.calls.append(("all_gather", bi))
        parts = self.sim.payloads(bi)
        chunks = out.view(self.world, -1)
        if self.sim.frozen:
            # timing mode: the W-1 frozen peer payloads land with one copy (the peers' block of
            # the output is contiguous around this rank's own chunk), as one RCCL kernel would
            # write them — not W-1 copy launches
            cat = self._frozen_cat.get(bi)
            if cat is None:
                cat = torch.stack([p.reshape(-1) for p in parts])
                self._frozen_cat[bi] = cat
            r = self.rank
            if r > 0:
                chunks[:r].copy_(cat[:r])
            if r < self.world - 1:
                chunks[r + 1:].copy_(cat[r:])
            if inp.data_ptr() != chunks[r].data_ptr():       # (in place: already there)
                chunks[r].copy_(inp.reshape(-1))
            self._wire(out, "all_gather", inp.numel() * inp.element_size())
            return _Done()
        it = iter(parts)
        for r in range(self.world):
            if r == self.rank:
                if inp.data_ptr() != chunks[r].data_ptr():
                    chunks[r].copy_(inp.reshape(-1))
            else:
                chunks[r].copy_(next(it).reshape(-1))
        self._wire(out, "all_gather", inp.numel() * inp.element_size())
        return _Done()

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        bi = self.sim.bucket_of(t)
        self.calls.append(("all_reduce", bi))
        if op != "sum":
            raise NotImplementedError("loopback all_reduce: sum only")
        # rank-ordered sum, as a ring/tree would produce bit-identically on every rank only up to
        # fp32 reassociation: RCCL's order is not ours, so the oracle compares with a tolerance
        if self.sim.frozen:
            # timing mode: the peers' sum is formed once; a step then pays one pass over the
            # vector, about the local memory work of a ring all-reduce (its reduce-scatter reads
            # and adds (W-1)/W of the vector, its all-gather writes it), not W-1 full adds
            tot = self._frozen_sum.get(bi)
            if tot is None:
                tot = torch.stack([p.reshape(-1) for p in self.sim.payloads(bi)]).sum(0)
                self._frozen_sum[bi] = tot.view_as(t)
                tot = self._frozen_sum[bi]
            t.add_(tot)
            self._wire(t, "all_reduce", t.numel() * t.element_size())
            return _Done()
        acc = None
        it = iter(self.sim.payloads(bi))
        for r in range(self.world):
            src = t if r == self.rank else next(it)
            acc = src.clone() if acc is None else acc.add_(src)
        t.copy_(acc)
        self._wire(t, "all_reduce", t.numel() * t.element_size())
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0):
        self.calls.append(("broadcast", -1))
        self._wire(t, "broadcast", t.numel() * t.element_size())
        return _Done()          # every simulated replica starts from the same state

    def send_recv(self, sends, send_peers, recvs, recv_peers, key=None):
        """Grouped point-to-point as W real ranks would deliver it, for the quantised
        reduce-scatter wire (``codecs.QuantRSCodec``; ``key = (codec, phase)``):

        * phase 1 — from peer q, the records of this rank's shard in peer q's payload;
        * phase 2 — from peer q, peer q's shard of the mean: the same shard kernel run over every
          rank's records of shard q (this rank's own payload included), as peer q computes it.

        Frozen mode (timing): the peers' pieces and shard means are formed once and replayed."""
        if key is None:
            raise NotImplementedError("loopback send_recv: needs the codec key")
        codec, phase = key
        bi = self.sim.bucket_of_codec(codec)
        self.calls.append((f"send_recv{phase}", bi))
        me = self.rank
        if phase == 1:
            # the peers compress once per bucket and step: phase 2 reuses these payloads
            payloads = self._payloads_by_rank(bi, codec)
            self._qrs_step[bi] = payloads
            by_peer = {}
            for t, p in zip(recvs, recv_peers):
                by_peer.setdefault(int(p), []).append(t)
            for p, slots in by_peer.items():    # (frozen: the peers' payloads are replayed)
                for dst, x in zip(slots, codec.pieces(payloads[p], me)):
                    dst.copy_(x)
            self._charge_p2p(sends, send_peers)
            return _Done()
        for t, p in zip(recvs, recv_peers):
            p = int(p)
            if p == me:
                continue
            part = self._frozen_sum.get(("qrs2", bi, p)) if self.sim.frozen else None
            if part is None:
                payloads = self._qrs_step[bi]
                r1 = torch.empty(self.world * codec.wpr[p], dtype=torch.int32, device=t.device)
                rows = r1.view(self.world, -1)
                for q in range(self.world):
                    for dst, x in zip(codec.piece_slots(rows[q], p), codec.pieces(payloads[q], p)):
                        dst.copy_(x)
                img = torch.zeros(codec.n, dtype=torch.bfloat16, device=t.device)
                codec.reduce_shard(r1, p, img)
                part = img[codec.A[p]:codec.A[p + 1]].clone()
                if self.sim.frozen:
                    self._frozen_sum[("qrs2", bi, p)] = part
            t.copy_(part)
        self._charge_p2p(sends, send_peers)
        return _Done()

    def _charge_p2p(self, sends, send_peers) -> None:
        per = {}
        for t, p in zip(sends, send_peers):
            if int(p) != self.rank:
                per[int(p)] = per.get(int(p), 0) + t.numel() * t.element_size()
        if per and sends:
            self._wire(sends[0], "p2p", max(per.values()))

    def _payloads_by_rank(self, bi: int, codec) -> dict:
        peers = self.sim.payloads(bi)
        out = {r: peers[j] for j, r in enumerate(self.sim.peers)}
        out[self.rank] = codec._last_send
        return out

    def close(self) -> None:
        pass


def attach_loopback(engine, peer_grads: Sequence[torch.Tensor],
                    rank: int = 0, frozen: bool = False,
                    wire_model: "WireModel" = None) -> LoopbackRccl:
    """Give ``engine`` (built with ``world_size=W``) a loopback communicator whose W-1 peers
    compress ``peer_grads`` (one arena-sized fp32 tensor per peer) every step (``frozen``: once,
    then their payloads are replayed — for timing; ``wire_model``: collectives also pay their
    modelled xGMI time)."""
    lb = LoopbackRccl(PeerSim(engine, peer_grads, rank, frozen), wire_model)
    engine.use_communicator(lb)
    return lb

