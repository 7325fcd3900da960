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


class LoopbackRccl:
    """:class:`~.comm.NativeRccl` stand-in for a world of ``world`` ranks on one GPU."""

    def __init__(self, peers: PeerSim):
        self.sim = peers
        self.world = peers.world
        self.rank = peers.rank
        self.calls: List[tuple] = []
        self._frozen_sum = {}
        self._frozen_cat = {}

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
            return _Done()
        it = iter(parts)
        for r in range(self.world):
            if r == self.rank:
                if inp.data_ptr() != chunks[r].data_ptr():
                    chunks[r].copy_(inp.reshape(-1))
            else:
                chunks[r].copy_(next(it).reshape(-1))
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
            return _Done()
        acc = None
        it = iter(self.sim.payloads(bi))
        for r in range(self.world):
            src = t if r == self.rank else next(it)
            acc = src.clone() if acc is None else acc.add_(src)
        t.copy_(acc)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0):
        self.calls.append(("broadcast", -1))
        return _Done()          # every simulated replica starts from the same state

    def close(self) -> None:
        pass


def attach_loopback(engine, peer_grads: Sequence[torch.Tensor],
                    rank: int = 0, frozen: bool = False) -> LoopbackRccl:
    """Give ``engine`` (built with ``world_size=W``) a loopback communicator whose W-1 peers
    compress ``peer_grads`` (one arena-sized fp32 tensor per peer) every step (``frozen``: once,
    then their payloads are replayed — for timing)."""
    lb = LoopbackRccl(PeerSim(engine, peer_grads, rank, frozen))
    engine.use_communicator(lb)
    return lb

