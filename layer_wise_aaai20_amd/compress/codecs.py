"""Wire codecs: turn one bucket of gradients into a collective payload and back.

Every codec reproduces the reference's *result* — the mean over ranks of each rank's compressed
dense vector (``CIFAR10/core.py:217-225``) — while changing what travels on the wire (SURVEY.md
§2.4 "MI355X-native equivalent"):

=================  ==============  ===========================================================
codec              collective      payload per rank
=================  ==============  ===========================================================
DenseCodec         all_reduce      the fp32 bucket itself (method ``none``; DP-3 equivalent)
TopkCodec          all_gather      (int32 index, fp32 value) pairs, cap_s = m_s + tie slack
ThresholdCodec     all_gather      pairs, capacity agreed by an all-reduce(MAX) of counts
RandkCodec         all_reduce      index-free values: shared-seed Philox masks (DP-4 equivalent)
TernGradCodec      all_gather      one fp32 scale per layer + 2-bit codes
QSGDCodec          all_gather      one fp32 norm per layer + int8 / 8+1 / int16-bit levels
DenseWrap(inner)   all_reduce      reference wire format: dense compressed vector (parity mode)
QuantRSCodec(q)    quant_rs        quantised reduce-scatter: all-to-all of each rank's codes for
                                   shard r to rank r, shard dequant-sum, bf16 all-gather
=================  ==============  ===========================================================

GPU tensors run the HIP kernels (``csrc/compress.hip``); CPU tensors run the torch code below,
which mirrors the kernels (same Philox streams, same packing, same rank-ordered sums) so the gloo
tests exercise the same semantics.

Error feedback (``error_feedback=True``) generalises the reference's Random-K-only residual
(``IMAGENET/training/sparsified_ddp.py:409-413``) to every method: ``g' = g + e`` before
compression, ``e <- g' - C(g')`` after it, where ``C(g')`` is this rank's decoded contribution.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

from . import reference as ref
from .plan import GROUP, SMALL_MAX, SegPlan, hdr_words
from ..ops._ext import ops_for
from ..utils import philox

SENT = 0x7FFFFFFF
KM_TOPK, KM_RANDK, KM_THRESH = 0, 1, 2
OUT_PAIRS, OUT_VALIDX = 0, 1
Q_TERN, Q_QS8, Q_QS9, Q_QS16 = 0, 1, 2, 3


def _ws_tensor(nbytes: int, device) -> torch.Tensor:
    # zeroed: the fused select chain expects zero radix histograms on its first call and leaves
    # them zeroed for the next (csrc/compress.hip k_write FW)
    return torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def tie_slack(m: int) -> int:
    """Extra payload slots per layer for Top-K values tied at the threshold (the reference keeps
    every element >= the k-th largest, so a tie can make it send more than k): 1/64 of k, and at
    least 16 — small layers (a 1000-way classifier bias keeps k = 1) can tie many ways."""
    return max(16, -(-m // 64))


class Codec:
    collective = "all_reduce"
    name = "codec"
    # True when compress/decompress issue no host synchronisation and depend on nothing that
    # changes from step to step on the host (e.g. a Philox step counter passed as a kernel
    # argument): the whole training step can then be captured once as a HIP graph and replayed
    graph_safe = False
    # device step counter (GradSyncEngine._dstep) the Philox-keyed kernels read instead of the
    # host `step` argument, so a replayed HIP graph draws fresh random keys every step
    step_t = None
    uses_step = False           # reads the device step counter step_t (Philox-keyed codecs)
    # device int32 counter of elements the reference rule selects that the payload could not
    # carry (Top-K ties beyond the slack, threshold hits beyond a fixed sparse capacity); they
    # stay in the error-feedback residual (GradSyncEngine.read_overflow)
    overflow = None
    # momentum correction (GradSyncEngine): the bucket's velocity while compress() runs; a codec
    # with mc_fused zeroes it at the coordinates it selected (segments not sent whole only)
    mc_mom = None
    mc_fused = False
    # (p, seg_wd, mc, wmul): the velocity update itself runs in the first select pass (Top-K,
    # layer-wise; GradSyncEngine._launch), with mc_mom as u
    mc_fuse = None
    # entire-model staging (GradSyncEngine): codecs with `stage` run their first pass per arena
    # slice during backward; `_staged` tells compress() that pass is done for this step
    _staged = False
    # in-place all-gather (GradSyncEngine sets it with a stream-ordered native communicator): the
    # payload is written straight into this rank's row of a persistent [world, payload] buffer,
    # which is then the collective's output — RCCL's in-place form, no local copy of our own row
    inplace_gather = False

    def can_stage(self) -> bool:
        return False

    def _inplace_slot(self, device, n: int, dtype, zero: bool = False) -> torch.Tensor:
        """This rank's row of the persistent in-place all-gather buffer ([world * n])."""
        if not hasattr(self, "_gather"):
            self._gather = {}
        k = str(device)
        buf = self._gather.get(k)
        if buf is None or buf.numel() != self.world * n:
            buf = (torch.zeros if zero else torch.empty)(self.world * n, dtype=dtype,
                                                         device=device)
            self._gather[k] = buf
        return buf[self.rank * n:(self.rank + 1) * n]

    def __init__(self, plan: SegPlan, world: int, rank: int, seed: int = 0,
                 error_feedback: bool = False):
        self.plan = plan
        self.world = int(world)
        self.rank = int(rank)
        self.seed = int(seed) & ((1 << 63) - 1)
        self.error_feedback = error_feedback
        self.last_payload_bytes = 0

    def compress(self, grad: torch.Tensor, ef: Optional[torch.Tensor], step: int) -> torch.Tensor:
        raise NotImplementedError

    def recv_buffer(self, send: torch.Tensor) -> Optional[torch.Tensor]:
        if self.collective == "all_gather":
            buf = getattr(self, "_gather", {}).get(str(send.device))
            if buf is not None and buf.dtype == send.dtype and \
                    send.data_ptr() == buf.data_ptr() + self.rank * send.numel() * \
                    send.element_size():
                return buf                       # (in place: send is our row of it)
            return torch.empty(send.numel() * self.world, dtype=send.dtype, device=send.device)
        return None

    def decompress(self, send: torch.Tensor, recv: Optional[torch.Tensor], grad: torch.Tensor,
                   world: Optional[int] = None) -> None:
        raise NotImplementedError

    # -- helpers
    def _segs(self, t: torch.Tensor):
        for s in range(self.plan.S):
            o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
            yield s, t[o:o + n]


# ================================================================================= dense
class DenseCodec(Codec):
    """No compression: bucketed in-place all-reduce, then ``/ world_size`` (core.py:318-319)."""
    name = "dense"
    graph_safe = True

    def compress(self, grad, ef, step):
        self.last_payload_bytes = grad.numel() * grad.element_size()
        return grad

    def decompress(self, send, recv, grad, world=None):
        w = int(world or self.world)
        if w != 1:                              # (world 1: no kernel for a division by 1)
            grad.div_(float(w))


# ================================================================================= Top-K
class TopkCodec(Codec):
    """Exact reference Top-K selection (``kthvalue`` threshold, ``>=`` keeps ties) → sparse pairs."""
    collective = "all_gather"
    name = "topk"
    km = KM_TOPK

    # exact Top-K ignores the step; Random-K reads it from the device counter (step_t)
    graph_safe = True
    mc_fused = True

    def __init__(self, plan, world, rank, K: float, seed=0, error_feedback=False,
                 dense_below: int = 0):
        super().__init__(plan, world, rank, seed, error_feedback)
        self.K = float(K)
        self.keep = np.asarray([ref.topk_keep_count(int(n), self.K) for n in plan.sizes],
                               dtype=np.int64)
        self.dense_below = int(dense_below or 0)
        if self.dense_below > 0:     # opt-in deviation: small tensors travel whole (see below)
            self.keep = np.where(np.asarray(plan.sizes) <= self.dense_below,
                                 np.asarray(plan.sizes, dtype=np.int64), self.keep)
        self.cap = self.keep + np.asarray([tie_slack(int(m)) for m in self.keep], dtype=np.int64)
        self.cap = np.minimum(self.cap, plan.sizes)
        self.cap_off = np.concatenate([[0], np.cumsum(self.cap)]).astype(np.int64)
        self.cap_total = int(self.cap_off[-1])
        self._ws = {}
        self._send = {}

    def _dev_tables(self, device):
        t = self.plan.select_tables(device)
        kk = f"{self.K}d{getattr(self, 'dense_below', 0)}"
        t["keep"] = self.plan.dev(device, f"keep{kk}", lambda: torch.from_numpy(
            self.keep.astype(np.int32)))
        t["cap_off"] = self.plan.dev(device, f"capoff{kk}{self.km}", lambda: torch.from_numpy(
            self.cap_off))
        return t

    def _workspace(self, device, lib):
        k = str(device)
        if k not in self._ws:
            small, large = self.plan.split(SMALL_MAX)
            nb = lib.workspace_bytes(len(small), len(large), self.plan.n_tasks(SMALL_MAX))
            self._ws[k] = _ws_tensor(nb, device)
        return self._ws[k]

    def send_buffer(self, device):
        if self.inplace_gather:
            return self._inplace_slot(device, 2 * max(self.cap_total, 1), torch.int32)
        k = str(device)
        if k not in self._send:
            self._send[k] = torch.empty(2 * max(self.cap_total, 1), dtype=torch.int32,
                                        device=device)
        return self._send[k]

    def can_stage(self) -> bool:
        """One large segment (entire-model mode): its radix pass 0 can run per task range."""
        small, large = self.plan.split(SMALL_MAX)
        return self.plan.S == 1 and len(large) == 1

    def stage(self, grad, ef, step, t_lo: int, t_hi: int, first: bool) -> None:
        """Radix pass 0 (+ the error-feedback fold for Top-K) over tasks [t_lo, t_hi) of the one
        segment; ``first`` zeroes the histograms (csrc/compress.hip select_stage)."""
        lib = ops_for(grad)
        if lib is None:
            return                      # (the CPU mirror does everything in compress)
        t = self._dev_tables(grad.device)
        lib.select_stage(grad, ef, t["seg_off"], t["seg_n"], t["keep"], t["cap_off"],
                         t["small_segs"], t["large_segs"], t["tasks"], t["task_lo"],
                         self._workspace(grad.device, lib), self.km, int(t_lo), int(t_hi),
                         bool(first), self.plan.gid_base, int(step) & 0xFFFFFFFF, self.seed,
                         self.step_t)

    def compress(self, grad, ef, step):
        lib = ops_for(grad)
        out = self.send_buffer(grad.device)
        self.last_payload_bytes = out.numel() * 4
        if lib is not None:
            t = self._dev_tables(grad.device)
            lib.select_compress(grad, ef, t["seg_off"], t["seg_n"], t["keep"], t["cap_off"],
                                t["small_segs"], t["large_segs"], t["tasks"], t["task_lo"],
                                self._workspace(grad.device, lib), self.km, OUT_PAIRS, out, None,
                                None, self.plan.gid_base, int(step) & 0xFFFFFFFF, self.seed,
                                self.step_t, self.overflow, self.mc_mom, self._staged,
                                self.plan.max_large_tasks(),
                                *(self.mc_fuse if self.mc_fuse is not None else ()))
            return out
        self._compress_cpu(grad, ef, step, out)
        return out

    def _select_cpu(self, s, x, step):
        """Return (indices selected in index order) with the kernel's exact semantics."""
        n, m, cap = x.numel(), int(self.keep[s]), int(self.cap[s])
        if self.km == KM_TOPK:
            keys = x.abs()
            t = keys.float().kthvalue(n - m + 1).values if m < n else keys.min()
            gt = keys > t
            eq = keys == t
            quota = 0 if float(t) == 0.0 else min(int(eq.sum()), cap - int(gt.sum()))
        else:
            kn = philox.randk_keys(n, self.plan.gid_base + s, int(step) & 0xFFFFFFFF, self.seed)
            keys = torch.from_numpy(kn.astype(np.int64))
            t = keys.kthvalue(n - m + 1).values if m < n else keys.min()
            gt = keys > t
            eq = keys == t
            quota = m - int(gt.sum())
        sel = gt | (eq & (torch.cumsum(eq.to(torch.int64), 0) <= quota))
        return torch.nonzero(sel, as_tuple=False).flatten()

    def _compress_cpu(self, grad, ef, step, out):
        pairs = out.view(-1, 2)
        pairs[:, 0] = SENT
        pairs[:, 1] = 0
        for s, x in self._segs(grad):
            o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
            if ef is not None:
                x.add_(ef[o:o + n])
            idx = self._select_cpu(s, x, step)
            c0 = int(self.cap_off[s])
            k = idx.numel()
            pairs[c0:c0 + k, 0] = idx.to(torch.int32)
            pairs[c0:c0 + k, 1] = x[idx].float().view(torch.int32)
            if ef is not None:
                e = ef[o:o + n]
                e.copy_(x)
                e[idx] = 0
            if self.mc_mom is not None and k < n:    # (the kernels' momentum factor masking)
                self.mc_mom[o:o + n][idx] = 0

    def decompress(self, send, recv, grad, world=None):
        world = world or self.world
        gathered = send if recv is None else recv
        lib = ops_for(grad)
        if lib is not None:
            t = self.plan.common(grad.device)
            t["cap_off"] = self._dev_tables(grad.device)["cap_off"]
            lib.unpack_pairs(gathered, world, grad, t["seg_off"], t["seg_n"], t["cap_off"],
                             self.plan.utasks(grad.device))
            return
        self.unpack_pairs_cpu(gathered, world, grad, self.cap_off)

    def decompress_sgd(self, send, recv, sgd: dict, world=None):
        """Decode fused with the SGD step of the bucket's parameters (GPU only;
        ``parallel/engine.py set_fused_sgd``): ``sgd`` holds the bucket's slices of the
        parameter / momentum / bf16-mirror arenas, its segments' weight decay and the optimizer's
        hyper-parameters."""
        world = world or self.world
        gathered = send if recv is None else recv
        p = sgd["p"]
        lib = ops_for(p)
        if lib is None:
            raise RuntimeError("decompress_sgd: GPU only")
        t = self.plan.common(p.device)
        lib.unpack_pairs_sgd(gathered, world, t["seg_off"], self._dev_tables(p.device)["cap_off"],
                             sgd["tasks"], p, sgd["buf"], sgd["seg_wd"], sgd["lr"], sgd["momentum"],
                             sgd["dampening"], int(sgd["nesterov"]), int(sgd["first"]),
                             sgd["grad_scale"], sgd["hyper"], sgd["pb"])

    def unpack_pairs_cpu(self, gathered, world, grad, cap_off):
        cap_total = gathered.numel() // 2 // world
        P = gathered.view(world, cap_total, 2)
        for s, x in self._segs(grad):
            acc = torch.zeros_like(x, dtype=torch.float32)
            c0, c1 = int(cap_off[s]), int(cap_off[s + 1])
            for r in range(world):
                seg = P[r, c0:c1]
                keep = seg[:, 0] != SENT
                idx = seg[keep, 0].long()
                val = seg[keep, 1].view(torch.float32)
                acc.index_add_(0, idx, val)
            x.copy_(acc / float(world))


class RandkSparseCodec(TopkCodec):
    """Random-K with explicit indices (masks need not be rank-coherent)."""
    name = "randk-sparse"
    km = KM_RANDK
    uses_step = True
    # Philox masks keyed by the device step counter (step_t): replays draw fresh masks. (Its
    # round-2 replay divergence was the runtime memset node that reset the radix histogram,
    # profiles/r3_graph_divergence_root_cause.md; graph == eager bit for bit since.)
    graph_safe = True

    def __init__(self, plan, world, rank, K, seed=0, error_feedback=False,
                 dense_below: int = 0):
        Codec.__init__(self, plan, world, rank, seed, error_feedback)
        self.K = float(K)
        self.keep = np.asarray([ref.randomk_keep_count(int(n), self.K) for n in plan.sizes],
                               dtype=np.int64)
        self.keep = np.maximum(self.keep, 1)
        self.dense_below = int(dense_below or 0)
        if self.dense_below > 0:
            self.keep = np.where(np.asarray(plan.sizes) <= self.dense_below,
                                 np.asarray(plan.sizes, dtype=np.int64), self.keep)
        self.cap = self.keep.copy()
        self.cap_off = np.concatenate([[0], np.cumsum(self.cap)]).astype(np.int64)
        self.cap_total = int(self.cap_off[-1])
        self._ws = {}
        self._send = {}


# ================================================================================= Random-K
class RandkCodec(RandkSparseCodec):
    """Index-free Random-K: identical Philox masks on every rank (shared seed), so only the
    ``k_s = ceil(n_s K)`` selected VALUES are all-reduced — the wire format of the reference's
    ``RandomKSparsifiedDDP`` (``sparsified_ddp.py:164, 410-412``) without ``randperm``."""
    collective = "all_reduce"
    name = "randk"

    def __init__(self, plan, world, rank, K, seed=0, error_feedback=False, dense_below=0):
        super().__init__(plan, world, rank, K, seed, error_feedback, dense_below)
        self._idx = {}
        self._slot_seg = {}

    def send_buffer(self, device):
        k = str(device)
        if k not in self._send:
            self._send[k] = torch.empty(max(self.cap_total, 1), dtype=torch.float32, device=device)
            self._idx[k] = torch.empty(max(self.cap_total, 1), dtype=torch.int32, device=device)
        return self._send[k]

    def compress(self, grad, ef, step):
        lib = ops_for(grad)
        vals = self.send_buffer(grad.device)
        idx = self._idx[str(grad.device)]
        self.last_payload_bytes = vals.numel() * 4
        if lib is not None:
            t = self._dev_tables(grad.device)
            lib.select_compress(grad, ef, t["seg_off"], t["seg_n"], t["keep"], t["cap_off"],
                                t["small_segs"], t["large_segs"], t["tasks"], t["task_lo"],
                                self._workspace(grad.device, lib), KM_RANDK, OUT_VALIDX, None,
                                vals, idx, self.plan.gid_base, int(step) & 0xFFFFFFFF, self.seed,
                                self.step_t, None, self.mc_mom, self._staged,
                                self.plan.max_large_tasks())
            return vals
        for s, x in self._segs(grad):
            o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
            xe = x + ef[o:o + n] if ef is not None else x
            sel = self._select_cpu(s, xe, step)
            c0 = int(self.cap_off[s])
            vals[c0:c0 + sel.numel()] = xe[sel]
            idx[c0:c0 + sel.numel()] = sel.to(torch.int32)
            if ef is not None:
                e = ef[o:o + n]
                e.copy_(xe)
                e[sel] = 0
            if self.mc_mom is not None and sel.numel() < n:
                self.mc_mom[o:o + n][sel] = 0
        return vals

    def decompress(self, send, recv, grad, world=None):
        world = world or self.world
        lib = ops_for(grad)
        idx = self._idx[str(grad.device)]
        grad.zero_()
        if lib is not None:
            slot_seg = self.plan.dev(grad.device, f"slotseg{self.K}d{self.dense_below}",
                                     lambda: torch.from_numpy(
                np.repeat(np.arange(self.plan.S, dtype=np.int32), self.cap)))
            lib.unpack_validx(send, idx, slot_seg, world, grad, self.plan.common(grad.device)
                              ["seg_off"])
            return
        for s, x in self._segs(grad):
            c0, c1 = int(self.cap_off[s]), int(self.cap_off[s + 1])
            x[idx[c0:c1].long()] = send[c0:c1] / float(world)


# ================================================================================= thresholds
class ThresholdCodec(TopkCodec):
    """``Thresholdv`` (|g| >= V) and ``AdaptiveThreshold`` (|2g| >= max|g|) on a sparse wire.

    The number of hits is data-dependent, so the payload capacity is either:

    * **fixed** (``max_density``, opt-in ``wire="sparse-capped"``): each segment carries at most
      ``max(16, ceil(density · n))`` pairs. It is sync-free and graph-capturable. Hits beyond the
      capacity — the first in index order travel, strictly-above-threshold hits first — stay in
      the error-feedback residual and are counted on the device (``GradSyncEngine.read_overflow``).
    * **agreed per step** (``max_density=None``, ``wire="sparse"`` / ``"sparse-exact"``): the ranks take an
      all-reduce(MAX) of the counts. This is exact for any density, but the capacity is read on
      the host in the middle of backward, so that step stays eager.
    """
    name = "threshold"
    km = KM_THRESH
    mc_fused = False               # (the engine masks the velocity where the residual is 0)

    def can_stage(self) -> bool:
        return False

    def __init__(self, plan, world, rank, V=None, adaptive=False, seed=0, error_feedback=False,
                 count_exchange=None, max_density=None):
        Codec.__init__(self, plan, world, rank, seed, error_feedback)
        self.V = float(V or 0.0)
        self.adaptive = bool(adaptive)
        self.count_exchange = count_exchange   # callable(int tensor) -> int tensor (MAX over ranks)
        self._ws = {}
        self._send = {}
        self.cap_off = None
        self.max_density = None if max_density is None else float(max_density)
        if self.max_density is not None:
            sizes = np.asarray(plan.sizes, dtype=np.int64)
            cap = np.minimum(sizes, np.maximum(16, np.ceil(sizes * self.max_density))).astype(
                np.int64)
            self.cap = cap
            self.cap_off = np.concatenate([[0], np.cumsum(cap)]).astype(np.int64)
            self.cap_total = int(self.cap_off[-1])

    @property
    def graph_safe(self) -> bool:
        return self.max_density is not None

    def _counts(self, grad, ef, lib, dev):
        """Threshold state + per-segment hit counts (device), or the CPU selection."""
        if lib is not None:
            t = self.plan.all_large_tables(dev)
            k = str(dev)
            if k not in self._ws:
                nb = lib.workspace_bytes(0, self.plan.S, int(t["tasks"].shape[0]))
                self._ws[k] = _ws_tensor(nb, dev)
            counts = torch.empty(self.plan.S, dtype=torch.int32, device=dev)
            lib.thresh_count(grad, ef, t["seg_off"], t["seg_n"], t["segs"], t["tasks"],
                             t["task_lo"], self._ws[k], self.V, int(self.adaptive), counts)
            return counts
        counts = torch.empty(self.plan.S, dtype=torch.int32)
        self._sel = []
        for s, x in self._segs(grad):
            if ef is not None:
                o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
                x.add_(ef[o:o + n])
            a = x.abs()
            thr = float(a.max()) * 0.5 if self.adaptive and x.numel() else self.V
            gt = (a > thr) & (x != 0)
            eq = (a == thr) & (x != 0) if thr != 0.0 else torch.zeros_like(gt)
            gi = torch.nonzero(gt, as_tuple=False).flatten()
            ei = torch.nonzero(eq, as_tuple=False).flatten()
            if self.max_density is not None:          # the kernels' capacity rule (k_set_caps)
                cap = int(self.cap[s])
                gi = gi[:cap]
                ei = ei[:max(0, cap - gi.numel())]
            idx = torch.sort(torch.cat([gi, ei])).values
            self._sel.append(idx)
            counts[s] = idx.numel()
        return counts

    def compress(self, grad, ef, step):
        lib = ops_for(grad)
        dev = grad.device
        counts = self._counts(grad, ef, lib, dev)
        if self.max_density is not None:
            out = self.send_buffer(dev)
            if lib is not None:
                self._cap_off_dev = self.plan.dev(dev, f"thrcap{self.max_density}",
                                                  lambda: torch.from_numpy(self.cap_off))
        else:
            caps = counts.to(torch.int64)
            if self.count_exchange is not None and self.world > 1:
                caps = self.count_exchange(caps)
            caps_h = caps.cpu().numpy().astype(np.int64)
            self.cap_off = np.concatenate([[0], np.cumsum(caps_h)]).astype(np.int64)
            cap_total = int(self.cap_off[-1])
            out = torch.empty(2 * max(cap_total, 1), dtype=torch.int32, device=dev)
            if lib is not None:
                self._cap_off_dev = torch.from_numpy(self.cap_off).to(dev)
        self.last_payload_bytes = out.numel() * 4
        if lib is not None:
            t = self.plan.all_large_tables(dev)
            lib.thresh_write(grad, ef, t["seg_off"], t["seg_n"], self._cap_off_dev, t["segs"],
                             t["tasks"], t["task_lo"], self._ws[str(dev)], out, self.overflow)
            return out
        pairs = out.view(-1, 2)
        pairs[:, 0] = SENT
        pairs[:, 1] = 0
        for s, x in self._segs(grad):
            idx = self._sel[s]
            c0 = int(self.cap_off[s])
            pairs[c0:c0 + idx.numel(), 0] = idx.to(torch.int32)
            pairs[c0:c0 + idx.numel(), 1] = x[idx].float().view(torch.int32)
            if ef is not None:
                o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
                e = ef[o:o + n]
                e.copy_(x)
                e[idx] = 0
        return out

    def decompress(self, send, recv, grad, world=None):
        world = world or self.world
        gathered = send if recv is None else recv
        lib = ops_for(grad)
        if lib is not None:
            t = self.plan.common(grad.device)
            lib.unpack_pairs(gathered, world, grad, t["seg_off"], t["seg_n"], self._cap_off_dev,
                             self.plan.utasks(grad.device))
            return
        self.unpack_pairs_cpu(gathered, world, grad, self.cap_off)

    def compress_dense(self, grad, ef):
        """In place: ``grad`` becomes the dense compressed vector (EF folded in, residual to
        ``ef``) — the reference wire's input, with no counts and no host round trip."""
        lib = ops_for(grad)
        if lib is not None:
            t = self.plan.all_large_tables(grad.device)
            k = str(grad.device)
            if k not in self._ws:
                nb = lib.workspace_bytes(0, self.plan.S, int(t["tasks"].shape[0]))
                self._ws[k] = _ws_tensor(nb, grad.device)
            lib.thresh_dense(grad, ef, t["seg_off"], t["seg_n"], t["segs"], t["tasks"],
                             t["task_lo"], self._ws[k], self.V, int(self.adaptive))
            return
        for s, x in self._segs(grad):
            o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
            if ef is not None:
                x.add_(ef[o:o + n])
            a = x.abs()
            if self.adaptive:
                keep = (x * 2).abs() >= a.max() if x.numel() else a > 0
            else:
                keep = a >= self.V
            keep &= x != 0
            if ef is not None:
                e = ef[o:o + n]
                e.copy_(x)
                e[keep] = 0
            x[~keep] = 0


# ================================================================================= quantisers
class _QuantCodec(Codec):
    collective = "all_gather"
    graph_safe = True           # stochastic rounding keyed by the device step counter (step_t)
    uses_step = True
    q = Q_TERN
    tag = philox.TAG_TERNGRAD
    qstates = 1

    def __init__(self, plan, world, rank, seed=0, error_feedback=False):
        super().__init__(plan, world, rank, seed, error_feedback)
        self.G = plan.groups()
        self.rec_off = plan.rec_off()
        self.Gtot = int(self.rec_off[-1])
        R = {Q_TERN: 2, Q_QS8: 8, Q_QS9: 9, Q_QS16: 16}[self.q]
        self.hdr = hdr_words(plan.S)
        self.words = (self.hdr + self.Gtot * R + 3) // 4 * 4
        self._ws = {}
        self._send = {}

    def send_buffer(self, device):
        if self.inplace_gather:
            return self._inplace_slot(device, self.words, torch.int32, zero=True)
        k = str(device)
        if k not in self._send:
            self._send[k] = torch.zeros(self.words, dtype=torch.int32, device=device)
        return self._send[k]

    def _qws(self, grad, lib, t):
        k = str(grad.device)
        if k not in self._ws:
            nb = lib.workspace_bytes(0, self.plan.S, int(t["tasks"].shape[0]))
            self._ws[k] = _ws_tensor(nb, grad.device)
        return self._ws[k]

    def can_stage(self) -> bool:
        return self.plan.S == 1

    def stage(self, grad, ef, step, t_lo: int, t_hi: int, first: bool) -> None:
        """The per-task (abs-max, sum of squares) partials with the error-feedback fold over
        tasks [t_lo, t_hi) of the one segment (csrc/compress.hip quant_stage)."""
        lib = ops_for(grad)
        if lib is None:
            return
        t = self.plan.all_large_tables(grad.device)
        lib.quant_stage(grad, ef, t["seg_off"], t["seg_n"], t["segs"], t["tasks"], t["task_lo"],
                        t["rec_off"], self._qws(grad, lib, t), self.qstates, int(t_lo), int(t_hi))

    def compress(self, grad, ef, step):
        lib = ops_for(grad)
        out = self.send_buffer(grad.device)
        self.last_payload_bytes = out.numel() * 4
        tag = self.tag | (self.rank & 0xFFFFFF)
        if lib is not None:
            t = self.plan.all_large_tables(grad.device)
            lib.quantize(grad, ef, t["seg_off"], t["seg_n"], t["segs"], t["tasks"], t["task_lo"],
                         t["rec_off"], self._qws(grad, lib, t), out, self.q, self.qstates,
                         self.plan.gid_base, int(step) & 0xFFFFFFFF, tag, self.seed, self.step_t,
                         self._staged)
            return out
        self._quant_cpu(grad, ef, step, out, tag)
        return out

    # ---- CPU mirror of k_partial/k_finalize/k_quant
    def _scale(self, x: torch.Tensor) -> float:
        raise NotImplementedError

    def _levels(self, x, sc, u):
        raise NotImplementedError

    def _quant_cpu(self, grad, ef, step, out, tag):
        words = out.numpy().view(np.uint32)
        hdr = words[:self.hdr]
        rec = words[self.hdr:]
        for s, x in self._segs(grad):
            o, n = int(self.plan.offsets[s]), int(self.plan.sizes[s])
            if ef is not None:
                x.add_(ef[o:o + n])
            sc = self._scale(x)
            hdr[s] = np.float32(sc).view(np.uint32)
            G = int(self.G[s])
            xv = np.zeros(G * GROUP, dtype=np.float32)
            xv[:n] = x.detach().float().numpy()
            u = philox.uniforms(G * GROUP, self.plan.gid_base + s, int(step) & 0xFFFFFFFF, tag,
                                self.seed)
            lv, dq = self._levels(xv, np.float32(sc), u)
            self._pack(rec, int(self.rec_off[s]), G, lv)
            if ef is not None:
                ef[o:o + n].copy_(torch.from_numpy(xv[:n] - dq[:n]))

    def _pack(self, rec, r0, G, lv):
        raise NotImplementedError

    def _unpack(self, rec, r0, G):
        raise NotImplementedError

    def decompress(self, send, recv, grad, world=None):
        world = world or self.world
        gathered = send if recv is None else recv
        lib = ops_for(grad)
        if lib is not None:
            t = self.plan.all_large_tables(grad.device)
            lib.dequantize(gathered, world, grad, t["seg_off"], t["seg_n"], t["segs"], t["tasks"],
                           t["task_lo"], t["rec_off"], self.q, self.qstates)
            return
        W = gathered.numpy().view(np.uint32).reshape(world, -1)
        for s, x in self._segs(grad):
            n = x.numel()
            G = int(self.G[s])
            acc = np.zeros(G * GROUP, dtype=np.float32)
            for r in range(world):
                sc = W[r, s].view(np.float32)
                lv = self._unpack(W[r, self.hdr:], int(self.rec_off[s]), G)
                acc += self._deq(lv, np.float32(sc))
            x.copy_(torch.from_numpy(acc[:n] / np.float32(world)))


class TernGradCodec(_QuantCodec):
    """TernGrad (core.py:200-206): s = max|g|, b ~ Bernoulli(|g|/s), out = sign(g)·s·b."""
    name = "terngrad"
    q = Q_TERN
    tag = philox.TAG_TERNGRAD

    def _scale(self, x):
        return float(x.abs().max()) if x.numel() else 0.0

    def _levels(self, xv, sc, u):
        if sc > 0:
            prob = np.abs(xv) / sc
            b = u < prob
        else:
            b = np.zeros_like(xv, dtype=bool)
        code = np.where(b & (xv > 0), 1, np.where(b & (xv < 0), 2, 0)).astype(np.uint32)
        dq = np.where(code == 1, sc, np.where(code == 2, -sc, np.float32(0))).astype(np.float32)
        return code, dq

    def _deq(self, code, sc):
        return np.where(code == 1, sc, np.where(code == 2, -sc, np.float32(0))).astype(np.float32)

    def _pack(self, rec, r0, G, code):
        c = code.reshape(G, 2, 16).astype(np.uint32)
        sh = (2 * np.arange(16, dtype=np.uint32))[None, None, :]
        w = np.bitwise_or.reduce(c << sh, axis=2)
        rec[r0 * 2:(r0 + G) * 2] = w.reshape(-1)

    def _unpack(self, rec, r0, G):
        w = rec[r0 * 2:(r0 + G) * 2].reshape(G, 2, 1)
        sh = (2 * np.arange(16, dtype=np.uint32))[None, None, :]
        return ((w >> sh) & np.uint32(3)).reshape(-1)


class QSGDCodec(_QuantCodec):
    """Random dithering / QSGD (core.py:207-213) with ``qstates`` levels:
    l = floor(|g|/‖g‖·s + u), out = sign(g)·‖g‖·l/s. Packing: s<=127 → int8, s<=255 → uint8 level
    + sign bit (9 bits/elem), else int16."""
    name = "qsgd"
    tag = philox.TAG_QSGD

    def __init__(self, plan, world, rank, qstates=255, seed=0, error_feedback=False):
        self.qstates = int(qstates)
        if self.qstates < 1 or self.qstates > 32767:
            raise ValueError("qstates must be in [1, 32767]")
        self.q = Q_QS8 if self.qstates <= 127 else (Q_QS9 if self.qstates <= 255 else Q_QS16)
        super().__init__(plan, world, rank, seed, error_feedback)

    def _scale(self, x):
        return float(torch.norm(x.float())) if x.numel() else 0.0

    def _levels(self, xv, sc, u):
        qs = np.float32(self.qstates)
        if sc > 0:
            lvl = np.floor(np.abs(xv) / sc * qs + u).astype(np.int64)
            lvl = np.minimum(lvl, self.qstates)
        else:
            lvl = np.zeros(xv.shape, dtype=np.int64)
        sg = np.sign(xv).astype(np.float32)
        dq = (sg * sc * (lvl.astype(np.float32) / qs)).astype(np.float32)
        signed = np.where(xv < 0, -lvl, lvl)
        return signed, dq

    def _deq(self, signed, sc):
        qs = np.float32(self.qstates)
        mag = np.abs(signed).astype(np.float32)
        return (np.sign(signed).astype(np.float32) * sc * (mag / qs)).astype(np.float32)

    def _pack(self, rec, r0, G, lv):
        if self.q == Q_QS8:
            b = (lv.astype(np.int64) & 0xFF).astype(np.uint8)
            rec[r0 * 8:(r0 + G) * 8] = b.view(np.uint32)
        elif self.q == Q_QS9:
            mag = np.abs(lv).astype(np.uint8)
            rec[r0 * 8:(r0 + G) * 8] = mag.view(np.uint32)
            sb = (lv < 0).reshape(G, 32).astype(np.uint32)
            rec[self.Gtot * 8 + r0:self.Gtot * 8 + r0 + G] = np.bitwise_or.reduce(
                sb << np.arange(32, dtype=np.uint32)[None, :], axis=1)
        else:
            h = (lv.astype(np.int64) & 0xFFFF).astype(np.uint16)
            rec[r0 * 16:(r0 + G) * 16] = h.view(np.uint32)

    def _unpack(self, rec, r0, G):
        if self.q == Q_QS8:
            return rec[r0 * 8:(r0 + G) * 8].copy().view(np.int8).astype(np.int64)
        if self.q == Q_QS9:
            mag = rec[r0 * 8:(r0 + G) * 8].copy().view(np.uint8).astype(np.int64)
            sw = rec[self.Gtot * 8 + r0:self.Gtot * 8 + r0 + G]
            neg = ((sw[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).reshape(-1)
            return np.where(neg == 1, -mag, mag)
        return rec[r0 * 16:(r0 + G) * 16].copy().view(np.int16).astype(np.int64)


# ================================================================================= parity mode
class DenseWrap(Codec):
    """Reference wire format: every rank all-reduces its *dense* compressed vector
    (``core.py:217-225``). Implemented as the inner codec's compress → local decode (world=1) →
    all-reduce → ``/ world_size``."""
    collective = "all_reduce"

    def __init__(self, inner: Codec):
        super().__init__(inner.plan, inner.world, inner.rank, inner.seed, inner.error_feedback)
        self.inner = inner
        self.uses_step = inner.uses_step
        self.name = f"dense({inner.name})"

    @property
    def graph_safe(self) -> bool:
        # the threshold methods' dense path is sync-free and step-invariant
        # (tests/test_sync_free_gpu.py)
        return isinstance(self.inner, ThresholdCodec) or bool(self.inner.graph_safe)

    def compress(self, grad, ef, step):
        if isinstance(self.inner, ThresholdCodec):
            self.inner.compress_dense(grad, ef)
            self.last_payload_bytes = grad.numel() * grad.element_size()
            return grad
        payload = self.inner.compress(grad, ef, step)
        if isinstance(self.inner, DenseCodec):
            return grad
        self.inner.decompress(payload, None, grad, world=1)
        self.last_payload_bytes = grad.numel() * grad.element_size()
        return grad

    def decompress(self, send, recv, grad, world=None):
        w = int(world or self.world)
        if w != 1:                              # (world 1: no kernel for a division by 1)
            grad.div_(float(w))


# ================================================================================= quantised RS
class QuantRSCodec(Codec):
    """Quantised reduce-scatter wire for TernGrad / QSGD at world > 1 (SURVEY.md §2.4
    "Quantisers"; the reference all-reduces the dequantised dense vector, ``CIFAR10/core.py:207-225``).

    Quantised codes do not sum, so the all-gather wire brings every rank all W code vectors —
    ``(W-1)·b·n`` bytes in for ``b`` bytes of code per element — and the parity wire all-reduces
    fp32 (``2(W-1)/W·4n``). Here each rank quantises its whole bucket exactly as the all-gather
    codec does (same Philox streams, same error-feedback residual), then:

    1. **all-to-all of codes** (grouped ``ncclSend``/``ncclRecv``, ``csrc/rccl.cpp``): rank ``q``
       receives, from every rank, only the code records of ITS shard of the bucket's 32-element
       groups plus the per-segment scale header — ``(W-1)/W·b·n`` bytes;
    2. **shard dequant-sum** (``csrc/compress.hip k_dequant_shard``): the rank-ordered mean over the
       W pieces — the all-gather decode's arithmetic, bit for bit — rounded once to bf16 into a
       bucket image;
    3. **bf16 all-gather of the shards** (grouped send/recv, shard sizes differ by at most one
       group plus alignment gaps) — ``(W-1)/W·2n`` bytes — and one expand into the fp32 gradient.

    QSGD-255 at world 8 moves ``(7/8)·(1.13 + 2) ≈ 2.7`` B/element instead of 7 (fp32
    all-reduce) or 7.9 (code all-gather). The result is the mean over ranks of each rank's
    dequantised vector rounded to bf16 — identical on every rank (every rank, the shard owner
    included, keeps the rounded value). ``wire="auto"`` takes it when it moves the fewest bytes;
    ``wire="qrs"`` forces it."""
    collective = "quant_rs"

    def __init__(self, inner: "_QuantCodec"):
        super().__init__(inner.plan, inner.world, inner.rank, inner.seed, inner.error_feedback)
        self.inner = inner
        self.uses_step = inner.uses_step
        self.name = f"qrs({inner.name})"
        plan, W = inner.plan, self.world
        self.q = inner.q
        self.RL = {Q_TERN: 2, Q_QS8: 8, Q_QS9: 8, Q_QS16: 16}[inner.q]
        self.signs = inner.q == Q_QS9
        self.hdr = inner.hdr
        self.Gtot = inner.Gtot
        G = plan.groups().astype(np.int64)
        seg = np.repeat(np.arange(plan.S, dtype=np.int64), G)
        j = np.arange(self.Gtot, dtype=np.int64) - inner.rec_off[seg]
        off = plan.offsets[seg] + GROUP * j
        nval = np.minimum(GROUP, plan.sizes[seg] - GROUP * j)
        self.gtab = np.stack([seg, off, nval, np.zeros_like(seg)], 1).astype(np.int32)
        self.n = int(plan.numel)
        self.g_lo = [r * self.Gtot // W for r in range(W + 1)]
        self.A = [int(off[g]) if g < self.Gtot else self.n for g in self.g_lo[:-1]] + [self.n]
        per = self.RL + (1 if self.signs else 0)
        self.wpr = [(self.hdr + (self.g_lo[r + 1] - self.g_lo[r]) * per + 3) // 4 * 4
                    for r in range(W)]
        r = self.rank
        sent = sum(self.hdr + (self.g_lo[p + 1] - self.g_lo[p]) * per for p in range(W) if p != r)
        self.wire_bytes = 4 * sent + 2 * (W - 1) * (self.A[r + 1] - self.A[r])
        self._bufs = {}
        self._last_send = None

    @property
    def graph_safe(self) -> bool:
        return bool(self.inner.graph_safe)

    def can_stage(self) -> bool:
        return self.inner.can_stage()

    def stage(self, grad, ef, step, t_lo, t_hi, first):
        return self.inner.stage(grad, ef, step, t_lo, t_hi, first)

    def _buf(self, key, device, n, dtype):
        k = (key, str(device))
        b = self._bufs.get(k)
        if b is None:
            b = torch.zeros(n, dtype=dtype, device=device)
            self._bufs[k] = b
        return b

    def gtab_dev(self, device) -> torch.Tensor:
        return self.plan.dev(torch.device(device), "qrs_gtab", lambda: torch.from_numpy(self.gtab))

    def compress(self, grad, ef, step):
        self.inner._staged = self._staged
        try:
            out = self.inner.compress(grad, ef, step)
        finally:
            self.inner._staged = False
        self.last_payload_bytes = self.wire_bytes
        return out

    # ---- phase 1: code pieces
    def pieces(self, payload: torch.Tensor, dest: int):
        """The records of shard ``dest`` in a full payload: header, level words, (QS9) sign words."""
        h, g0, g1 = self.hdr, self.g_lo[dest], self.g_lo[dest + 1]
        out = [payload[:h], payload[h + g0 * self.RL:h + g1 * self.RL]]
        if self.signs:
            s0 = h + self.Gtot * 8
            out.append(payload[s0 + g0:s0 + g1])
        return out

    def piece_slots(self, row: torch.Tensor, shard: int):
        """Where the pieces of :meth:`pieces` land in one rank's row of the shard receive buffer."""
        h, ng = self.hdr, self.g_lo[shard + 1] - self.g_lo[shard]
        out = [row[:h], row[h:h + ng * self.RL]]
        if self.signs:
            out.append(row[h + ng * self.RL:h + ng * self.RL + ng])
        return out

    def recv1(self, device, shard: int) -> torch.Tensor:
        return self._buf(("r1", shard), device, self.world * self.wpr[shard], torch.int32)

    def image(self, device) -> torch.Tensor:
        return self._buf("img", device, self.n, torch.bfloat16)

    def reduce_shard(self, recv1: torch.Tensor, shard: int, img: torch.Tensor) -> None:
        """Rank-ordered dequantise-and-average of shard ``shard`` into the bf16 bucket image."""
        W, g0 = self.world, self.g_lo[shard]
        ng = self.g_lo[shard + 1] - g0
        lib = ops_for(img) if img.is_cuda else None
        if lib is not None:
            lib.dequant_shard(recv1, W, self.hdr, self.gtab_dev(img.device), g0, ng, self.q,
                              self.inner.qstates, img)
            return
        rows = recv1.view(W, -1).numpy().view(np.uint32)
        h = self.hdr
        gt = self.gtab[g0:g0 + ng]
        acc = np.zeros(ng * GROUP, dtype=np.float32)
        for r in range(W):
            row = rows[r]
            sc = row[:h].view(np.float32)[gt[:, 0]].repeat(GROUP)
            lv = row[h:h + ng * self.RL]
            if self.q == Q_TERN:
                codes = ((lv.reshape(ng, 2, 1) >> (2 * np.arange(16, dtype=np.uint32))[None, None, :])
                         & np.uint32(3)).reshape(-1)
                acc += self.inner._deq(codes, sc)
                continue
            if self.q == Q_QS8:
                signed = lv.copy().view(np.int8).astype(np.int64)
            elif self.q == Q_QS9:
                mag = lv.copy().view(np.uint8).astype(np.int64)
                sw = row[h + ng * 8:h + ng * 9]
                neg = ((sw[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).reshape(-1)
                signed = np.where(neg == 1, -mag, mag)
            else:
                signed = lv.copy().view(np.int16).astype(np.int64)
            acc += self.inner._deq(signed, sc)
        mean = torch.from_numpy(acc / np.float32(W)).to(torch.bfloat16)
        for gi in range(ng):
            o, nv = int(gt[gi, 1]), int(gt[gi, 2])
            img[o:o + nv] = mean[gi * GROUP:gi * GROUP + nv]

    def exchange(self, comm, send: torch.Tensor) -> torch.Tensor:
        """Phases 1-3 over ``comm`` (``send_recv(sends, send_peers, recvs, recv_peers, key)``:
        the native RCCL communicator, its loopback stand-in or the c10d adapter). Returns the bf16
        bucket image every rank ends with."""
        W, r, dev = self.world, self.rank, send.device
        self._last_send = send
        r1 = self.recv1(dev, r)
        rows = r1.view(W, -1)
        sends, sp, recvs, rp = [], [], [], []
        for q in range(W):
            ps = self.pieces(send, q)
            sends += ps
            sp += [q] * len(ps)
            slots = self.piece_slots(rows[q], r)
            recvs += slots
            rp += [q] * len(slots)
        comm.send_recv(sends, sp, recvs, rp, key=(self, 1))
        img = self.image(dev)
        self.reduce_shard(r1, r, img)
        mine = img[self.A[r]:self.A[r + 1]]
        peers = [q for q in range(W) if q != r]
        comm.send_recv([mine] * len(peers), peers,
                       [img[self.A[q]:self.A[q + 1]] for q in peers], peers, key=(self, 2))
        return img

    def decompress(self, send, recv, grad, world=None):
        img = recv if recv is not None else self.image(grad.device)
        dst = grad[:self.n]
        lib = ops_for(dst) if dst.is_cuda else None
        if lib is not None:
            lib.bf16_expand(img, dst)
        else:
            dst.copy_(img.float())


# ================================================================================= factory
def make_codec(method, plan: SegPlan, world: int, rank: int, K=None, V=None, qstates=None,
               seed: int = 0, error_feedback: bool = False, wire: str = "auto",
               count_exchange=None, max_density=None, dense_below: int = 0) -> Codec:
    """Build the codec for ``method`` honouring the reference's falsy-parameter guards
    (``core.py:178-215``: ``Topk`` without K, ``Thresholdv`` without V... mean no compression).

    ``dense_below`` (opt-in deviation, Top-K / Random-K): a tensor of at most that many elements
    travels whole instead of keeping ``ceil(nK)``. The reference keeps >= 1 element of every
    layer, so a 64-element BatchNorm tensor at K = 1 % sends 1 element a step; with error
    feedback the other 63 accumulate ~64 steps of gradient and are released in bursts
    (``profiles/r4/ef_root_cause.md``)."""
    method = ref.canonical_method(method)
    if method == "Topk" and K:
        if K >= 1.0:
            c = DenseCodec(plan, world, rank, seed)
        else:
            c = TopkCodec(plan, world, rank, K, seed, error_feedback, dense_below)
    elif method == "Randomk" and K:
        if wire in ("sparse",):
            c = RandkSparseCodec(plan, world, rank, K, seed, error_feedback, dense_below)
        else:
            c = RandkCodec(plan, world, rank, K, seed, error_feedback, dense_below)
    elif method in ("Thresholdv", "AdaptiveThreshold") and (V or method == "AdaptiveThreshold"):
        # sparse wire capacity: agreed per step by the count exchange ("sparse" /
        # "sparse-exact": exact, like the reference's |g| >= V), or fixed per segment
        # ("sparse-capped": sync-free and graph-capturable, hits beyond the cap are counted and
        # stay in the error-feedback residual — dropped without EF)
        dens = None
        if wire == "sparse-capped" or max_density is not None:
            dens = float(max_density if max_density is not None else 0.05)
            if not error_feedback and rank == 0:
                import warnings
                msg = (f"{method} on the capped sparse wire without error feedback: hits beyond "
                       f"{dens:.1%} of a segment are dropped (counted in comm/overflow); use "
                       f"wire='sparse' for the exact rule")
                warnings.warn(msg, stacklevel=2)
        c = ThresholdCodec(plan, world, rank, V=V, adaptive=method == "AdaptiveThreshold",
                           seed=seed, error_feedback=error_feedback,
                           count_exchange=count_exchange, max_density=dens)
    elif method == "TernGrad":
        c = TernGradCodec(plan, world, rank, seed, error_feedback)
    elif method == "RandomDithering" and qstates:
        c = QSGDCodec(plan, world, rank, qstates, seed, error_feedback)
    else:
        c = DenseCodec(plan, world, rank, seed)
    if wire == "dense" and not isinstance(c, DenseCodec):
        return DenseWrap(c)
    if wire == "qrs":
        if not isinstance(c, _QuantCodec):
            raise ValueError(f"wire='qrs' (quantised reduce-scatter) needs TernGrad / QSGD, "
                             f"not {method}")
        return QuantRSCodec(c) if world > 1 else c
    if wire == "auto" and isinstance(c, ThresholdCodec):
        # data-dependent counts: the sparse wire needs the per-step count exchange and a host
        # read of the agreed capacity (a sync in the middle of backward); the reference's dense
        # wire (compressed vector, all-reduce) is exact and sync-free — `wire="sparse"` opts in
        return DenseWrap(c)
    if wire == "auto" and isinstance(c, TopkCodec) and c.collective == "all_gather" and \
            not isinstance(c, ThresholdCodec):
        # pairs cost 8 B per kept element on every rank: dense all-reduce wins above ~1/world
        # (index-free Random-K sends only its values, one all-reduce: never worth densifying)
        if c.cap_total * max(world, 2) > plan.numel:
            return DenseWrap(c)
    if wire == "auto" and isinstance(c, _QuantCodec) and world > 1:
        # bytes into each rank per element (b = code bytes per element): the code all-gather
        # (W-1)·b; the quantised reduce-scatter (W-1)/W·(b + 2); the ring all-reduce of the
        # dequantised fp32 vector 2(W-1)/W·4. QSGD-255 (b ≈ 1.13): all-gather at W = 2,
        # reduce-scatter from 3 on; TernGrad (b ≈ 0.25): all-gather up to 9 ranks
        n, W = max(plan.numel, 1), world
        b = c.words * 4 / n
        cost = {"ag": (W - 1) * b, "qrs": (W - 1) / W * (b + 2), "dense": 2 * (W - 1) / W * 4}
        best = min(cost, key=lambda k: (cost[k], k != "ag"))
        if best == "qrs":
            return QuantRSCodec(c)
        if best == "dense":
            return DenseWrap(c)
    return c
