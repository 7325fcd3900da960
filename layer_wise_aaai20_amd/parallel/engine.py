"""Gradient synchronisation engine: arena + buckets + codecs + async collectives.

One engine drives both entry styles of the reference:

* **hook-driven, overlapped with backward** — what ``CompressedDDP`` uses. Each parameter's
  post-accumulate-grad hook marks its segment ready; when every segment of a bucket is ready the
  bucket is compressed and its collective launched asynchronously, strictly in bucket order so all
  ranks issue collectives identically (the reference's reverse-order ``next_bucket`` rule,
  ``ddp.py:434-450``, ``sparsified_ddp.py:424-445``). A callback queued on the autograd engine
  finishes the step: launch leftovers, wait, decompress.
* **after backward** — the reference's functional ``layerwise_compressed_comm`` /
  ``entiremodel_compressed_comm`` / ``all_reduce`` (``CIFAR10/core.py:175-301``,
  ``train_imagenet_nv.py:382-386``): :meth:`sync_now` launches every bucket, then finishes.

Both end with ``param.grad`` = mean over ranks of each rank's compressed gradient, written into the
flat arena. No gradient is ever reduced twice.
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from . import comm
from .arena import Bucket, GradArena, plan_buckets
from ..compress import reference as ref
from ..compress.codecs import Codec, DenseCodec, DenseWrap, TopkCodec, make_codec
from ..compress.plan import SegPlan

MODES = ("layerwise", "entiremodel", "none")
# entire-model first-pass staging during backward (_plan_stages); False (tests only): the whole
# chain after backward, the single-launch form the staged one must equal bit for bit
EM_STAGE = True
# claimed overwrites (claim_overwrite); False (tests only): zero every segment and accumulate
CLAIM_OVERWRITE = True
MODE_ALIASES = {"enitremodel": "entiremodel", "entire": "entiremodel", "entire-model": "entiremodel",
                "layer-wise": "layerwise", "layer": "layerwise", None: "none", "": "none",
                "None": "none"}


def canonical_mode(mode) -> str:
    mode = MODE_ALIASES.get(mode, mode)
    if mode not in MODES:
        raise ValueError(f"unknown --compress mode {mode!r}; expected one of {MODES}")
    return mode


@dataclass
class SyncStats:
    steps: int = 0
    payload_bytes: int = 0          # bytes this rank sent last step
    dense_bytes: int = 0            # fp32 gradient bytes (what an uncompressed all-reduce moves)
    buckets: int = 0
    overflow: int = 0               # last read_overflow(): selected elements the payload dropped
    history: List[float] = field(default_factory=list)

    @property
    def ratio(self) -> float:
        return self.payload_bytes / max(self.dense_bytes, 1)


class GradSyncEngine:
    def __init__(self, named_params, mode: str = "layerwise", method="none", K=None, V=None,
                 qstates=None, error_feedback: bool = False, bucket_cap_mb: float = 25.0,
                 first_bucket_mb: Optional[float] = None, last_bucket_mb: Optional[float] = 4.0,
                 wire: str = "auto",
                 seed: int = 2147483647, process_group=None, flat_params: bool = False,
                 world_size: Optional[int] = None, timing: bool = False,
                 overlap_compress: bool = True, dense_below: int = 0,
                 momentum_correction: float = 0.0, ef_lr_scaled: bool = False,
                 max_density: Optional[float] = None):
        self.mode = canonical_mode(mode)
        self.method = ref.canonical_method(method) if self.mode != "none" else "none"
        self.pg = process_group
        self.world = world_size or comm.world_size(self.pg)
        self.rank = comm.rank(self.pg)
        named = list(named_params)
        align = 1 if self.mode == "entiremodel" else 64
        self.arena = GradArena(named, flat_params=flat_params, align=align)
        self.device = self.arena.device
        cap = int(bucket_cap_mb * 2 ** 20)
        first = int(first_bucket_mb * 2 ** 20) if first_bucket_mb else None
        last = int(last_bucket_mb * 2 ** 20) if last_bucket_mb else None
        self.buckets: List[Bucket] = plan_buckets(self.arena, self.mode, cap, first,
                                                  last if last and last < cap else None)
        self.seed = int(seed)
        self.ef = torch.zeros_like(self.arena.grad) if (error_feedback and
                                                       self.method != "none") else None
        if self.method == "RandomDithering" and self.ef is not None and qstates and \
                int(qstates) <= 255:
            # EF needs a contractive compressor (||C(v) - v|| < ||v||); QSGD with s levels on n
            # elements has relative variance up to sqrt(n)/s — ~20 on ResNet-9 at s = 127 —
            # so the residual grows geometrically (loss 1e14 within 200 steps on MI355X,
            # tests/test_convergence_gpu.py)
            import warnings
            msg = (f"QSGD (RandomDithering) with qstates={qstates} and error feedback is not "
                   f"contractive on large tensors: the residual can diverge; use qstates >= "
                   f"~4096 (16-bit codes) with --error_feedback, or drop error feedback")
            warnings.warn(msg, stacklevel=2)
            if self.rank == 0:
                print(f"[lwaaai] warning: {msg}", flush=True)
        # DGC-style momentum correction (opt-in, Lin et al. 2018; profiles/r4/ef_root_cause.md):
        # each rank accumulates its velocity u = m·u + (g + wd·p) locally and the error-feedback
        # residual accumulates u instead of g; the coordinates that were sent have their velocity
        # zeroed (momentum factor masking). With the Top-K / Random-K selection kernels, tensors
        # sent whole (dense_below, or every element kept) keep ordinary momentum; codecs without
        # a selection (thresholds, quantisers, the dense parity wire) are masked by k_mc_mask
        # wherever the residual is zero, so a tensor they send whole restarts its velocity every
        # step (pinned by tests/test_engine_cpu.py::test_mc_mask_resets_whole_segments). Weight decay enters the gradient
        # BEFORE the velocity, as in DGC (set_mc_weight_decay; the optimizer then runs without
        # momentum and without weight decay — the trainers switch both off). One kernel does the
        # prologue (csrc/optim.hip k_mc_prep); the masking runs inside the select kernels
        # (csrc/compress.hip, SelectArgs::mom) or, for codecs without a selection, in k_mc_mask.
        # Needs error feedback.
        self.mc = float(momentum_correction or 0.0)
        self.mom = None
        self._mc_wd = None                # per arena segment (device fp32) or None
        self._mc_wmul = 1.0
        self._mc_plans = {}
        if self.mc > 0:
            if self.ef is None:
                raise ValueError("momentum correction needs error_feedback=True")
            self.mom = torch.zeros_like(self.arena.grad)
        # LR-scaled residuals (opt-in, EF-SGD's "residual in update units"): the residual left at
        # step t-1 was meant to be applied at lr_{t-1}; before step t adds it to the new gradient
        # it is rescaled by lr_{t-1} / lr_t, so a warm-up / decay schedule neither amplifies nor
        # damps the deferred updates. The LR comes from ``lr_source`` (a callable returning the
        # optimizer's 1-element device LR, FlatSGD.lr_device) and the ratio is computed on the
        # device in begin_step, so it stays inside a captured step.
        self.lr_scaled = bool(ef_lr_scaled)
        self.lr_source = None
        if self.lr_scaled:
            if self.ef is None:
                raise ValueError("LR-scaled residuals need error_feedback=True")
            self._lr_prev = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._lr_ratio = torch.ones(1, dtype=torch.float32, device=self.device)
        # what a peer needs to build this engine's codecs for another rank (loopback tests)
        # (max_density: the capped sparse threshold wire's per-segment capacity, default 5 %)
        self.codec_kw = dict(K=K, V=V, qstates=qstates, seed=self.seed,
                             error_feedback=self.ef is not None, wire=wire,
                             dense_below=int(dense_below or 0), max_density=max_density)
        self.codecs: List[Codec] = []
        self.plans: List[SegPlan] = []
        for b in self.buckets:
            segs = self.arena.segments[b.seg_lo:b.seg_hi]
            if self.mode == "entiremodel":
                plan = SegPlan([0], [self.arena.numel], gid_base=0)
            else:
                plan = SegPlan([s.offset - b.start for s in segs], [s.numel for s in segs],
                               gid_base=b.seg_lo)
            self.plans.append(plan)
            self.codecs.append(make_codec(self.method, plan, self.world, self.rank,
                                          count_exchange=self._count_exchange,
                                          **self.codec_kw))
        # device mirror of self.step for the Philox-keyed kernels (Random-K, TernGrad, QSGD):
        # advanced by finish() on the GPU, so a replayed HIP graph of the step advances it too
        self._dstep = (torch.zeros(1, dtype=torch.int64, device=self.device)
                       if self.device.type == "cuda" else None)
        # device count of elements the reference rule selected but the payload could not carry
        # (Top-K ties beyond the slack, threshold hits beyond a fixed capacity; read_overflow)
        self._overflow = (torch.zeros(1, dtype=torch.int64, device=self.device)
                          if self.device.type == "cuda" else None)
        for c in self.codecs:
            c.step_t = self._dstep
            c.overflow = self._overflow
            inner = getattr(c, "inner", None)          # (DenseWrap, QuantRSCodec)
            if inner is not None:
                inner.step_t = self._dstep
                inner.overflow = self._overflow
        self.seg_bucket = [0] * len(self.arena.segments)
        for b in self.buckets:
            for i in range(b.seg_lo, b.seg_hi):
                self.seg_bucket[i] = b.index
        self._plan_stages(cap)
        self._sgd = None                 # set_fused_sgd: decode + optimizer step in one pass
        self._sgd_buckets = frozenset()
        # claimed overwrites (claim_overwrite): segments left out of the per-step zeroing
        self._claims = [0] * len(self.arena.segments)
        self._no_zero = frozenset()
        self.step = 0
        self.stats = SyncStats(dense_bytes=self.arena.numel * 4, buckets=len(self.buckets))
        self.timing = timing and self.device.type == "cuda"
        self.timings: List[dict] = []
        # compression + collective launch run on a side HIP stream, ordered after the bucket's
        # last gradient by an event, so they overlap the rest of the backward pass; the compute
        # stream waits on a second event only when it decodes in finish()
        self._side = (torch.cuda.Stream(device=self.device)
                      if overlap_compress and self.device.type == "cuda" else None)
        # inside a captured step (LWAAAI_GRAPH_OVERLAP):
        #   "0"    each bucket is compressed, exchanged and decoded inline on the compute stream,
        #          in backward order as its gradients complete;
        #   "comm" compression inline, only the bucket's RCCL collective on a side branch;
        #   "1"    compression and collective both on the side branch, overlapping the rest of
        #          backward (the reference's hook-driven DDP, sparsified_ddp.py:403-452);
        #   "auto" (default) = "0": the measured winner with the xGMI transfer priced in. The
        #          world-8 simulation with every collective paying its modelled wire time on 16
        #          busy workgroups (profiles/r6/sim8_wire_r50_overlap_modes.jsonl, train/simworld.py) exposed
        #          ResNet-50 layer-wise Top-K 0.1 % by 0.22 ms inline vs 0.74 ms ("1") and 0.87 ms
        #          ("comm"); entire-model QSGD-255 on the quantised reduce-scatter wire 0.48 /
        #          0.83 / 0.41 ms; AlexNet entire-model Top-K 0.07 ms in all three. The step is
        #          throughput-bound: side-branch kernels slow the backward GEMMs they run beside
        #          by more than the transfers they hide (3 x ~75 KB / 15 us latency per step for
        #          Top-K).
        # Eager (uncaptured) steps keep the side stream.
        # Known issue: in the one-GPU rehearsal (2 ranks sharing the card, RCCL over its socket
        # transport) capturing "1" or "comm" segfaults inside hipStreamEndCapture (profiles/r6/
        # multigpu_overlap1_r6d.txt, multigpu_overlap_comm_r6f.txt): an RCCL collective on a
        # forked capture branch; "0" captures and matches eager there (tests/test_multigpu_gpu.py).
        mode = os.environ.get("LWAAAI_GRAPH_OVERLAP", "auto")
        if mode not in ("0", "1", "comm", "auto"):
            raise ValueError(f"LWAAAI_GRAPH_OVERLAP={mode!r}: expected auto, 0, 1 or comm")
        self._overlap_mode = mode
        self._graph_overlap = False
        self._comm_only = False
        self._retired = []            # (fence event, events held until it completes)
        self._check = os.environ.get("LWAAAI_ENGINE_CHECK", "0") == "1"
        # bucket collectives on a native RCCL communicator (csrc/rccl.cpp) when the group is
        # nccl: stream-ordered calls without c10d Work objects, so a captured step never puts
        # events on the ProcessGroup watchdog's list (see graph_safe)
        self._native = (comm.native_rccl(self.pg, self.device)
                        if self.device.type == "cuda" else None)
        self._stream_waitable = self._native is not None or (
            comm.is_dist() and comm.world_size(self.pg) > 1 and
            comm.dist.get_backend(self.pg) == "nccl")
        # a rank that stops taking part would leave the others blocked inside RCCL forever: the
        # watchdog (csrc/rccl.cpp) turns that into an abort + non-zero exit after the deadline
        self._watch = None
        if self._native is not None and self.world > 1 and comm.comm_timeout() > 0:
            self._watch = (getattr(self._native, "watch", None) or
                           self._native.start_watchdog(comm.comm_timeout()))
        self._set_inplace_gather()
        self.set_graph_overlap(self._overlap_mode)
        self._reset_state()
        self.all_reduced_last = True
        self.verify_plan()

    def set_graph_overlap(self, mode: str) -> None:
        """Where a captured step runs each bucket's exchange (see LWAAAI_GRAPH_OVERLAP above)."""
        if mode not in ("0", "1", "comm", "auto"):
            raise ValueError(f"graph overlap mode {mode!r}: expected auto, 0, 1 or comm")
        self._overlap_mode = mode
        if mode == "auto":
            mode = "0"
        self._graph_overlap = mode != "0"
        self._comm_only = mode == "comm"

    def graph_overlap_mode(self) -> str:
        """The effective captured-step exchange mode: "0", "1" or "comm"."""
        return "0" if not self._graph_overlap else ("comm" if self._comm_only else "1")

    # ----------------------------------------------------------------- failure detection
    def plan_signature(self) -> List[int]:
        """Layout fingerprint: every rank must build the same buckets / codecs, otherwise the
        collectives would silently pair mismatched payloads (or hang)."""
        import zlib
        desc = repr([(b.start, b.end, c.name, getattr(c, "cap_total", 0))
                     for b, c in zip(self.buckets, self.codecs)]) + self.mode + self.method
        return [zlib.crc32(desc.encode()) & 0x7FFFFFFF, self.arena.numel, len(self.buckets)]

    def verify_plan(self) -> None:
        if not comm.is_dist() or comm.world_size(self.pg) == 1:
            return
        mine = torch.tensor(self.plan_signature(), dtype=torch.int64,
                            device=self.device if comm.dist.get_backend(self.pg) == "nccl"
                            else "cpu")
        lo, hi = mine.clone(), mine.clone()
        comm.dist.all_reduce(lo, op=comm.dist.ReduceOp.MIN, group=self.pg)
        comm.dist.all_reduce(hi, op=comm.dist.ReduceOp.MAX, group=self.pg)
        if not torch.equal(lo, hi):
            raise RuntimeError(
                f"rank {self.rank}: gradient bucket plans differ across ranks (signature "
                f"{mine.tolist()} vs min {lo.tolist()} / max {hi.tolist()}): the model, the "
                f"compression settings or the bucket size are not identical on every rank")

    # ----------------------------------------------------------------- entire-model staging
    def _plan_stages(self, cap_bytes: int) -> None:
        """Entire-model mode compresses the flattened model as ONE segment, so its statistic —
        the Top-K radix pass-0 histogram, the QSGD norm / TernGrad max — covers every gradient and
        the whole chain used to run after backward. Here the arena is cut into slices of whole
        8192-element tasks (about ``bucket_cap_mb`` each); when every parameter overlapping a
        slice has its gradient, that slice's share of the first pass runs (with the
        error-feedback fold) on the side stream, overlapped with the rest of backward. The
        histogram counts are integers and the quantisers' partials land in per-task slots, so
        the result is bit-identical to the single launch (tests/test_loopback_gpu.py); only the
        rest of the chain stays after backward. (Momentum correction
        and LR-scaled residuals rewrite the gradient in their prologue: no staging with them.)"""
        self._stages = []
        if not (self.mode == "entiremodel" and self.device.type == "cuda" and self.mom is None
                and not self.lr_scaled and len(self.codecs) == 1 and EM_STAGE):
            return
        codec = self.codecs[0]
        sel = codec.inner if isinstance(codec, DenseWrap) else codec
        if not sel.can_stage():
            return
        from ..compress.plan import LARGE_EPB
        n = self.arena.numel
        per = max(LARGE_EPB, (cap_bytes // 4) // LARGE_EPB * LARGE_EPB)
        if n <= per:
            return
        bounds = list(range(0, n, per)) + [n]
        segs = self.arena.segments
        self._stages = [(lo, hi, -(-hi // LARGE_EPB) if hi == n else hi // LARGE_EPB)
                        for lo, hi in zip(bounds[:-1], bounds[1:])]
        self._stage_need = [0] * len(self._stages)
        self._seg_stages = [[] for _ in segs]
        for i, s in enumerate(segs):
            for si, (lo, hi, _) in enumerate(self._stages):
                if s.offset < hi and s.offset + s.numel > lo:
                    self._seg_stages[i].append(si)
                    self._stage_need[si] += 1

    def _stage_reset(self) -> None:
        self._stage_cnt = [0] * len(self._stages)
        self._stage_next = 0
        self._stage_events = []

    def _stage_in_order(self, force: bool = False) -> None:
        while self._stage_next < len(self._stages) and (
                force or self._stage_cnt[self._stage_next] == self._stage_need[self._stage_next]):
            self._stage(self._stage_next)
            self._stage_next += 1

    def _stage(self, si: int) -> None:
        self._flush_splitk()
        lo, hi, t_hi = self._stages[si]
        t_lo = lo // 8192 if si > 0 else 0
        codec = self.codecs[0]
        sel = codec.inner if isinstance(codec, DenseWrap) else codec
        e = self.ef if self.ef is not None else None
        side = self._side
        if side is not None and (not self._graph_overlap or self._comm_only) and \
                torch.cuda.is_current_stream_capturing():
            side = None                      # (inline inside a capture, as _launch's compression)
        if side is not None:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.device))
            side.wait_event(ready)
            self._stage_events.append(ready)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            sel.stage(self.arena.grad, e, self.step, t_lo, t_hi, si == 0)

    def set_mc_weight_decay(self, opt) -> None:
        """Momentum correction: take the weight decay of ``opt`` (a :class:`FlatSGD` over this
        engine's arena) into the velocity update, ``u = mc·u + g + wd·p`` per segment with each
        param group's decay (so ``--no-bn-wd`` still holds), and set the optimizer's groups to no
        decay. Without it, decay applied by the optimizer after the exchange never enters u and
        acts ~1/(1-mc) times weaker than in the momentum-SGD baseline."""
        if self.mom is None:
            raise RuntimeError("set_mc_weight_decay: momentum correction is off")
        if self.arena.param_buf is None:
            raise RuntimeError("set_mc_weight_decay: the arena has no flat parameter buffer")
        wd = opt._seg_wd(self.device).clone()
        self._mc_wd = wd if bool((wd != 0).any()) else None
        self._mc_wmul = 1.0 / float(getattr(opt, "grad_scale", 1.0) or 1.0)
        for g in opt.param_groups:
            g["weight_decay"] = 0.0
        self._mc_plans = {}

    def set_fused_sgd(self, opt) -> int:
        """Decode the Top-K buckets straight into the SGD step of ``opt`` (a
        :class:`FlatSGD` over this engine's arena): each 4096-element chunk's averaged gradient
        goes from LDS into the update of the same parameters (``csrc/compress.hip
        k_unpack_sgd``), so the dense gradient is neither written by the decode nor read back by
        the optimizer, and ``opt.step()`` then updates only the other
        buckets' segments. Same arithmetic as the separate passes (``csrc/sgd_elem.h``;
        tests/test_fused_sgd_gpu.py pins it bit for bit).

        Needs the trainer's order of operations: the step's LR set before backward (a captured
        step reads it from ``opt``'s device hyper tensor), ``opt.step()`` after backward. Returns
        the number of buckets fused (0: nothing changes)."""
        self._sgd, self._sgd_buckets = None, frozenset()
        if self.device.type != "cuda" or self.arena.param_buf is None:
            opt.exclude_segments(())
            return 0
        from ..compress.plan import UNPACK_CHUNK
        fused, segs = [], []
        self._sgd_tasks = {}
        for bi, b in enumerate(self.buckets):
            c = self.codecs[bi]
            if type(c) is not TopkCodec:
                continue
            plan = self.plans[bi]
            ours = self.arena.segments[b.seg_lo:b.seg_hi]
            rows = []
            if self.mode == "layerwise":
                if plan.S != len(ours) or any(int(plan.offsets[i]) != s.offset - b.start or
                                              int(plan.sizes[i]) != s.numel
                                              for i, s in enumerate(ours)):
                    continue
                for i, s in enumerate(ours):
                    rows += [(i, cb, min(cb + UNPACK_CHUNK, s.numel), i)
                             for cb in range(0, s.numel, UNPACK_CHUNK)]
            else:
                # one codec segment over the bucket: chunks cut at every parameter's bounds, so
                # each task has one weight decay
                if plan.S != 1 or int(plan.offsets[0]) != 0:
                    continue
                for i, s in enumerate(ours):
                    lo, hi = s.offset - b.start, s.offset - b.start + s.numel
                    rows += [(0, cb, min(cb + UNPACK_CHUNK, hi), i)
                             for cb in range(lo, hi, UNPACK_CHUNK)]
            self._sgd_tasks[bi] = torch.tensor(rows, dtype=torch.int32,
                                               device=self.device).reshape(-1, 4)
            fused.append(bi)
            segs.extend(range(b.seg_lo, b.seg_hi))
        opt.exclude_segments(segs)
        if fused:
            self._sgd, self._sgd_buckets = opt, frozenset(fused)
        return len(fused)

    def _sgd_args(self, bi: int) -> dict:
        opt, b = self._sgd, self.buckets[bi]
        pb = getattr(self.arena, "param_bf16", None)
        hyper = opt._hyper if (opt.device_hyper and opt._hyper is not None and
                               torch.cuda.is_current_stream_capturing()) else None
        return dict(tasks=self._sgd_tasks[bi],
                    p=self.arena.param_buf[b.start:b.end], buf=opt.buf[b.start:b.end],
                    pb=pb[b.start:b.end] if pb is not None else None,
                    seg_wd=opt._seg_wd(self.device)[b.seg_lo:b.seg_hi],
                    lr=float(opt._uniform("lr")), momentum=float(opt._uniform("momentum")),
                    dampening=float(opt._uniform("dampening")),
                    nesterov=bool(opt._uniform("nesterov")), first=bool(opt._first),
                    grad_scale=float(opt.grad_scale), hyper=hyper)

    def _mc_plan(self, bi: int):
        """The bucket's arena segments (a plan of its own: in entire-model mode the codec sees
        one segment, but weight decay is per parameter) and their weight decays."""
        if bi not in self._mc_plans:
            b = self.buckets[bi]
            segs = self.arena.segments[b.seg_lo:b.seg_hi]
            plan = SegPlan([s.offset - b.start for s in segs], [s.numel for s in segs])
            wd = self._mc_wd[b.seg_lo:b.seg_hi].contiguous() if self._mc_wd is not None else None
            self._mc_plans[bi] = (plan, wd)
        return self._mc_plans[bi]

    def _mc_fusable(self, bi: int, sel, g: torch.Tensor) -> bool:
        """The velocity update can run inside the Top-K chain's first pass: a GPU Top-K codec
        whose segments are the bucket's parameters (layer-wise), unstaged."""
        return (g.device.type == "cuda" and type(sel) is TopkCodec and
                self.mode == "layerwise" and not self._stages)

    def _mc_prologue(self, bi: int, g: torch.Tensor, u: torch.Tensor) -> None:
        """g' = g + wd·p/grad_scale ; u = mc·u + g' ; g = u over bucket ``bi``."""
        from ..ops._ext import ops_for
        b = self.buckets[bi]
        plan, wd = self._mc_plan(bi)
        p = self.arena.param_buf[b.start:b.end] if wd is not None else None
        lib = ops_for(g)
        if lib is not None:
            t = plan.all_large_tables(g.device)
            lib.mc_prep(g, u, p, t["seg_off"], t["seg_n"], t["segs"], t["tasks"], wd, self.mc,
                        self._mc_wmul)
            return
        for i in range(plan.S):                  # (segments may be padded apart: align 64)
            o, n = int(plan.offsets[i]), int(plan.sizes[i])
            if wd is not None and float(wd[i]) != 0.0:       # (product, then sum: the kernel's
                w32 = torch.tensor(float(wd[i]), dtype=torch.float32) * \
                    torch.tensor(self._mc_wmul, dtype=torch.float32)   # roundings)
                g[o:o + n].add_(p[o:o + n] * w32)
            u[o:o + n].mul_(self.mc).add_(g[o:o + n])
            g[o:o + n].copy_(u[o:o + n])

    def _set_inplace_gather(self) -> None:
        """All-gather codecs write their payload into their row of the collective's output when
        the communicator is a stream-ordered native one (RCCL's in-place all-gather; the loopback
        stand-in then copies only the peers' rows). c10d keeps separate buffers."""
        for c in self.codecs:
            c.inplace_gather = self._native is not None and c.collective == "all_gather"

    def use_communicator(self, native) -> None:
        """Route the bucket collectives through ``native`` (a :class:`~.comm.NativeRccl`-like
        object: stream-ordered ``all_gather(out, inp)`` / ``all_reduce(t)`` / ``broadcast``),
        e.g. the single-GPU :class:`~.loopback.LoopbackRccl` that stands in for a world of W
        ranks. Its world size must be the one the codecs were built for."""
        w = getattr(native, "world", self.world)
        if w != self.world:
            raise ValueError(f"communicator world {w} != engine world {self.world}")
        self._native = native
        self._stream_waitable = True
        self._set_inplace_gather()
        self.set_graph_overlap(self._overlap_mode)

    # ----------------------------------------------------------------- state machine
    def _reset_state(self):
        self._stage_reset()
        self._marked = bytearray(len(self.arena.segments))
        nb = len(self.buckets)
        self._ready_cnt = [0] * nb
        self._ready = [False] * nb
        self._next = 0
        self._pending = []
        self._active = False
        self._payload = 0

    def _count_exchange(self, caps: torch.Tensor) -> torch.Tensor:
        return comm.all_reduce_max(caps, self.pg)

    def claim_overwrite(self, seg_index: int) -> bool:
        """A fused op about to write segment ``seg_index``'s whole gradient asks whether it may
        overwrite (True) instead of accumulating into the arena view (False). True only for a
        segment that the previous step's backward wrote through exactly one claim — those are
        left out of begin_step's zeroing — and only for its first claim of this step (a second
        use of the weight in the same step accumulates, and the segment is zeroed again from the
        next step on). The caller must be the segment's only gradient contribution when it
        overwrites (ops/gemm.py _ReplicatedLinearFn: VGG-16's 103 M-weight fc1, whose zeroing
        plus read-add-write cost about three passes over 412 MB a step)."""
        if not CLAIM_OVERWRITE:
            return False                 # (not counted: the segment stays under zeroing)
        self._claims[seg_index] += 1
        return self._claims[seg_index] == 1 and seg_index in self._no_zero

    def begin_step(self) -> None:
        """Zero the arena (but for the segments whole-written by a claimed overwrite in the last
        step) and re-point ``.grad`` at it (called before forward/backward)."""
        if any(self._claims):            # (a backward ran since the last call)
            self._no_zero = frozenset(i for i, c in enumerate(self._claims) if c == 1)
            self._claims = [0] * len(self.arena.segments)
        if not self._no_zero:
            self.arena.zero_()
        else:
            self.arena.zero_except(self._no_zero)
        if self.device.type == "cuda":
            from ..ops import block as _block
            from ..ops._ext import splitk_discard, splitk_pending
            if splitk_pending():
                # left over from a step that never reached its flush (a backward that raised):
                # their slabs belong to that step and must not be added into this one's arena
                n = splitk_discard(self.arena.grad)
                print(f"[lwaaai] dropped {n} split-K reduces left by an unfinished step",
                      flush=True)
            _block.new_step()            # (per-step weight-pack batch: ops/conv.py kc_pack)
        if not self.arena.grads_attached():
            self.arena.attach_grads()
        if self.lr_scaled:
            if self.lr_source is None:
                raise RuntimeError("ef_lr_scaled: set engine.lr_source to the optimizer's LR")
            cur = self.lr_source()
            ok = (self._lr_prev > 0) & (cur > 0)
            self._lr_ratio.copy_(torch.where(ok, self._lr_prev / torch.where(ok, cur, 1.0), 1.0))
            self._lr_prev.copy_(cur)
        self._reset_state()

    def mark_ready(self, seg_index: int) -> None:
        """A segment's gradient is complete in the arena. Idempotent within a step: a parameter
        whose gradient a fused op wrote straight into the arena is announced by that op, and
        autograd then runs its post-accumulate-grad hook as well (PyTorch calls those hooks even
        when the Function returned no gradient for the input) — counted twice, the bucket would
        launch before its other segments were written (profiles/r2_vgg_fault.md)."""
        if self._marked[seg_index]:
            return
        self._marked[seg_index] = 1
        if self._check and self.seg_bucket[seg_index] < self._next:
            raise RuntimeError(f"segment {self.arena.segments[seg_index].name} marked ready "
                               f"after its bucket {self.seg_bucket[seg_index]} was launched")
        self._active = True
        if self._stages:
            for si in self._seg_stages[seg_index]:
                self._stage_cnt[si] += 1
            self._stage_in_order()
        b = self.seg_bucket[seg_index]
        self._ready_cnt[b] += 1
        n = self.buckets[b].seg_hi - self.buckets[b].seg_lo
        if self._ready_cnt[b] == n:
            self._ready[b] = True
            self._launch_in_order()

    def _launch_in_order(self) -> None:
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def _event(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _flush_splitk(self) -> None:
        """Run the split-K reduces the fused blocks deferred (ops/block.py _deferred_reduce,
        csrc/gemm.hip splitk_flush) before anything reads the arena."""
        if self.device.type == "cuda":
            from ..ops._ext import is_loaded, load
            if is_loaded():
                load().splitk_flush(self.arena.grad)

    def _launch(self, bi: int) -> None:
        self._flush_splitk()
        b = self.buckets[bi]
        codec = self.codecs[bi]
        g = self.arena.grad[b.start:b.end]
        e = self.ef[b.start:b.end] if self.ef is not None else None
        side = self._side
        if side is not None and not self._graph_overlap and \
                torch.cuda.is_current_stream_capturing():
            # inside a captured step the side-stream branch costs more than it hides (ResNet-50,
            # 1 GPU: 24.67 ms/step with it, 24.17 ms without; profiles/r2_graph_overlap_ab.log):
            # the bucket is compressed and exchanged inline on the compute stream
            side = None
        # "comm" mode inside a capture: compress on the compute stream, fork before the collective
        late = side is not None and self._comm_only and torch.cuda.is_current_stream_capturing()
        if self._stages:
            # slices of parameters that got no gradient (or every slice, after backward: sync_now)
            # are staged now — on the compute stream's side of the fork below, in order
            self._stage_in_order(force=True)
        ready = None

        def fork():
            # the event must outlive the side stream's wait on it: it stays in _pending until
            # finish() (a HIP event destroyed while a queued wait still references it faulted
            # the VGG-16 run: hipErrorIllegalAddress, profiles/r2_vgg_fault.md)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            side.wait_event(ev)
            return ev

        if side is not None and not late:
            ready = fork()
        with torch.cuda.stream(side) if side is not None and not late else \
                contextlib.nullcontext():
            t0 = self._event() if self.timing else None
            if self.lr_scaled:
                e.mul_(self._lr_ratio)                   # residual re-expressed at this step's LR
            u = None
            sel = codec.inner if isinstance(codec, DenseWrap) else codec
            if self._stages:
                sel._staged = True
            if self.mom is not None:
                u = self.mom[b.start:b.end]
                if self._mc_fusable(bi, sel, g):
                    # velocity update in the first select pass (compress.hip McArgs)
                    _, wd = self._mc_plan(bi)
                    p = self.arena.param_buf[b.start:b.end] if wd is not None else None
                    sel.mc_fuse = (p, wd, float(self.mc), float(self._mc_wmul))
                else:
                    self._mc_prologue(bi, g, u)          # velocity; the residual accumulates it
                sel.mc_mom = u                           # masked by the select kernels
            send = codec.compress(g, e, self.step)
            sel._staged = False
            if u is not None:
                sel.mc_mom = None
                sel.mc_fuse = None
                if not getattr(sel, "mc_fused", False):  # no selection: sent <=> residual 0
                    self._mc_mask(u, e)
            t1 = self._event() if self.timing else None
            self._payload += codec.last_payload_bytes
        if late:
            ready = fork()
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            if codec.collective == "all_reduce":
                work = (self._native.all_reduce(send) if self._native is not None
                        else comm.all_reduce(send, self.pg))
                recv = None
            elif codec.collective == "quant_rs":
                # quantised reduce-scatter: code all-to-all, shard dequant-sum, bf16 all-gather
                # (codecs.py QuantRSCodec); stream-ordered on the native communicator
                recv = codec.exchange(self._native if self._native is not None
                                      else comm.C10dP2P(self.pg), send)
                work = comm._Done()
            elif self.world == 1:
                recv, work = None, comm._Done()       # (one rank: decode straight from send)
            else:
                recv = codec.recv_buffer(send)
                work = (self._native.all_gather(recv, send) if self._native is not None
                        else comm.all_gather(recv, send, self.pg))
            tx = None
            if side is not None and self._stream_waitable:
                # RCCL: wait() only orders the side stream after the collective (no host block),
                # so the exchange itself can be timed and `done` covers compress + exchange
                work.wait()
                tx = self._event() if self.timing else None
            done = None
            if side is not None:
                done = torch.cuda.Event()
                done.record(side)
        self._pending.append((bi, work, send, recv, (t0, t1, tx), done, ready))

    @staticmethod
    def _mc_mask(u: torch.Tensor, e: torch.Tensor) -> None:
        from ..ops._ext import ops_for
        lib = ops_for(u)
        if lib is not None:
            lib.mc_mask(u, e)
        else:
            u.mul_(e != 0)

    def finish(self) -> None:
        """Launch buckets that never became ready (unused params keep zero grads), wait for every
        collective and decode into the arena."""
        self._flush_splitk()
        if self.device.type == "cuda":
            from ..ops import block as _block
            _block.end_step()
        for i in self._no_zero:
            if self._claims[i] == 0:     # (not zeroed by begin_step and not written this step)
                self.arena.grad_view(self.arena.segments[i]).zero_()
        for i in range(self._next, len(self.buckets)):
            self._ready[i] = True
        self._launch_in_order()
        rec = []
        fused = False
        hold = list(self._stage_events)          # events some stream still waits on (see below)
        for bi, work, send, recv, (t0, t1, tx), done, ready in self._pending:
            hold += [e for e in (ready, done) if e is not None]
            work.wait()
            if done is not None:                 # decode on the compute stream after the side
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(done)
                for t in (send, recv):           # allocated on the side stream, used here
                    if t is not None:
                        t.record_stream(cur)
            t2 = self._event() if self.timing else None
            b = self.buckets[bi]
            if bi in self._sgd_buckets:
                if not fused:
                    self._sgd.mark_fused_update(self._sgd.fused_hyper())
                    fused = True
                self.codecs[bi].decompress_sgd(send, recv, self._sgd_args(bi))
            else:
                self.codecs[bi].decompress(send, recv, self.arena.grad[b.start:b.end])
            if self.timing:
                rec.append((bi, t0, t1, tx, t2, self._event()))
        self._pending = []
        if self._dstep is not None and any(c.uses_step for c in self.codecs):
            from ..ops._ext import ops_for
            lib = ops_for(self._dstep)
            if lib is not None:
                lib.step_bump(self._dstep)          # (a native kernel, no ATen elementwise add)
            else:
                self._dstep.add_(1)
        if not torch.cuda.is_available() or not torch.cuda.is_current_stream_capturing():
            self.heartbeat()
        if hold and not torch.cuda.is_current_stream_capturing():
            # (under HIP-graph capture the event record / wait pairs become graph edges: there is
            # nothing to keep alive, and an event query would invalidate the capture)
            # Keep the cross-stream events alive until a fence on the compute stream, recorded
            # after every wait on them, has completed: destroying a HIP event while a queued
            # stream wait still references it is what faulted the VGG-16 run
            # (hipErrorIllegalAddress; profiles/r2_vgg_fault.md).
            fence = torch.cuda.Event()
            fence.record(torch.cuda.current_stream(self.device))
            self._retired = [(f, h) for f, h in self._retired if not f.query()]
            self._retired.append((fence, hold))
        if self.timing:
            self._last_events = rec
        self.step += 1
        self.stats.steps += 1
        self.stats.payload_bytes = self._payload
        self._active = False
        self.all_reduced_last = True

    def read_overflow(self) -> int:
        """Cumulative count of elements the compression rule selected that did not fit the
        payload (they stayed in the error-feedback residual, or were dropped without EF): Top-K
        ties beyond ``tie_slack``, threshold hits beyond the fixed sparse capacity. Synchronises;
        call at logging time. Also kept in ``stats.overflow``."""
        if self._overflow is None:
            return 0
        self.stats.overflow = int(self._overflow.item())
        return self.stats.overflow

    def heartbeat(self) -> None:
        """Mark the end of a step for the communicator watchdog (no-op without one; never
        inside a graph capture — a replayed step is marked by StepGraph after the replay)."""
        if self._watch is not None:
            self._watch.mark()

    def sync_now(self) -> None:
        """Post-backward path: copy any foreign ``.grad`` into the arena, then sync every bucket."""
        self.arena.gather_grads()
        self._reset_state()
        for i in range(len(self.buckets)):
            self._ready[i] = True
        self._launch_in_order()
        self.finish()

    def set_step(self, step: int) -> None:
        """Set the step counter (host and device), e.g. when a checkpoint is restored."""
        self.step = int(step)
        if self._dstep is not None:
            self._dstep.fill_(self.step)

    def graph_safe(self) -> bool:
        """Whether a whole step through this engine can be captured as one HIP graph and
        replayed: every codec is sync-free and step-invariant, and per-bucket timing is off."""
        if comm.is_dist() and self._native is None:
            # gloo collectives run on the host; c10d RCCL calls leave Work events for the
            # ProcessGroup watchdog, which may query one recorded inside the capture and abort
            # (hipErrorCapturedEvent): capture only with the native communicator
            return False
        return (self.device.type == "cuda" and not self.timing and
                all(bool(c.graph_safe) for c in self.codecs))

    def read_timings(self) -> List[dict]:
        """Per-bucket µs of the last step (HIP events): ``compress_us`` (select + pack on the side
        stream), ``exchange_us`` (compress end → collective complete; RCCL, whose wait() is
        stream-ordered: includes queueing behind earlier buckets' collectives), ``idle_us``
        (exchange done → the compute stream decodes it, i.e. the rest of the backward pass the
        exchange was hidden behind) and ``decode_us``. Without a stream-waitable backend (gloo,
        world 1) ``exchange_us`` is None and ``idle_us`` spans compress end → decode.
        Synchronises; call outside the hot loop."""
        out = []
        for bi, t0, t1, tx, t2, t3 in getattr(self, "_last_events", []):
            t3.synchronize()
            out.append({"bucket": bi, "compress_us": 1e3 * t0.elapsed_time(t1),
                        "exchange_us": 1e3 * t1.elapsed_time(tx) if tx is not None else None,
                        "idle_us": 1e3 * (tx if tx is not None else t1).elapsed_time(t2),
                        "decode_us": 1e3 * t2.elapsed_time(t3)})
        return out

    # ----------------------------------------------------------------- introspection
    def describe(self) -> str:
        cs = {}
        for c in self.codecs:
            cs[c.name] = cs.get(c.name, 0) + 1
        return (f"GradSyncEngine(mode={self.mode}, method={self.method}, world={self.world}, "
                f"buckets={len(self.buckets)}, codecs={cs}, ef={self.ef is not None}, "
                f"{self.arena})")
