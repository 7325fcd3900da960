"""Data-parallel wrappers built on :class:`GradSyncEngine`.

* :class:`CompressedDDP` — bucketed, backward-overlapped DP with any of the reference compressors
  in layer-wise or entire-model mode, optional error feedback for every method.
* :func:`DistributedDataParallel` — the uncompressed bucketed DDP (DP-3, the vendored
  ``IMAGENET/training/ddp.py:19-489``).
* :func:`RandomKSparsifiedDDP` — shared-seed Random-K with error feedback and index-free payloads
  (DP-4, ``IMAGENET/training/sparsified_ddp.py:20-495``).

Start-up: module state (parameters AND buffers) is broadcast from rank 0, as in ``ddp.py:190-194``;
unlike the reference's CIFAR path every mode starts from identical replicas.
Buffers (BatchNorm running statistics) follow rank 0 when ``broadcast_buffers`` is set. The
reference re-broadcasts them before every forward (``ddp.py:361-386``); their training-mode
readers never look at them (BatchNorm normalises with batch statistics), and rank 0 — the source —
never receives, so its buffers evolve identically either way. ``buffer_sync="lazy"`` (default)
therefore broadcasts them, as one coalesced message, only where they are read: the first
eval-mode forward after training, :meth:`sync_buffers` (the trainers call it before evaluation
and checkpoints, on every rank) — the values there are exactly the reference's. A captured
training step then carries no per-step broadcast collective. ``buffer_sync="step"`` keeps the
reference's per-forward broadcast.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
from torch import nn

from . import comm
from .engine import GradSyncEngine


class CompressedDDP(nn.Module):
    def __init__(self, module: nn.Module, compress: str = "layerwise", method="Topk", K=0.001,
                 V=1e-3, qstates=255, error_feedback: bool = False, bucket_cap_mb: float = 25.0,
                 first_bucket_mb: Optional[float] = None, process_group=None,
                 broadcast_buffers: bool = True, wire: str = "auto", seed: int = 2147483647,
                 flat_params: bool = True, check_reduction: bool = True, device_ids=None,
                 output_device=None, dim: int = 0, timing: bool = False,
                 bf16_weights: bool = True, world_size: Optional[int] = None,
                 dense_below: int = 0, momentum_correction: float = 0.0,
                 ef_lr_scaled: bool = False, buffer_sync: str = "lazy"):
        super().__init__()
        if buffer_sync not in ("lazy", "step"):
            raise ValueError(f"buffer_sync={buffer_sync!r}: expected 'lazy' or 'step'")
        self.buffer_sync = buffer_sync
        self._buf_dirty = False
        self.module = module
        self.bf16_weights = bf16_weights and flat_params
        self.process_group = process_group
        self.broadcast_buffers = broadcast_buffers
        self.check_reduction = check_reduction
        self.dim = dim
        if device_ids is not None and len(device_ids) > 1:
            raise RuntimeError("one process per GPU: pass at most one device id")
        # identical replicas and an agreed RNG seed on every rank
        comm.broadcast_coalesced(list(module.state_dict().values()), 0, process_group)
        if comm.is_dist() and comm.world_size(process_group) > 1:
            s = torch.tensor([seed], dtype=torch.int64,
                             device=next(module.parameters()).device)
            comm.broadcast_coalesced([s], 0, process_group)
            seed = int(s.item())
        self.engine = GradSyncEngine(module.named_parameters(), mode=compress, method=method, K=K,
                                     V=V, qstates=qstates, error_feedback=error_feedback,
                                     bucket_cap_mb=bucket_cap_mb,
                                     first_bucket_mb=first_bucket_mb, wire=wire, seed=seed,
                                     process_group=process_group, flat_params=flat_params,
                                     timing=timing, world_size=world_size,
                                     dense_below=dense_below,
                                     momentum_correction=momentum_correction,
                                     ef_lr_scaled=ef_lr_scaled)
        self._buffers_list = self._flatten_buffers(module) if broadcast_buffers else []
        self._bcast_events = []          # (ready, done) of the last buffer broadcasts
        self._hooks = []
        self._register_hooks()
        self._callback_queued = False

    @staticmethod
    def _flatten_buffers(module: nn.Module):
        """Re-point every floating-point buffer (BN running statistics) at a view of one flat
        tensor per (dtype, device), so the per-forward buffer broadcast (``ddp.py:361-386``) is a
        single in-place collective with no gather/scatter copies. Integer buffers already shared
        through a flat base (``share_bn_counters``) are broadcast via that base."""
        groups, ints, seen = {}, [], set()
        for mod in module.modules():
            for name, b in mod._buffers.items():
                if b is None:
                    continue
                if b.is_floating_point():
                    groups.setdefault((b.dtype, b.device), []).append((mod, name, b))
                elif b.dtype in (torch.int64, torch.int32):
                    base = b._base if b._base is not None else b
                    if id(base) not in seen:
                        seen.add(id(base))
                        ints.append(base)
        flats = []
        for (dtype, dev), items in groups.items():
            flat = torch.empty(sum(b.numel() for _, _, b in items), dtype=dtype, device=dev)
            off = 0
            for mod, name, b in items:
                n = b.numel()
                v = flat[off:off + n].view_as(b)
                v.copy_(b)
                mod._buffers[name] = v
                off += n
            flats.append(flat)
        return flats + ints

    # ------------------------------------------------------------------ hooks
    def _register_hooks(self) -> None:
        for seg in self.engine.arena.segments:
            p = seg.param
            hook = self._make_hook(seg.index)
            self._hooks.append(p.register_post_accumulate_grad_hook(hook))
            # fused ops (ops/block.py) write this parameter's gradient straight into its arena
            # view and then call the same hook, bypassing AccumulateGrad
            p._lw_grad_ready = hook
            # may a fused op overwrite (not accumulate into) this gradient? (engine.claim_overwrite)
            p._lw_grad_overwrite = (lambda i=seg.index: self.engine.claim_overwrite(i))

    def _make_hook(self, seg_index: int):
        engine = self.engine
        arena = engine.arena
        seg = arena.segments[seg_index]

        def hook(p):
            v = arena.grad_view(seg)
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                # someone replaced .grad (e.g. zero_grad(set_to_none=True)): fold it back in
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
            engine.mark_ready(seg_index)
        return hook

    def _finish(self) -> None:
        self._callback_queued = False
        self.engine.finish()

    # ------------------------------------------------------------------ module API
    def sync_buffers(self) -> None:
        """Collective: give every rank rank 0's buffers now (a no-op when nothing changed since
        the last sync, on one rank, or with ``broadcast_buffers=False``). Call on every rank."""
        if self._bcast_events:
            torch.cuda.current_stream(self.engine.device).wait_event(self._bcast_events[-1][1])
        if self._buf_dirty and self.broadcast_buffers and self._buffers_list:
            comm.broadcast_coalesced(self._buffers_list, 0, self.process_group,
                                     native=self.engine._native)
        self._buf_dirty = False

    def forward(self, *inputs, **kwargs):
        if not self.training:
            self.sync_buffers()             # (evaluation reads the broadcast running statistics)
            return self.module(*inputs, **kwargs)
        if self.check_reduction and self.engine._active:
            raise RuntimeError("Not all gradients have been reduced from the backward of the "
                               "previous iteration (ddp.py:312-327 check_reduction).")
        if self.buffer_sync == "lazy":
            # no collective in the training step: broadcast where the buffers are read
            self._buf_dirty = self._buf_dirty or (self.broadcast_buffers and
                                                  bool(self._buffers_list) and
                                                  comm.world_size(self.process_group) > 1)
            self.engine.begin_step()
            if self.bf16_weights and self.engine.arena.device.type == "cuda":
                self.engine.arena.refresh_bf16()
            return self.module(*inputs, **kwargs)
        side = self._buffer_side()
        if side is not None:
            # the buffers were broadcast on the side stream right after the previous forward,
            # overlapped with its backward: only their use waits for it
            if self._bcast_events:
                torch.cuda.current_stream(self.engine.device).wait_event(self._bcast_events[-1][1])
        elif self.broadcast_buffers and self._buffers_list:
            comm.broadcast_coalesced(self._buffers_list, 0, self.process_group,
                                     native=self.engine._native)
        self.engine.begin_step()
        if self.bf16_weights and self.engine.arena.device.type == "cuda":
            self.engine.arena.refresh_bf16()
        out = self.module(*inputs, **kwargs)
        if side is not None:
            self._broadcast_after_forward(side)
        return out

    def _buffer_side(self):
        """The side stream the buffer broadcast runs on, or None (eager broadcast at forward)."""
        eng = self.engine
        if not (self.broadcast_buffers and self._buffers_list) or eng._native is None or \
                eng._side is None or eng.world <= 1:
            return None
        if eng.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            # a captured step broadcasts inline at the forward's start, as the reference: a
            # side-stream broadcast would only be joined by the NEXT forward, i.e. never inside
            # this capture — an unjoined branch at capture end crashed (SIGSEGV in capture_end)
            # or hung the 2-rank captured training tests
            return None
        return eng._side

    def _broadcast_after_forward(self, side) -> None:
        """The reference broadcasts the buffers (BN running statistics) at the start of every
        forward (``ddp.py:361-386``). No kernel touches them between the end of one forward and
        the start of the next, so broadcasting right after the forward sends the same values;
        done on the side stream, the broadcast overlaps this step's backward instead of
        delaying the next forward. The events stay alive for a few steps (a HIP event
        destroyed while a queued wait references it faults: profiles/r2_vgg_fault.md)."""
        cur = torch.cuda.current_stream(self.engine.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        side.wait_event(ready)
        with torch.cuda.stream(side):
            comm.broadcast_coalesced(self._buffers_list, 0, self.process_group,
                                     native=self.engine._native)
            done = torch.cuda.Event()
            done.record(side)
        self._bcast_events = (self._bcast_events + [(ready, done)])[-4:]

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Keep ``.grad`` as arena views: zeroing means clearing the arena."""
        self.engine.begin_step()

    @property
    def arena(self):
        return self.engine.arena

    def sync_stats(self):
        return self.engine.stats

    # checkpoint extras: per-rank error-feedback residuals and the step counter (extra keys that
    # reference readers ignore; SURVEY.md §5 checkpoint row)
    def compression_state(self, dst: int = 0) -> dict:
        """Collective (call on every rank): the step counter and EVERY rank's error-feedback
        residual, ``ef_per_rank[r]`` = rank r's buffer (each rank's residual is its own
        compression error, so restoring rank 0's everywhere would bias the resumed run).
        The residuals are gathered to the checkpoint writer ``dst`` only (group rank); on every
        other rank ``ef_per_rank`` is None, so no rank but the writer holds world x |arena|."""
        e = self.engine
        st = {"step": e.step, "world": e.world, "ef_per_rank": None}
        if e.ef is not None:
            ef = e.ef.detach().contiguous()
            if e.world > 1 and dist.is_available() and dist.is_initialized():
                mine = e.rank == dst
                parts = [torch.empty_like(ef) for _ in range(e.world)] if mine else None
                gdst = dist.get_global_rank(e.pg, dst) if e.pg is not None else dst
                dist.gather(ef, parts, dst=gdst, group=e.pg)
                if mine:
                    st["ef_per_rank"] = torch.stack([p.cpu() for p in parts])
            else:
                st["ef_per_rank"] = ef.clone()[None].cpu()
        return st

    def load_compression_state(self, st: dict) -> None:
        """Each rank restores its own residual; a checkpoint from a different world size (or
        one without residuals) restarts error feedback from zero, with a warning."""
        e = self.engine
        e.set_step(int(st.get("step", 0)))
        if e.ef is None:
            return
        per = st.get("ef_per_rank")
        if per is not None and per.shape[0] == e.world and per.shape[1] == e.ef.numel():
            e.ef.copy_(per[e.rank].to(e.ef.device))
        elif st.get("ef") is not None and e.world == 1:          # single-rank legacy layout
            e.ef.copy_(st["ef"])
        else:
            import warnings
            warnings.warn("checkpoint has no error-feedback residuals for this world size: "
                          "restarting them from zero")
            e.ef.zero_()

    def extra_repr(self) -> str:
        return self.engine.describe()


def DistributedDataParallel(module, device_ids=None, output_device=None, dim=0,
                            broadcast_buffers=True, process_group=None, bucket_cap_mb=25,
                            check_reduction=False, **kw) -> CompressedDDP:
    """Uncompressed bucketed DDP (DP-3): reverse-order 25 MB buckets, overlapped all-reduce."""
    return CompressedDDP(module, compress="none", method="none", bucket_cap_mb=bucket_cap_mb,
                         process_group=process_group, broadcast_buffers=broadcast_buffers,
                         check_reduction=check_reduction, device_ids=device_ids, **kw)


def RandomKSparsifiedDDP(module, device_ids=None, output_device=None, dim=0,
                         broadcast_buffers=True, process_group=None, bucket_cap_mb=25,
                         check_reduction=False, randk=1, seed=2147483647, **kw) -> CompressedDDP:
    """Shared-seed Random-K with error feedback, index-free payloads (DP-4)."""
    if randk >= 1:
        return DistributedDataParallel(module, device_ids, output_device, dim, broadcast_buffers,
                                       process_group, bucket_cap_mb, check_reduction, **kw)
    return CompressedDDP(module, compress="layerwise", method="Randomk", K=randk,
                         error_feedback=True, bucket_cap_mb=bucket_cap_mb, seed=seed,
                         process_group=process_group, broadcast_buffers=broadcast_buffers,
                         check_reduction=check_reduction, device_ids=device_ids, wire="indexfree",
                         **kw)
