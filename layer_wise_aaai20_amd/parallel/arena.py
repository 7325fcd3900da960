"""Flat parameter / gradient arenas and the bucket layout built on them.

Replaces two things in the reference:
  * the per-step ``torch.cat`` of every gradient in entire-model mode and the views written back
    afterwards (``CIFAR10/core.py:230-236, 292-301``), and
  * the private c10d ``_dist_bucket_tensors`` bucketing of the vendored DDPs
    (``IMAGENET/training/ddp.py:238-241``, ``sparsified_ddp.py:232-254``).

Every trainable parameter's ``.grad`` is a strided view into ONE contiguous fp32 buffer, laid out in
*reverse registration order* (the order autograd produces gradients in), so that

  * layer-wise compression works on per-parameter *segments* of that buffer,
  * entire-model compression works on the whole buffer with no copy, and
  * a communication bucket is just a contiguous slice ``[start, end)`` of it.

Parameters themselves can optionally also live in a flat arena (``flat_params=True``), which lets
the fused SGD kernel update the whole model in one launch.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from ..ops._ext import h16

ALIGN = 64  # elements: keeps every segment 256-B aligned for 16-B vector loads


def _align(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


def _dense_strided_view(buf: torch.Tensor, offset: int, like: torch.Tensor) -> torch.Tensor:
    """A view of ``buf[offset:offset+numel]`` with ``like``'s shape and dense memory format
    (so a channels_last conv weight gets a channels_last gradient view)."""
    stride = torch.empty_like(like, device="meta", memory_format=torch.preserve_format).stride()
    return buf.as_strided(like.shape, stride, offset)


@dataclass
class Segment:
    index: int              # position in arena order
    name: str
    numel: int
    offset: int             # element offset into the arena
    param: torch.nn.Parameter = field(repr=False, default=None)


class GradArena:
    """Owns the flat gradient buffer and the parameter→segment map.

    ``params`` is taken in registration order; the arena order is reversed. Parameters that do not
    require grad are skipped (the reference buckets only ``requires_grad`` params,
    ``sparsified_ddp.py:244``).
    """

    def __init__(self, named_params: Sequence, device=None, dtype=torch.float32,
                 flat_params: bool = False, align: int = ALIGN):
        named = [(n, p) for n, p in named_params if p.requires_grad]
        if not named:
            raise ValueError("GradArena needs at least one trainable parameter")
        self.device = torch.device(device) if device is not None else named[0][1].device
        self.dtype = dtype
        self.align = align
        order = list(reversed(named))
        self.segments: List[Segment] = []
        off = 0
        for i, (name, p) in enumerate(order):
            self.segments.append(Segment(i, name, p.numel(), off, p))
            off += _align(p.numel(), align)
        self.numel = off
        self.grad = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.by_param: Dict[int, Segment] = {id(s.param): s for s in self.segments}
        self.flat_params = flat_params
        self.param_buf: Optional[torch.Tensor] = None
        if flat_params:
            self._flatten_params()
        self.attach_grads()

    # ------------------------------------------------------------------ views
    def grad_view(self, seg: Segment) -> torch.Tensor:
        return _dense_strided_view(self.grad, seg.offset, seg.param)

    def flat_grad_of(self, seg: Segment) -> torch.Tensor:
        return self.grad[seg.offset: seg.offset + seg.numel]

    def attach_grads(self) -> None:
        """(Re)point every ``param.grad`` at its arena view.

        Autograd's AccumulateGrad adds in place into an existing ``.grad`` of matching layout, so
        once attached the backward pass writes straight into the arena.
        """
        for s in self.segments:
            v = self.grad_view(s)
            if s.param.grad is not None and s.param.grad.data_ptr() != v.data_ptr():
                v.copy_(s.param.grad)
            s.param.grad = v

    def grads_attached(self) -> bool:
        for s in self.segments:
            g = s.param.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + s.offset * self.grad.element_size():
                return False
        return True

    def gather_grads(self) -> None:
        """Copy detached grads into the arena (used when a caller replaced ``.grad``)."""
        for s in self.segments:
            g = s.param.grad
            v = self.grad_view(s)
            if g is None:
                v.zero_()
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
        self.attach_grads()

    def zero_(self) -> None:
        self.grad.zero_()

    def zero_except(self, keep) -> None:
        """Zero the gradient arena but for the segments in ``keep`` (one fill per gap)."""
        lo = 0
        for s in sorted((self.segments[i] for i in keep), key=lambda s: s.offset):
            if s.offset > lo:
                self.grad[lo:s.offset].zero_()
            lo = s.offset + s.numel
        if lo < self.numel:
            self.grad[lo:].zero_()

    def _flatten_params(self) -> None:
        self.param_buf = torch.zeros(self.numel, dtype=self.segments[0].param.dtype,
                                     device=self.device)
        for s in self.segments:
            v = _dense_strided_view(self.param_buf, s.offset, s.param.data)
            v.copy_(s.param.data)
            s.param.data = v

    # ------------------------------------------------------------------ bf16 weight mirror
    def refresh_bf16(self) -> None:
        """One cast of the whole flat fp32 parameter buffer into a bf16 mirror (instead of one
        cast kernel per layer per forward). ``bf16_of(p)`` hands out views of it while the
        parameters are unchanged since the refresh — tracked by version counters: the flat
        buffer's (the fused optimizer writes through it) and each parameter's own (in-place
        updates such as ``load_state_dict``), so a stale mirror is never used."""
        if self.param_buf is None:
            return
        if getattr(self, "param_bf16", None) is None:
            self.param_bf16 = torch.empty(self.numel, dtype=h16(), device=self.device)
            for s in self.segments:
                view = _dense_strided_view(self.param_bf16, s.offset, s.param.data)
                s.param._lw_bf16_of = (lambda v=view, s=s: v if self.bf16_valid(s) else None)
        if getattr(self, "_bf16_by_sgd", False) and self._bf16_current():
            return                 # the fused SGD kernel already wrote it (FlatSGD)
        self.param_bf16.copy_(self.param_buf)
        self._bf16_by_sgd = False
        self._bf16_version = self.param_buf._version
        self._bf16_pver = [s.param._version for s in self.segments]

    def mark_bf16_fresh(self) -> None:
        """The optimizer kernel has just written the mirror along with the fp32 parameters."""
        self._bf16_by_sgd = True
        self._bf16_version = self.param_buf._version
        self._bf16_pver = [s.param._version for s in self.segments]

    def _bf16_current(self) -> bool:
        return (getattr(self, "_bf16_version", None) == self.param_buf._version and
                self._bf16_pver == [s.param._version for s in self.segments])

    def bf16_valid(self, seg: Segment) -> bool:
        return (getattr(self, "_bf16_version", None) == self.param_buf._version and
                self._bf16_pver[seg.index] == seg.param._version)

    def layer_sizes(self) -> List[int]:
        return [s.numel for s in self.segments]

    def __repr__(self) -> str:
        return (f"GradArena(segments={len(self.segments)}, numel={self.numel}, "
                f"bytes={self.numel * self.grad.element_size() / 2**20:.1f} MiB)")


@dataclass
class Bucket:
    index: int
    seg_lo: int              # first segment (arena order)
    seg_hi: int              # one past last segment
    start: int               # arena element range [start, end)
    end: int

    @property
    def numel(self) -> int:
        return self.end - self.start


def plan_buckets(arena: GradArena, mode: str, cap_bytes: int,
                 first_bucket_bytes: Optional[int] = None,
                 last_bucket_bytes: Optional[int] = None) -> List[Bucket]:
    """Contiguous buckets over the arena.

    ``mode == 'entiremodel'`` → one bucket, one segment spanning everything (the compressor sees the
    concatenated model, ``core.py:227-236``).  ``layerwise``/``none`` → consecutive segments are
    grouped until ``cap_bytes`` (of fp32 gradient) is reached; a bucket never splits a segment. A
    smaller first bucket lets communication start earlier in backward (the last layers' grads come
    first). A smaller LAST bucket shortens the tail: the first layers' gradients are the last to be
    computed, so that bucket's compression and exchange cannot overlap any backward work — its
    size is what the step waits for after the backward pass.
    """
    segs = arena.segments
    if mode == "entiremodel":
        return [Bucket(0, 0, len(segs), 0, arena.numel)]
    esize = arena.grad.element_size()
    # tail: whole segments from the end until last_bucket_bytes (never all of them)
    tail = len(segs)
    if last_bucket_bytes:
        acc = 0
        while tail > 1 and acc < last_bucket_bytes:
            tail -= 1
            acc += segs[tail].numel * esize
        if tail == 0:
            tail = len(segs)
    buckets: List[Bucket] = []
    lo = 0
    acc = 0
    cap = first_bucket_bytes if first_bucket_bytes else cap_bytes
    for i in range(tail):
        acc += segs[i].numel * esize
        if acc >= cap and i + 1 < tail:
            buckets.append(Bucket(len(buckets), lo, i + 1, segs[lo].offset,
                                  segs[i + 1].offset))
            lo, acc, cap = i + 1, 0, cap_bytes
    end = segs[tail].offset if tail < len(segs) else arena.numel
    buckets.append(Bucket(len(buckets), lo, tail, segs[lo].offset, end))
    if tail < len(segs):
        buckets.append(Bucket(len(buckets), tail, len(segs), segs[tail].offset, arena.numel))
    return buckets
