"""Fused SGD over the flat parameter / gradient arenas (one HIP launch per step).

Drop-in for the ``torch.optim.SGD`` the reference builds in both workloads
(``CIFAR10/torch_backend.py:142-143``, ``IMAGENET/training/train_imagenet_nv.py:188-191``):
same hyper-parameters, same param-group API (the LR ``Scheduler`` writes ``param_groups[i]['lr']``,
``--no-bn-wd`` gives BN parameters their own ``weight_decay=0`` group, ``experimental_utils.py``),
and a ``state_dict`` in torch.optim.SGD's format, so checkpoints stay compatible
(``train_imagenet_nv.py:663-669``). Internally every momentum buffer is a view into one flat buffer
laid out like the parameter arena, and the update (grad unscale, weight decay, momentum,
Nesterov) is one kernel (``csrc/optim.hip``).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
from torch.optim import Optimizer

from ..compress.plan import SegPlan
from ..parallel.arena import _dense_strided_view
from ..ops._ext import ops_for


class FlatSGD(Optimizer):
    def __init__(self, params, arena, lr: float = 0.0, momentum: float = 0.0,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                 grad_scale: float = 1.0):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults)
        self.arena = arena
        if arena.param_buf is None:
            raise ValueError("FlatSGD needs an arena built with flat_params=True")
        self.grad_scale = grad_scale
        segs = arena.segments
        self._seg_of = {id(s.param): s.index for s in segs}
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) not in self._seg_of:
                    raise ValueError("every optimised parameter must live in the arena")
        self.plan = SegPlan([s.offset for s in segs], [s.numel for s in segs])
        self.buf = torch.zeros_like(arena.param_buf)
        self._first = True
        self._wd_cache = None
        # graph mode (train/imagenet.py GraphedStep): lr / grad_scale live in a device tensor the
        # kernel reads, written by load_hyper() outside the captured graph before each replay
        self.device_hyper = False
        self._hyper = None
        self._hyper_host = None
        # segments a GradSyncEngine updates itself, fused with their decode (set_fused_sgd), and
        # the hyper-parameters that update used (None: no fused update since the last step)
        self._exclude = frozenset()
        self._sub = None
        self._fused_mark = None

    # torch.optim.SGD-compatible state: momentum_buffer views into the flat buffer
    def _bind_state(self):
        for g in self.param_groups:
            if g["momentum"] == 0:
                continue
            for p in g["params"]:
                s = self.arena.segments[self._seg_of[id(p)]]
                self.state[p]["momentum_buffer"] = _dense_strided_view(self.buf, s.offset, p)

    def _seg_wd(self, device):
        key = tuple(float(g["weight_decay"]) for g in self.param_groups)
        if self._wd_cache is None or self._wd_cache[0] != key:
            wd = np.zeros(len(self.arena.segments), dtype=np.float32)
            for g in self.param_groups:
                for p in g["params"]:
                    wd[self._seg_of[id(p)]] = g["weight_decay"]
            self._wd_cache = (key, torch.from_numpy(wd).to(device))
        return self._wd_cache[1]

    def exclude_segments(self, segs) -> None:
        """Leave arena segments ``segs`` to the gradient engine's fused decode-and-step
        (``GradSyncEngine.set_fused_sgd``): :meth:`step` updates the others only."""
        self._exclude = frozenset(int(i) for i in segs)
        self._sub = None

    def _tables(self, device):
        """(plan tables, per-table-segment weight decay) over the segments step() updates."""
        wd = self._seg_wd(device)
        if not self._exclude:
            return self.plan.all_large_tables(device), wd
        if self._sub is None or self._sub[0] is not wd:
            keep = [s for s in self.arena.segments if s.index not in self._exclude]
            if not keep:
                self._sub = (wd, None, None)
            else:
                plan = SegPlan([s.offset for s in keep], [s.numel for s in keep])
                idx = torch.tensor([s.index for s in keep], dtype=torch.long, device=device)
                self._sub = (wd, plan.all_large_tables(device), wd[idx].contiguous())
        return self._sub[1], self._sub[2]

    def fused_hyper(self) -> tuple:
        """What a fused decode-and-step reads: (lr, momentum, dampening, nesterov, first-step
        flag, grad_scale, weight decays)."""
        return (float(self._uniform("lr")), float(self._uniform("momentum")),
                float(self._uniform("dampening")), bool(self._uniform("nesterov")),
                bool(self._first), float(self.grad_scale),
                tuple(float(g["weight_decay"]) for g in self.param_groups))

    def mark_fused_update(self, hyper: tuple) -> None:
        """Called by the gradient engine when backward has already updated the excluded segments
        (``GradSyncEngine.set_fused_sgd``). A second backward before :meth:`step` would update
        them twice — the fused contract is one backward, then one step."""
        if self._fused_mark is not None:
            raise RuntimeError("a second backward ran before optimizer.step(): the segments "
                               "updated inside backward (GradSyncEngine.set_fused_sgd) would be "
                               "stepped twice; call step() after every backward, or build the "
                               "trainer with fused_sgd=False for gradient accumulation")
        self._fused_mark = hyper

    def _uniform(self, k):
        vals = {g[k] for g in self.param_groups}
        if len(vals) != 1:
            raise ValueError(f"FlatSGD needs a single {k} across param groups, got {vals}")
        return vals.pop()

    def load_hyper(self) -> None:
        """Write the current (lr, grad_scale) into the device tensor a captured step reads (a
        stream-ordered fill per value that changed — usually the LR alone; call outside graph
        capture)."""
        vals = (float(self._uniform("lr")), float(self.grad_scale))
        if self._hyper is None:
            self._hyper = torch.empty(2, dtype=torch.float32, device=self.arena.param_buf.device)
            self._hyper_host = None
        old = self._hyper_host or (None, None)
        for i in (0, 1):
            if vals[i] != old[i]:
                self._hyper[i].fill_(vals[i])
        self._hyper_host = vals

    def lr_device(self) -> torch.Tensor:
        """The current LR as a 1-element device tensor (the one a captured step reads; refreshed
        by load_hyper, which the trainers call before every step)."""
        if self._hyper is None:
            self.load_hyper()
        return self._hyper[:1]

    def graph_signature(self) -> tuple:
        """Everything a captured SGD launch bakes in as kernel arguments (lr and grad_scale are
        read from device memory instead): a change means the step must be re-captured."""
        return (float(self._uniform("momentum")), float(self._uniform("dampening")),
                bool(self._uniform("nesterov")), self._first,
                tuple(float(g["weight_decay"]) for g in self.param_groups))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self._exclude:
            # the segments the engine stepped inside backward used the hyper-parameters of that
            # moment: a change since then would update the two halves of the model differently
            mark, self._fused_mark = self._fused_mark, None
            if mark is not None and mark != self.fused_hyper():
                raise RuntimeError(f"optimizer hyper-parameters changed between backward and "
                                   f"step() (fused decode used {mark}, step sees "
                                   f"{self.fused_hyper()}): set the LR before backward")
        lr = float(self._uniform("lr"))
        mom = float(self._uniform("momentum"))
        damp = float(self._uniform("dampening"))
        nest = bool(self._uniform("nesterov"))
        p, g = self.arena.param_buf, self.arena.grad
        lib = ops_for(p)
        wd = self._seg_wd(p.device)
        if self.device_hyper and not torch.cuda.is_current_stream_capturing():
            self.load_hyper()
        if lib is not None:
            t, wd = self._tables(p.device)
            # the bf16 weight mirror the next forward reads is written by the same kernel
            # (master -> model copy of fp16util.py:103-138 fused: no separate cast pass)
            pb = getattr(self.arena, "param_bf16", None)
            if t is not None:        # (None: every segment was stepped with its decode)
                lib.sgd_step(p, g, self.buf, t["seg_off"], t["seg_n"], t["segs"], t["tasks"], wd,
                             lr, mom, damp, int(nest), int(self._first), float(self.grad_scale),
                             self._hyper if self.device_hyper else None, pb)
            if pb is not None:
                self.arena.mark_bf16_fresh()
        else:
            wdv = torch.repeat_interleave(
                wd, torch.from_numpy(np.diff(np.append(self.plan.offsets, self.arena.numel))))
            d = g * self.grad_scale + wdv * p
            if mom != 0:
                if self._first:
                    self.buf.copy_(d)
                else:
                    self.buf.mul_(mom).add_(d, alpha=1 - damp)
                d = d + mom * self.buf if nest else self.buf
            p.add_(d, alpha=-lr)
        if self._first and mom != 0:
            self._bind_state()
        self._first = False
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.arena.zero_()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        any_buf = False
        for g in self.param_groups:
            for p in g["params"]:
                st = self.state.get(p, {})
                b = st.get("momentum_buffer")
                if b is not None:
                    s = self.arena.segments[self._seg_of[id(p)]]
                    _dense_strided_view(self.buf, s.offset, p).copy_(b)
                    any_buf = True
        self._first = not any_buf
        if any_buf:
            self._bind_state()
