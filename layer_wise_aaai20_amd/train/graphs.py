"""Whole-training-step HIP graphs.

A compressed-gradient training step on MI355X issues hundreds of short kernels (ResNet-50: ~650,
CIFAR nets: ~150-300 at 1.5-6 ms per step). Launched one by one from Python, the host's launch
rate — not the GPU — sets the step time whenever the host is slower than the kernels (measured on
ResNet-50: 27.6 ms wall for 24.6 ms of kernels on one box, ``profiles/r2_head3_step_breakdown.txt``).
The reference has no counterpart (it launches per-op CUDA kernels and per-tensor NCCL calls from
Python, ``IMAGENET/training/train_imagenet_nv.py:388-441``, ``CIFAR10/core.py:175-301``).

:class:`StepGraph` runs a step closure eagerly for ``warmup`` calls (GEMM tile tuner, workspaces,
RCCL communicators and the caching allocator settle), then captures it once with
``torch.cuda.graph`` — forward, backward with the side-stream compression and the bucket
collectives, decode, fused SGD — and afterwards every call is: copy the inputs into the captured
buffers, write the learning rate / loss scale into the device tensor the SGD kernel reads
(``FlatSGD.load_hyper``), replay. Anything else a capture bakes in is part of the signature
(input shapes/dtypes, ``FlatSGD.graph_signature``); a change re-captures. The Philox-keyed codecs
(Random-K, TernGrad, QSGD) read the step counter from device memory (``GradSyncEngine._dstep``,
advanced inside the graph), so every replay draws fresh keys. Steps the capture cannot represent
— the threshold methods' sparse wire (a host read of the agreed capacity), gloo collectives,
c10d RCCL calls — stay eager (``GradSyncEngine.graph_safe``).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

import torch


def graphs_enabled(default: bool = True) -> bool:
    return os.environ.get("LWAAAI_GRAPH", "1" if default else "0") != "0"


class StepGraph:
    def __init__(self, fn: Callable, engine, optimizer, device, warmup: int = 3,
                 enabled: Optional[bool] = None):
        self.fn = fn
        self.engine = engine
        self.opt = optimizer
        self.device = torch.device(device)
        self.warmup = int(warmup)
        if enabled is None:
            enabled = graphs_enabled()
        self.enabled = (bool(enabled) and self.device.type == "cuda" and
                        hasattr(optimizer, "load_hyper"))
        self.replays = 0
        self._eager_done = 0
        self._g = None        # (graph, static inputs, static outputs, signature)

    def active(self) -> bool:
        return self.enabled and self.engine.graph_safe()

    def _signature(self, inputs: Sequence[torch.Tensor]) -> tuple:
        return (tuple((tuple(t.shape), t.dtype, t.stride()) for t in inputs),
                self.opt.graph_signature())

    def __call__(self, *inputs: torch.Tensor):
        if not self.active():
            return self.fn(*inputs)
        sig = self._signature(inputs)
        if self._g is None or self._g[-1] != sig:
            if self._eager_done < self.warmup:
                self._eager_done += 1
                return self.fn(*inputs)
            try:
                self._capture(inputs, sig)
            except RuntimeError as e:          # capture unsupported here: stay eager
                self.enabled = False
                self._g = None
                torch.cuda.synchronize(self.device)
                self.engine._reset_state()
                print(f"[lwaaai] HIP-graph capture failed, running eagerly: {e}", flush=True)
                return self.fn(*inputs)
        graph, static_in, static_out, _ = self._g
        for dst, src in zip(static_in, inputs):
            dst.copy_(src, non_blocking=True)
        self.opt.load_hyper()
        graph.replay()
        self.replays += 1
        # host mirror of what the replayed finish() did on the device (engine._dstep += 1)
        self.engine.step += 1
        self.engine.stats.steps += 1
        return static_out

    def _capture(self, inputs, sig) -> None:
        self._g = None
        static_in = [t.clone() for t in inputs]
        self.opt.device_hyper = True
        self.opt.load_hyper()
        torch.cuda.synchronize(self.device)
        host_step = (self.engine.step, self.engine.stats.steps)
        graph = torch.cuda.CUDAGraph()
        try:
            # thread_local: RCCL's watchdog thread queries events while this thread captures
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                static_out = self.fn(*static_in)
            torch.cuda.synchronize(self.device)
        finally:
            # the capture ran the step's Python (finish() counted a step) but no kernel
            self.engine.step, self.engine.stats.steps = host_step
        # the capture recorded the step without running it: the caller's replay performs it
        self._g = (graph, static_in, static_out, sig)
