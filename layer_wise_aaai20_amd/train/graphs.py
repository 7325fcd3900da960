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
import time
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
        # find-style choice on one rank: the last eager warm-up steps and the first replays are
        # timed and the graph is dropped if it is not faster (a GPU-bound step whose side-stream
        # overlap outweighs the saved launches, e.g. VGG-16: 5.96 ms eager vs 6.08 ms graph).
        # Multi-rank jobs keep the graph (one decision for every rank, no extra collective).
        self.auto = os.environ.get("LWAAAI_GRAPH_AUTO", "1") != "0"
        self.decided = False
        self._eager_ms = []
        self._t0 = 0.0
        self._replay_t0 = None
        self._timed_replays = 0

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
                # steady-state eager rate: the last two warm-up steps timed back to back
                deciding = self.warmup >= 3 and self._deciding()
                if deciding and self._eager_done == self.warmup - 1:
                    self._t0 = self._sync_time()
                out = self.fn(*inputs)
                if deciding and self._eager_done == self.warmup:
                    self._eager_ms = [(self._sync_time() - self._t0) / 2]
                return out
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
        timing = self._deciding() and bool(self._eager_ms)
        if timing and self._replay_t0 is None:
            self._replay_t0 = self._sync_time()       # first two replays timed back to back
        for dst, src in zip(static_in, inputs):
            dst.copy_(src, non_blocking=True)
        self.opt.load_hyper()
        graph.replay()
        self.replays += 1
        if timing:
            self._timed_replays += 1
            if self._timed_replays == 2:
                graph_ms = (self._sync_time() - self._replay_t0) / 2
                self.decided = True
                if graph_ms > self._eager_ms[0]:
                    # not faster than launching from Python on this host: stay eager
                    self.enabled = False
                    self._g = None
                    print(f"[lwaaai] HIP-graph step {graph_ms:.2f} ms vs eager "
                          f"{self._eager_ms[0]:.2f} ms: staying eager", flush=True)
        # host mirror of what the replayed finish() did on the device (engine._dstep += 1)
        self.engine.step += 1
        self.engine.stats.steps += 1
        return static_out

    def _deciding(self) -> bool:
        return self.auto and not self.decided and getattr(self.engine, "world", 1) == 1

    def _sync_time(self) -> float:
        """Milliseconds on the host clock after the device has drained."""
        torch.cuda.synchronize(self.device)
        return time.perf_counter() * 1e3

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
