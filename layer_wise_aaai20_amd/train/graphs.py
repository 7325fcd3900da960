"""Whole-training-step HIP graphs.

A compressed-gradient training step on MI355X issues hundreds of short kernels (ResNet-50: ~650,
CIFAR nets: ~150-300 at 1.5-6 ms per step). Launched one by one from Python, the host's launch
rate — not the GPU — sets the step time whenever the host is slower than the kernels (measured on
ResNet-50: 27.6 ms wall for 24.6 ms of kernels on one box, ``profiles/r2_head3_step_breakdown.txt``).
The reference has no counterpart (it launches per-op CUDA kernels and per-tensor NCCL calls from
Python, ``IMAGENET/training/train_imagenet_nv.py:388-441``, ``CIFAR10/core.py:175-301``).

:class:`StepGraph` keeps one captured graph per step *signature* (input shapes / dtypes / strides
plus everything the optimizer bakes into its launch, ``FlatSGD.graph_signature``). A signature is
run eagerly for ``warmup`` calls (GEMM tile tuner, workspaces, RCCL communicators and the caching
allocator settle for exactly these shapes), then captured once with ``torch.cuda.graph`` — forward,
backward with the bucket compression and collectives, decode, fused SGD — and every later call with
that signature is: copy the inputs into the captured buffers, write the learning rate / loss scale
into the device tensor the SGD kernel reads (``FlatSGD.load_hyper``), replay. An epoch's odd-sized
last batch therefore never evicts the full-size graph; it stays eager until it has been seen
``warmup`` times. The Philox-keyed codecs (Random-K, TernGrad, QSGD) read the step counter from
device memory (``GradSyncEngine._dstep``, advanced inside the graph), so every replay draws fresh
keys. Steps the capture cannot represent — gloo collectives, per-bucket timing — stay eager
(``GradSyncEngine.graph_safe``).

Graph-vs-eager choice (``auto``, MIOpen-find style): once per run, after the first capture, the
first replay (which pays the one-time graph upload) is discarded, ``timed`` replays are timed back
to back and compared with the last ``timed`` eager warm-up steps; the graph is dropped when it is
not faster. At world > 1 every rank measures and the sums are all-reduced, so all ranks take the
same decision (a rank replaying while another runs eagerly would still pair its collectives
correctly, but the step would then be as slow as the slowest mode).
"""
from __future__ import annotations

import gc
import os
import time
import weakref
from typing import Callable, Dict, Optional, Sequence

import torch


def graphs_enabled(default: bool = True) -> bool:
    return os.environ.get("LWAAAI_GRAPH", "1" if default else "0") != "0"


_LIVE = weakref.WeakSet()      # every StepGraph, for release_graphs()


def release_graphs() -> None:
    """Drop every captured step graph (after draining the device). A communicator whose
    collectives live on in a captured graph cannot be torn down: ncclCommAbort waited forever on
    one in a 2-rank run (scripts/mgpu_probe.py), so ``comm.shutdown_native`` calls this first."""
    live = list(_LIVE)
    if any(sg._graphs for sg in live) and torch.cuda.is_available():
        torch.cuda.synchronize()
    for sg in live:
        sg._graphs.clear()
        sg.enabled = False


class StepGraph:
    MAX_GRAPHS = 4            # distinct captured signatures kept (LRU beyond that)

    def __init__(self, fn: Callable, engine, optimizer, device, warmup: int = 3,
                 enabled: Optional[bool] = None, auto: Optional[bool] = None, timed: int = 5):
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
        self.captures = 0
        self._graphs: Dict[tuple, tuple] = {}     # signature -> (graph, static_in, static_out)
        self._seen: Dict[tuple, int] = {}         # input signature -> eager calls so far
        if auto is None:
            auto = os.environ.get("LWAAAI_GRAPH_AUTO", "1") != "0"
        self.auto = bool(auto)
        self.timed = max(1, int(timed))
        self.decided = not self.auto
        self._eager_t = []        # host ms of consecutive eager steps (device drained)
        self._replay_t = []
        self._t_last = None
        self.choice = None        # (graph ms, eager ms) of the decision, for the logs
        _LIVE.add(self)

    # ------------------------------------------------------------------ policy
    def active(self) -> bool:
        return self.enabled and self.engine.graph_safe()

    def _signature(self, inputs: Sequence[torch.Tensor]) -> tuple:
        return (tuple((tuple(t.shape), t.dtype, t.stride()) for t in inputs),
                self.opt.graph_signature())

    @property
    def _g(self):
        """The most recently used captured graph (compatibility with older callers/tests)."""
        return next(reversed(self._graphs.values())) if self._graphs else None

    def _fn(self, *inputs: torch.Tensor):
        """The eager step. At world > 1 its kernel-tuning decisions are agreed across ranks
        (``ops/tuning.py`` ``rank_agreement``): every rank then runs the same kernels."""
        if getattr(self.engine, "world", 1) <= 1:
            return self.fn(*inputs)
        from ..ops.tuning import rank_agreement
        with rank_agreement(getattr(self.engine, "pg", None), self.device):
            return self.fn(*inputs)

    def __call__(self, *inputs: torch.Tensor):
        if not self.active():
            return self._fn(*inputs)
        sig = self._signature(inputs)
        g = self._graphs.get(sig)
        if g is None:
            # warm-up is counted per input shape (what the tuners / allocator settle on); the
            # optimizer part of the signature (e.g. SGD's first-step flag) does not restart it
            n = self._seen.get(sig[0], 0)
            if n < self.warmup:
                self._seen[sig[0]] = n + 1
                return self._eager_timed(inputs, n)
            err = None
            try:
                from ..parallel.comm import inject_fault
                if inject_fault("capture", self._rank()):
                    raise RuntimeError("injected capture failure (LWAAAI_INJECT_FAULT)")
                g = self._capture(inputs, sig)
            except Exception as e:             # noqa: BLE001 — any failure joins the agreement
                # (a rank that skipped _agree would leave its peers blocked in it until the
                # process group times out; every rank falls back to eager instead)
                err = e
            # one decision for all ranks: a rank replaying while another runs eagerly would
            # still pair its collectives, but the whole job would then run at the slow mode
            if err is not None:
                # the failed capture may have queued deferred split-K reduces over slabs it never
                # wrote: the eager step's flush must not add them into the arena
                from ..ops._ext import splitk_discard
                splitk_discard(torch.empty(0, device=self.device))
                if hasattr(self.opt, "_fused_mark"):
                    self.opt._fused_mark = None  # (its fused update never ran either)
            if not self._agree(err is None):
                self.enabled = False
                self._graphs.clear()
                torch.cuda.synchronize(self.device)
                self.engine._reset_state()
                why = err if err is not None else "another rank's capture failed"
                print(f"[lwaaai] HIP-graph capture failed ({why}): every rank runs eagerly",
                      flush=True)
                return self._fn(*inputs)
        else:
            self._graphs[sig] = self._graphs.pop(sig)      # LRU order
        return self._replay(g, inputs)

    def _rank(self) -> int:
        from ..parallel import comm
        return comm.rank(getattr(self.engine, "pg", None))

    def _agree(self, ok: bool) -> bool:
        if getattr(self.engine, "world", 1) <= 1:
            return ok
        from ..parallel import comm
        return comm.agree(ok, getattr(self.engine, "pg", None), self.device)

    def _eager_timed(self, inputs, n: int):
        deciding = not self.decided
        if deciding and n >= 1:                 # (the first call of a signature tunes tiles)
            self._mark()
        out = self._fn(*inputs)
        if deciding and n >= 1:
            self._eager_t.append(self._lap())
            self._eager_t = self._eager_t[-self.timed:]
        return out

    def _replay(self, g, inputs):
        graph, static_in, static_out = g
        deciding = not self.decided
        if deciding:
            self._mark()
        for dst, src in zip(static_in, inputs):
            dst.copy_(src, non_blocking=True)
        self.opt.load_hyper()
        graph.replay()
        self.replays += 1
        hb = getattr(self.engine, "heartbeat", None)
        if hb is not None:
            hb()                     # communicator watchdog deadline for this step
        # host mirror of what the replayed finish() did on the device (engine._dstep += 1)
        self.engine.step += 1
        self.engine.stats.steps += 1
        if deciding:
            self._replay_t.append(self._lap())
            if len(self._replay_t) > self.timed:          # [0] paid the graph upload
                self._decide()
        return static_out

    def _mark(self) -> None:
        torch.cuda.synchronize(self.device)
        self._t_last = time.perf_counter()

    def _lap(self) -> float:
        torch.cuda.synchronize(self.device)
        return (time.perf_counter() - self._t_last) * 1e3

    def _decide(self) -> None:
        self.decided = True
        graph_ms = sum(self._replay_t[1:]) / len(self._replay_t[1:])
        eager_ms = sum(self._eager_t) / len(self._eager_t) if self._eager_t else float("inf")
        world = getattr(self.engine, "world", 1)
        if world > 1:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                backend = dist.get_backend(getattr(self.engine, "pg", None))
                dev = self.device if backend == "nccl" else torch.device("cpu")
                t = torch.tensor([graph_ms, eager_ms], dtype=torch.float64, device=dev)
                dist.all_reduce(t, group=getattr(self.engine, "pg", None))
                graph_ms, eager_ms = (float(v) / world for v in t.tolist())
        self.choice = (graph_ms, eager_ms)
        if graph_ms > eager_ms:
            # not faster than launching from Python on this host: stay eager
            self.enabled = False
            self._graphs.clear()
            print(f"[lwaaai] HIP-graph step {graph_ms:.2f} ms vs eager {eager_ms:.2f} ms: "
                  f"staying eager", flush=True)

    # ------------------------------------------------------------------ capture
    def _capture(self, inputs, sig) -> tuple:
        static_in = [t.clone() for t in inputs]
        self.opt.device_hyper = True
        self.opt.load_hyper()
        torch.cuda.synchronize(self.device)
        host_step = (self.engine.step, self.engine.stats.steps)
        graph = torch.cuda.CUDAGraph()
        # (each signature keeps its own private memory pool: graphs sharing a pool would alias
        # each other's step temporaries; 288 GB of HBM affords a few copies of the activations)
        # no garbage collection while capturing: a collection triggered by the step's own
        # allocations can free an unreachable object holding another HIP graph, whose destructor
        # is not permitted during a capture (it aborted a process that built many trainers:
        # "operation not permitted when stream is capturing" in ~CUDAGraph)
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            # thread_local: RCCL's watchdog thread queries events while this thread captures
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                static_out = self.fn(*static_in)
            torch.cuda.synchronize(self.device)
        finally:
            if gc_on:
                gc.enable()
            # the capture ran the step's Python (finish() counted a step) but no kernel
            self.engine.step, self.engine.stats.steps = host_step
        while len(self._graphs) >= self.MAX_GRAPHS:
            self._graphs.pop(next(iter(self._graphs)))
        g = (graph, static_in, static_out)
        self._graphs[sig] = g
        self.captures += 1
        return g
