"""CIFAR-10 training engine with the reference signatures (``CIFAR10/core.py:303-341``).

``run_batches`` → forward → ``loss.sum().backward()`` → gradient sync selected by ``compress``
(layer-wise / entire-model compression or plain averaging) → ``optimizer_step()`` →
``model.zero_grad()``. ``train`` optionally initialises the process group (gloo, TCP
``init_method``, as ``core.py:334``) and runs epochs, emitting the summary dict to loggers.

Differences, all deliberate: the sync goes through :mod:`..parallel.functional` (bucketed, one
collective per bucket, compressed wire formats), model state is broadcast from rank 0 before the
first step, and ``world_size`` may be an int or the env-callable of D5.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..parallel import comm
from ..parallel import functional as F
from ..parallel.engine import canonical_mode
from ..utils.logging import StatsLogger, Timer
from ..models.graph import union


def _graphed_step(model, optimizer_step, autocast, dev_type, graph):
    """The hooked (CompressedDDP + FlatSGD) training step as a :class:`~.graphs.StepGraph`
    (forward, summed-loss backward with the bucket compression, fused SGD): built once per model.
    The step-number-dependent LR is pushed into the param groups outside the graph and reaches
    the captured SGD kernel through device memory (``FlatSGD.load_hyper``)."""
    opt = getattr(optimizer_step, "__self__", None)           # TorchOptimiser.step
    inner = getattr(opt, "_opt", None)
    if not graph or dev_type != "cuda" or not hasattr(inner, "load_hyper"):
        return None
    sg = getattr(model, "_lw_step_graph", None)
    if sg is None:
        from .graphs import StepGraph

        def body(x, target):
            with torch.autocast(device_type=dev_type, dtype=autocast or torch.float32,
                                enabled=autocast is not None):
                out = model({"input": x, "target": target})
            out["loss"].float().sum().backward()
            inner.step()
            return {"loss": out["loss"].detach(), "correct": out["correct"].detach()}

        sg = StepGraph(body, model.engine, inner, next(model.parameters()).device)
        model._lw_step_graph = sg
    return opt, sg


def run_batches(model, batches, training, world_size=1, optimizer_step=None, stats=None,
                compress=None, method=None, K=None, V=None, qstates=None,
                error_feedback: bool = False, wire: str = "auto", max_batches: Optional[int] = None,
                autocast=None, graph: Optional[bool] = None):
    """``autocast``: compute dtype of the forward (the MI355X path: bf16). A model wrapped in
    :class:`~..parallel.ddp.CompressedDDP` synchronises its gradients from backward hooks and
    zeroes its gradient arena at the next forward, so no post-backward sync / zero_grad here;
    its whole step is replayed as one HIP graph once warm (``graph``, default on:
    ``LWAAAI_GRAPH=0`` keeps it eager)."""
    stats = stats or StatsLogger(("loss", "correct"))
    if not training and hasattr(model, "sync_buffers"):
        model.sync_buffers()             # collective: rank 0's BN statistics before evaluation
    model.train(training)
    mode = canonical_mode(compress) if compress not in (None, "none") else "none"
    hooked = getattr(model, "engine", None) is not None
    dev_type = next(model.parameters()).device.type
    if graph is None:
        import os
        graph = os.environ.get("LWAAAI_GRAPH", "1") != "0"
    gs = _graphed_step(model, optimizer_step, autocast, dev_type, graph) \
        if training and hooked else None
    for i, batch in enumerate(batches):
        if max_batches is not None and i >= max_batches:
            break
        if training and gs is not None:
            opt, sg = gs
            opt.step_number += 1                  # TorchOptimiser.step's LR update, host side
            vals = opt.param_values()
            for g in opt.param_groups:
                g.update(**vals)
            out = sg(batch["input"], batch["target"])
            # a replay rewrites the same output buffers: keep this step's values
            stats.append({k: v.clone() for k, v in out.items()} if sg.replays else out)
            continue
        if training:
            with torch.autocast(device_type=dev_type, dtype=autocast or torch.float32,
                                enabled=autocast is not None):
                output = model(batch)
            stats.append(output)
            output["loss"].float().sum().backward()
            if hooked:
                optimizer_step()
                continue
            if mode == "layerwise":
                F.layerwise_compressed_comm(model, world_size, method, K, V, qstates,
                                            error_feedback=error_feedback, wire=wire)
            elif mode == "entiremodel":
                F.entiremodel_compressed_comm(model, world_size, method, K, V, qstates,
                                              error_feedback=error_feedback, wire=wire)
            else:
                F.all_reduce(model, world_size)
            optimizer_step()
            model.zero_grad(set_to_none=False)   # torch 1.x semantics: keep arena views
        else:
            with torch.no_grad(), torch.autocast(device_type=dev_type,
                                                 dtype=autocast or torch.float32,
                                                 enabled=autocast is not None):
                output = model(batch)
            stats.append(output)
    return stats


def train_epoch(model, train_batches, test_batches, optimizer_step, timer, world_size=1,
                test_time_in_total=True, compress=None, method=None, K=None, V=None, qstates=None,
                **kw):
    train_stats = run_batches(model, train_batches, True, world_size, optimizer_step,
                              compress=compress, method=method, K=K, V=V, qstates=qstates, **kw)
    train_time = timer()
    test_stats = run_batches(model, test_batches, False, world_size,
                             autocast=kw.get("autocast"))
    test_time = timer(test_time_in_total)
    return {
        "train time": train_time, "train loss": train_stats.mean("loss"),
        "train acc": train_stats.mean("correct"),
        "test time": test_time, "test loss": test_stats.mean("loss"),
        "test acc": test_stats.mean("correct"),
        "total time": timer.total_time,
    }


def default_backend() -> str:
    """RCCL ("nccl") when the ranks train on GPUs — the bucket collectives then go through the
    native, graph-capturable RCCL communicator (csrc/rccl.cpp) — gloo for CPU plumbing. (The
    reference hard-codes gloo, core.py:334, which stages every GPU tensor through the host.)"""
    return "nccl" if torch.cuda.is_available() else "gloo"


def init_distributed(master_address, world_size, rank, backend: Optional[str] = None):
    """``dist.init_process_group(init_method=master_address, ...)`` (core.py:334). A bare host
    (the reference default ``127.0.0.1``) is completed to ``tcp://host:$MASTER_PORT`` (29500
    by default). On a GPU the group is created even for one rank, as the reference does, so the
    single-rank run takes the same (RCCL) path as a multi-rank one; a one-rank group on a bare
    host takes a free ephemeral port, so concurrent single-GPU runs on one host do not collide."""
    backend = backend or default_backend()
    if comm.is_dist() or (int(world_size) <= 1 and backend != "nccl"):
        return
    addr = master_address or "127.0.0.1"
    if "://" not in addr and ":" not in addr:
        if int(world_size) <= 1:
            import socket
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                s.bind((addr, 0))
                port = s.getsockname()[1]
        else:
            import os
            port = int(os.environ.get("MASTER_PORT", "29500"))
        addr = f"tcp://{addr}:{port}"
    elif "://" not in addr:
        addr = f"tcp://{addr}"
    if backend == "nccl":
        torch.cuda.set_device(torch.cuda.current_device())
    kw = {"device_id": torch.device("cuda", torch.cuda.current_device())} \
        if backend == "nccl" else {}
    dist.init_process_group(backend=backend, init_method=addr, world_size=int(world_size),
                            rank=int(rank), **kw)
    print(f"process group: backend={dist.get_backend()} world={dist.get_world_size()} "
          f"rank={dist.get_rank()}", flush=True)


def train(model, optimizer, train_batches, test_batches, epochs, master_address=None,
          world_size=1, rank=0, loggers=(), test_time_in_total=True, timer=None, compress=None,
          method=None, K=None, V=None, qstates=None, backend: Optional[str] = None, **kw):
    init_distributed(master_address, world_size, rank, backend)
    if comm.is_dist() and comm.world_size() > 1:
        comm.broadcast_coalesced(list(model.state_dict().values()), 0)
    timer = timer or Timer()
    summary = {}
    for epoch in range(epochs):
        epoch_stats = train_epoch(model, train_batches, test_batches, optimizer.step, timer,
                                  world_size, test_time_in_total=test_time_in_total,
                                  compress=compress, method=method, K=K, V=V, qstates=qstates,
                                  **kw)
        lr = optimizer.param_values()["lr"] if hasattr(optimizer, "param_values") else \
            optimizer.param_groups[0]["lr"]
        summary = union({"epoch": epoch + 1, "lr": lr * train_batches.batch_size}, epoch_stats)
        eng = getattr(model, "engine", None)
        if eng is not None:              # compression telemetry: wire bytes of the last step
            summary = union(summary, {"comm MB": eng.stats.payload_bytes / 1e6,
                                      "comm ratio": eng.stats.ratio})
        for logger in loggers:
            logger.append(summary)
    return summary
