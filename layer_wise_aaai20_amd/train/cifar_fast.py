"""GPU-resident CIFAR-10 trainer used by ``bench_cifar.py`` (BASELINE configs 2, 3 and the
uncompressed ResNet-9 anchor).

Recipe of ``CIFAR10/dawn.py:105-148``: batch 512 per rank, summed cross-entropy with a per-sample
LR (``PiecewiseLinear([0,5,E],[0,0.4,0]) / bs``), SGD weight decay ``5e-4·bs``, Nesterov momentum
0.9, crop / flip / cutout augmentation. MI355X path: the dataset lives in HBM and is augmented
there (``GPUBatches``), bf16 autocast + channels_last, fused BN+ReLU in the graph networks,
CompressedDDP (compression overlapped with backward) and the fused flat-arena SGD.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..data import cifar as D
from ..models.cifar import build_network
from ..ops import nn as lwnn
from ..ops._ext import h16
from ..optim.flat_sgd import FlatSGD
from ..parallel.ddp import CompressedDDP
from ..utils.logging import PiecewiseLinear
from .graphs import StepGraph


def _first_conv_pads(net) -> bool:
    """The net's input feeds exactly one MFMA convolution of 3 input channels (which reads a
    zero-padded 4-channel copy of its input, ops/conv.py _c4_input)."""
    from ..ops.conv import MFMAConv2d
    graph = getattr(net, "graph", None)
    if graph is None:
        # the module nets (VGG-16, the module AlexNet: models/cifar.py) feed batch["input"]
        # straight into features[0]
        feats = getattr(net, "features", None)
        first = feats[0] if isinstance(feats, torch.nn.Sequential) and len(feats) else None
        return isinstance(first, MFMAConv2d) and first.in_channels == 3
    users = [m for m, ins in graph.values() if "input" in ins]
    return len(users) == 1 and isinstance(users[0], MFMAConv2d) and users[0].in_channels == 3


class CifarTrainer:
    def __init__(self, network="resnet9", device=None, compress="none", method="none", K=None,
                 V=None, qstates=None, error_feedback=False, batch_size=512, epochs=24,
                 momentum=0.9, dtype=torch.bfloat16, bucket_cap_mb=25.0, wire="auto",
                 n_train=50000, seed=0, fused=True, graph=None, n_test=1000,
                 task="textures", amp=None, dense_below=0, momentum_correction=False,
                 lr_scale=1.0, ef_lr_scaled=False, world_size=None, fused_sgd=True):
        self.device = torch.device(device or "cuda")
        self.dtype = dtype
        self.bs = batch_size
        net = build_network(network)
        if fused and self.device.type == "cuda":
            from ..ops.conv import fuse_convs
            from ..ops.gemm import fuse_linears
            lwnn.fuse_graph_network(net)
            lwnn.fuse_dict_losses(net)
            fuse_convs(net)          # every conv / Linear on the MFMA kernels
            fuse_linears(net)
        net = net.to(self.device)
        if self.device.type == "cuda":
            net = net.to(memory_format=torch.channels_last)
            if fused:
                lwnn.share_bn_counters(net)   # one counter-bump kernel per step, not one per BN
        self.model = net
        # momentum_correction (DGC, opt-in): the velocity lives in the compressor's residual and
        # the optimizer runs without momentum (parallel/engine.py)
        mc = float(momentum) if momentum_correction else 0.0
        self.ddp = CompressedDDP(net, compress=compress, method=method, K=K, V=V,
                                 qstates=qstates, error_feedback=error_feedback,
                                 bucket_cap_mb=bucket_cap_mb, wire=wire, flat_params=True,
                                 dense_below=dense_below, momentum_correction=mc,
                                 ef_lr_scaled=ef_lr_scaled, world_size=world_size)
        om = 0.0 if mc > 0 else momentum
        self.opt = FlatSGD(net.parameters(), self.ddp.arena, lr=0.0, momentum=om,
                           nesterov=om > 0, weight_decay=5e-4 * batch_size)
        if mc > 0:           # weight decay enters the velocity (and leaves the optimizer)
            self.ddp.engine.set_mc_weight_decay(self.opt)
        if ef_lr_scaled:
            self.ddp.engine.lr_source = self.opt.lr_device
        # layer-wise Top-K buckets: decode and SGD step in one pass (step() sets the LR first;
        # fused_sgd=False for gradient accumulation / clipping between backward and the step)
        if fused_sgd:
            self.ddp.engine.set_fused_sgd(self.opt)
        ds = D.synthetic_cifar10(n_train, n_test, seed, task=task, amp=amp)
        x = D.transpose(D.normalise(D.pad(ds["train"]["data"], 4)))
        tx = D.transpose(D.normalise(ds["test"]["data"]))
        self.test_batches = D.GPUBatches(
            torch.from_numpy(np.ascontiguousarray(tx)).to(self.device),
            torch.as_tensor(ds["test"]["labels"]).to(self.device), batch_size, shuffle=False,
            channels_last=self.device.type == "cuda", dtype=torch.float32)
        # fused GPU nets: training batches in the compute dtype, already zero-padded to the 4
        # channels the MFMA image convolution reads (csrc/augment.hip) — the image conv then
        # casts / pads nothing (the same bf16 values: the conv rounded the fp32 batch itself)
        gpu_fused = fused and self.device.type == "cuda" and _first_conv_pads(net)
        self.batches = D.GPUBatches(torch.from_numpy(np.ascontiguousarray(x)).to(self.device),
                                    torch.as_tensor(ds["train"]["labels"]).to(self.device),
                                    batch_size, shuffle=True, augment=True, drop_last=True,
                                    seed=seed, channels_last=self.device.type == "cuda",
                                    dtype=h16() if gpu_fused else torch.float32,
                                    pad4=gpu_fused)
        # lr_scale: the peak LR as a multiple of the dawn recipe's 0.4 (the Random-K + EF
        # stability sweep, scripts/ef_trace.py)
        self.sched = PiecewiseLinear([0, 5, epochs], [0, 0.4 * float(lr_scale), 0])
        self.steps_per_epoch = len(self.batches)
        self.step_count = 0
        self._it = None
        self.last = None
        # whole step as one HIP graph after 3 eager steps (train/graphs.py): at 1.5-6 ms per
        # step the per-kernel host launch cost is a large share of an eager CIFAR step
        if graph is None:          # LWAAAI_GRAPH=0 keeps the CIFAR step eager
            graph = os.environ.get("LWAAAI_GRAPH", "1") != "0"
        self.graphed = StepGraph(self._eager, self.ddp.engine, self.opt, self.device, 3, graph)

    def next_batch(self):
        if self._it is None:
            self._it = iter(self.batches)
        try:
            return next(self._it)
        except StopIteration:
            self._it = iter(self.batches)
            return next(self._it)

    def _eager(self, x, target):
        with torch.autocast(device_type=self.device.type, dtype=self.dtype,
                            enabled=self.dtype != torch.float32, cache_enabled=False):
            out = self.ddp({"input": x, "target": target})
            loss = out["loss"].float().sum()
        loss.backward()
        self.opt.step()
        return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}, \
            loss.detach()

    def step(self, batch=None):
        batch = batch or self.next_batch()
        lr = self.sched(self.step_count / self.steps_per_epoch) / self.bs
        for g in self.opt.param_groups:
            g["lr"] = lr
        if self.ddp.engine.lr_scaled:
            self.opt.load_hyper()             # the residual rescale reads this step's LR
        out, loss = self.graphed(batch["input"], batch["target"])
        self.step_count += 1
        self.last = out
        return loss

    @torch.no_grad()
    def evaluate(self) -> float:
        """Held-out accuracy on the synthetic test split (eval-mode BatchNorm)."""
        self.ddp.sync_buffers()          # rank 0's running statistics on every rank
        self.model.eval()
        correct = total = 0
        for b in self.test_batches:
            with torch.autocast(device_type=self.device.type, dtype=self.dtype,
                                enabled=self.dtype != torch.float32):
                out = self.model({"input": b["input"], "target": b["target"]})
            correct += int(out["correct"].float().sum())
            total += int(b["target"].numel())
        self.model.train()
        return correct / max(total, 1)
