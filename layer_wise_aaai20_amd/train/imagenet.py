"""ImageNet training engine (ResNet family): the step used by ``bench.py`` and by the
reference-compatible entry point ``IMAGENET/training/train_imagenet_nv.py``.

Reference step (``IMAGENET/training/train_imagenet_nv.py:388-441``): LR update → forward →
cross-entropy → (fp16: ×loss_scale) → backward → per-layer compressed all-reduce → master-weight
SGD. Here the same step is: fused uint8→bf16 NHWC normalise → bf16-autocast channels_last forward →
backward with bucketed compression overlapped (CompressedDDP) → one fused SGD launch.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch import nn

from ..models import resnet as resnet_models
from ..ops import nn as lwnn
from ..optim.flat_sgd import FlatSGD
from ..parallel.ddp import CompressedDDP

IMAGENET_MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
IMAGENET_STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


def bn_param_groups(model: nn.Module, weight_decay: float, no_bn_wd: bool):
    """Two groups with BN parameters excluded from weight decay (``experimental_utils.py:5-22``),
    done on the module itself so the fp32 path keeps every parameter (fixes SURVEY.md D12)."""
    if not no_bn_wd:
        return [{"params": [p for p in model.parameters() if p.requires_grad],
                 "weight_decay": weight_decay}]
    bn_ids = set()
    for m in model.modules():
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            bn_ids.update(id(p) for p in m.parameters())
    bn, rest = [], []
    for p in model.parameters():
        if p.requires_grad:
            (bn if id(p) in bn_ids else rest).append(p)
    return [{"params": bn, "weight_decay": 0.0}, {"params": rest, "weight_decay": weight_decay}]


class ImageNetTrainer:
    """One training step = normalise → forward → loss → backward (+ overlapped compressed
    gradient exchange) → fused SGD.

    **HIP-graph mode** (``graph=True``, the default on a GPU when every codec is graph-safe): the
    step issues ~650 kernels, and on a host whose Python launch rate is below the GPU's kernel rate
    the GPU idles between them (measured: 27.6 ms wall for 24.6 ms of kernels,
    ``profiles/r2_head3_step_breakdown.txt``). After ``graph_warmup`` eager steps (GEMM tile tuner
    populated, RCCL communicators and the allocator warm), the whole step — forward, backward with
    its side-stream compression and collectives, decode, SGD — is captured once with
    ``torch.cuda.graph`` and each later step is two input copies plus one graph replay. The
    learning rate and loss scale are read by the SGD kernel from device memory
    (:meth:`FlatSGD.load_hyper`), so the reference's per-iteration LR schedule needs no
    re-capture; anything else the capture bakes in (momentum, weight decay, input shapes) triggers
    a re-capture when it changes. Codecs whose kernels take a host step counter (Random-K, the
    quantisers) or synchronise (sparse threshold wire) keep the eager path."""

    def __init__(self, ddp: CompressedDDP, optimizer, device, dtype=torch.bfloat16,
                 criterion: Optional[nn.Module] = None, channels_last: bool = True,
                 graph: Optional[bool] = None, graph_warmup: int = 3):
        self.ddp = ddp
        self.opt = optimizer
        self.device = device
        self.dtype = dtype
        self.channels_last = channels_last
        self.criterion = criterion or lwnn.FusedCrossEntropyLoss()
        self.mean = torch.tensor(IMAGENET_MEAN, device=device, dtype=torch.float32)
        self.std = torch.tensor(IMAGENET_STD, device=device, dtype=torch.float32)
        self._last = None
        if graph is None:
            graph = os.environ.get("LWAAAI_GRAPH", "1") != "0"
        self.graph = bool(graph) and device.type == "cuda" and hasattr(optimizer, "load_hyper")
        self.graph_warmup = int(graph_warmup)
        self._g = None                 # (CUDAGraph, static inputs/outputs, signature)
        self._eager_done = 0
        self.graph_replays = 0

    def normalize(self, images_u8_nhwc: torch.Tensor) -> torch.Tensor:
        # a fused ResNet takes the image as 4 bf16 channels (the implicit-GEMM stem's layout)
        pad4 = bool(getattr(self.ddp.module, "_lw_stem_c4", False))
        # host-side mean/std: reading the device copies would synchronise every step
        return lwnn.normalize_nhwc_u8(images_u8_nhwc, IMAGENET_MEAN, IMAGENET_STD, self.dtype,
                                      pad4=pad4)

    def forward_loss(self, x, target):
        # (no autocast weight cache: cached casts would be stale across graph replays)
        with torch.autocast(device_type=self.device.type, dtype=self.dtype,
                            enabled=self.dtype != torch.float32, cache_enabled=False):
            out = self.ddp(x)
            loss = self.criterion(out.float(), target)
        return out, loss

    def _eager(self, images_u8_nhwc: torch.Tensor, target: torch.Tensor):
        x = self.normalize(images_u8_nhwc)
        out, loss = self.forward_loss(x, target)
        loss.backward()
        self.opt.step()
        return out.detach(), loss.detach()

    def graph_active(self) -> bool:
        return (self.graph and self.ddp.training and self.ddp.engine.graph_safe())

    def step(self, images_u8_nhwc: torch.Tensor, target: torch.Tensor):
        if not self.graph_active():
            out, loss = self._eager(images_u8_nhwc, target)
            self._last = (out, target, loss)
            return loss
        sig = (tuple(images_u8_nhwc.shape), images_u8_nhwc.dtype, tuple(target.shape),
               self.opt.graph_signature())
        if self._g is None or self._g[-1] != sig:
            if self._eager_done < self.graph_warmup:
                self._eager_done += 1
                out, loss = self._eager(images_u8_nhwc, target)
                self._last = (out, target, loss)
                return loss
            try:
                self._capture(images_u8_nhwc, target, sig)
            except RuntimeError as e:          # capture unsupported here: stay eager
                self.graph = False
                self._g = None
                torch.cuda.synchronize(self.device)
                self.ddp.engine._reset_state()
                print(f"[lwaaai] HIP-graph capture failed, running eagerly: {e}", flush=True)
                out, loss = self._eager(images_u8_nhwc, target)
                self._last = (out, target, loss)
                return loss
        graph, xin, tin, out, loss, _ = self._g
        xin.copy_(images_u8_nhwc, non_blocking=True)
        tin.copy_(target, non_blocking=True)
        self.opt.load_hyper()
        graph.replay()
        self.graph_replays += 1
        self._last = (out, tin, loss)
        return loss

    def _capture(self, images_u8_nhwc, target, sig) -> None:
        self._g = None
        xin = images_u8_nhwc.clone()
        tin = target.clone()
        self.opt.device_hyper = True
        self.opt.load_hyper()
        torch.cuda.synchronize(self.device)
        graph = torch.cuda.CUDAGraph()
        # thread_local: RCCL's watchdog thread queries events while this thread captures
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            out, loss = self._eager(xin, tin)
        torch.cuda.synchronize(self.device)
        # the capture recorded the step without running it: the caller's replay performs it
        self._g = (graph, xin, tin, out, loss, sig)

    def last_top1(self) -> Optional[float]:
        if self._last is None:
            return None
        out, target, _ = self._last
        return float((out.argmax(1) == target).float().mean().item() * 100.0)


def build_model(name: str = "resnet50", bn0: bool = False) -> nn.Module:
    return getattr(resnet_models, name)(bn0=bn0)


def build_trainer(model="resnet50", device=None, compress="layerwise", method="Topk", K=0.001,
                  V=1e-3, qstates=255, error_feedback=False, bucket_cap_mb=25.0, dtype="bf16",
                  fused=True, momentum=0.9, weight_decay=1e-4, no_bn_wd=True, lr=0.1,
                  bn0=True, wire="auto", graph=None) -> ImageNetTrainer:
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    net = build_model(model, bn0=bn0) if isinstance(model, str) else model
    if fused:
        lwnn.fuse_resnet(net)
    net = net.to(device)
    if device.type == "cuda":
        net = net.to(memory_format=torch.channels_last)
    if fused:
        lwnn.share_bn_counters(net)
    ddp = CompressedDDP(net, compress=compress, method=method, K=K, V=V, qstates=qstates,
                        error_feedback=error_feedback, bucket_cap_mb=bucket_cap_mb, wire=wire,
                        flat_params=True)
    groups = bn_param_groups(net, weight_decay, no_bn_wd)
    opt = FlatSGD(groups, ddp.arena, lr=lr, momentum=momentum, nesterov=momentum > 0,
                  weight_decay=weight_decay)
    tdtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[dtype] \
        if isinstance(dtype, str) else dtype
    return ImageNetTrainer(ddp, opt, device, tdtype, graph=graph)
