"""ImageNet training engine (ResNet family): the step used by ``bench.py`` and by the
reference-compatible entry point ``IMAGENET/training/train_imagenet_nv.py``.

Reference step (``IMAGENET/training/train_imagenet_nv.py:388-441``): LR update → forward →
cross-entropy → (fp16: ×loss_scale) → backward → per-layer compressed all-reduce → master-weight
SGD. Here the same step is: fused uint8→bf16 NHWC normalise → bf16-autocast channels_last forward →
backward with bucketed compression overlapped (CompressedDDP) → one fused SGD launch.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from ..models import resnet as resnet_models
from ..ops import nn as lwnn
from ..ops._ext import set_half
from ..optim.flat_sgd import FlatSGD
from ..parallel.ddp import CompressedDDP
from .graphs import StepGraph

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

    **HIP-graph mode** (``graph=True``, the default on a GPU when every codec is graph-safe): after
    ``graph_warmup`` eager steps the whole step is captured once and replayed
    (:class:`~.graphs.StepGraph`): ~650 kernel launches become two input copies and one replay,
    so the host's launch rate no longer sets the step time. The LR schedule reaches the captured
    SGD kernel through device memory (:meth:`FlatSGD.load_hyper`)."""

    def __init__(self, ddp: CompressedDDP, optimizer, device, dtype=torch.bfloat16,
                 criterion: Optional[nn.Module] = None, channels_last: bool = True,
                 graph: Optional[bool] = None, graph_warmup: int = 3,
                 graph_auto: Optional[bool] = None, loss_scale: float = 1.0):
        self.ddp = ddp
        self.opt = optimizer
        self.device = device
        self.dtype = dtype
        # static loss scale (fp16: the reference's --loss-scale, train_imagenet_nv.py:412-428);
        # the optimizer unscales inside its kernel (FlatSGD grad_scale = 1 / loss_scale)
        self.loss_scale = float(loss_scale)
        self.channels_last = channels_last
        self.criterion = criterion or lwnn.FusedCrossEntropyLoss()
        self.mean = torch.tensor(IMAGENET_MEAN, device=device, dtype=torch.float32)
        self.std = torch.tensor(IMAGENET_STD, device=device, dtype=torch.float32)
        self._last = None
        self.graphed = StepGraph(self._eager, ddp.engine, optimizer, device, graph_warmup, graph,
                                 auto=graph_auto)

    @property
    def graph_replays(self) -> int:
        return self.graphed.replays

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
        (loss * self.loss_scale if self.loss_scale != 1.0 else loss).backward()
        self.opt.step()
        return out.detach(), target, loss.detach()

    def step(self, images_u8_nhwc: torch.Tensor, target: torch.Tensor):
        run = self.graphed if self.ddp.training else self._eager
        self._last = run(images_u8_nhwc, target)
        return self._last[2]

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
                  bn0=True, wire="auto", graph=None, graph_warmup: int = 3,
                  world_size=None, graph_auto=None, dense_below=0,
                  momentum_correction=False, loss_scale=None,
                  fused_sgd: bool = True) -> ImageNetTrainer:
    """``world_size``: build the codecs for that many ranks without a process group (a simulated
    world driven by ``parallel/loopback.py``); default: the process group's size.

    ``dtype="fp16"`` with ``fused``: the reference's fp16 recipe on the MFMA kernels — the fp16
    build of the kernel library (``ops/_ext.py set_half``), fp32 master weights with an fp16
    mirror written by the SGD kernel, and a static loss scale (default 1024, as the reference's
    ``--loss-scale``) unscaled inside that kernel.

    ``fused_sgd`` (default on): the layer-wise Top-K buckets' decode and their SGD step run in
    one pass inside backward (``GradSyncEngine.set_fused_sgd``). The contract is one backward,
    then ``opt.step()`` with the hyper-parameters unchanged in between — FlatSGD raises
    otherwise; ``fused_sgd=False`` for callers that accumulate, clip or read gradients between
    backward and the step."""
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    tdtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[dtype] \
        if isinstance(dtype, str) else dtype
    if fused and device.type == "cuda":
        set_half(tdtype == torch.float16)       # before any 16-bit buffer or kernel choice
    if loss_scale is None:
        loss_scale = 1024.0 if tdtype == torch.float16 else 1.0
    net = build_model(model, bn0=bn0) if isinstance(model, str) else model
    if fused:
        lwnn.fuse_resnet(net)
    net = net.to(device)
    if device.type == "cuda":
        net = net.to(memory_format=torch.channels_last)
    if fused:
        lwnn.share_bn_counters(net)
    mc = float(momentum) if momentum_correction else 0.0     # DGC: velocity in the residual
    ddp = CompressedDDP(net, compress=compress, method=method, K=K, V=V, qstates=qstates,
                        error_feedback=error_feedback, bucket_cap_mb=bucket_cap_mb, wire=wire,
                        flat_params=True, world_size=world_size, dense_below=dense_below,
                        momentum_correction=mc)
    groups = bn_param_groups(net, weight_decay, no_bn_wd)
    om = 0.0 if mc > 0 else momentum
    opt = FlatSGD(groups, ddp.arena, lr=lr, momentum=om, nesterov=om > 0,
                  weight_decay=weight_decay, grad_scale=1.0 / float(loss_scale))
    if mc > 0:               # weight decay enters the velocity (and leaves the optimizer)
        ddp.engine.set_mc_weight_decay(opt)
    # layer-wise Top-K buckets: decode and SGD step in one pass (the LR is set before each step)
    if fused_sgd:
        ddp.engine.set_fused_sgd(opt)
    return ImageNetTrainer(ddp, opt, device, tdtype, graph=graph, graph_warmup=graph_warmup,
                           graph_auto=graph_auto, loss_scale=loss_scale)
