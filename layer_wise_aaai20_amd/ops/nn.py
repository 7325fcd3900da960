"""Model-path ops backed by the HIP kernels of ``csrc/nn.hip`` and ``csrc/bn.hip`` (GPU) or torch
(CPU): fused uint8 normalisation, and BatchNorm with the following ReLU and residual add fused in
(``FusedBatchNorm2d``), plus ``fuse_resnet`` which switches a reference-layout ResNet to them
without changing a single parameter / buffer name (checkpoints stay compatible).
"""
from __future__ import annotations


import torch
import torch.nn.functional as F
from torch import nn

from ._ext import h16, load, ops_for

MAX_BN_C = 2048          # csrc/bn.hip: one 8-channel group per thread of a 256-thread block


def normalize_nhwc_u8(images: torch.Tensor, mean, std, dtype=None,
                      pad4: bool = False) -> torch.Tensor:
    """uint8 [N, H, W, C] → ``(x - mean) / std`` as an NCHW tensor in channels_last memory.

    One fused pass on the GPU; the reference does collate → ``.cuda()`` →
    ``.half()`` → ``sub_`` → ``div_`` (``IMAGENET/training/dataloader.py:81-93``). ``pad4``
    (GPU, bf16, 3 channels): write 4 channels with a zero 4th — the input layout of the
    implicit-GEMM stem convolution (``ops/conv.py``). ``mean`` / ``std`` are per-channel
    sequences of floats (preferred: no device read) or tensors."""
    assert images.dtype == torch.uint8 and images.dim() == 4
    dtype = h16() if dtype is None else dtype
    N, H, W, C = images.shape
    lib = ops_for(images)
    mh = [float(m) for m in (mean.tolist() if torch.is_tensor(mean) else mean)]
    sh = [float(v) for v in (std.tolist() if torch.is_tensor(std) else std)]
    if lib is not None and pad4 and C == 3 and dtype == h16() and images.is_contiguous():
        out = torch.empty((N, H, W, 4), dtype=dtype, device=images.device).permute(0, 3, 1, 2)
        lib.normalize_u8(images, out, mh, sh)
        return out
    if lib is not None and images.is_contiguous():
        out = torch.empty((N, C, H, W), dtype=dtype, device=images.device,
                          memory_format=torch.channels_last)
        lib.normalize_u8(images, out, mh, sh)
        return out
    mean = torch.as_tensor(mh, dtype=torch.float32)
    std = torch.as_tensor(sh, dtype=torch.float32)
    x = images.permute(0, 3, 1, 2).float()
    x = (x - mean.view(1, -1, 1, 1).to(x.device)) / std.view(1, -1, 1, 1).to(x.device)
    return x.to(dtype).contiguous(memory_format=torch.channels_last)


# ----------------------------------------------------------------------------- fused BN
def _nhwc(t: torch.Tensor) -> torch.Tensor:
    if t.dim() == 4:
        return t.contiguous(memory_format=torch.channels_last)
    return t.contiguous()


class _FusedBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, training, momentum,
                eps, relu):
        lib = load()
        x = _nhwc(x)
        if residual is not None:
            residual = _nhwc(residual).to(x.dtype)
        y, mean, invstd, scale_shift = lib.bn_fwd(x, residual, weight, bias, running_mean,
                                                  running_var, bool(training), float(momentum),
                                                  float(eps), bool(relu))
        # ReLU mask in backward: recomputed from x (saved scale/shift) unless a residual was
        # added before the ReLU, in which case the output y is kept instead.
        if relu and residual is None:
            ctx.save_for_backward(x, None, weight, mean, invstd, scale_shift)
        else:
            ctx.save_for_backward(x, y if relu else None, weight, mean, invstd, None)
        ctx.flags = (bool(training), bool(relu), residual is not None)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import block
        x, y, weight, mean, invstd, scale_shift = ctx.saved_tensors
        training, relu, has_res = ctx.flags
        lib = load()
        dy = _nhwc(dy).to(x.dtype)
        w, b = ctx.params
        need_w = weight is not None and ctx.needs_input_grad[2]
        need_b = ctx.needs_input_grad[3]
        # arena-managed gamma / beta: the kernel accumulates their gradients in place (as the
        # fused blocks do), no AccumulateGrad add kernels
        outs = block._bn_grad_outs(w, b) if (need_w and need_b and w is not None and
                                             b is not None) else (None, None)
        dx, dgamma, dbeta, dres = lib.bn_bwd(dy, x, y, weight, mean, invstd, scale_shift,
                                             training, relu, has_res, None, outs[0], outs[1])
        if outs[0] is not None:
            block._finish_bn(w, b, dgamma, dbeta, outs)
            return (dx, dres if has_res else None, None, None, None, None, None, None, None,
                    None)
        return (dx, dres if has_res else None, dgamma if need_w else None,
                dbeta if need_b else None, None, None, None, None, None, None)


def fused_batch_norm(x, weight, bias, running_mean, running_var, training, momentum, eps,
                     relu=False, residual=None):
    """BN → (+ residual) → (ReLU). HIP kernels for channels_last GPU tensors with C % 8 == 0,
    torch ops otherwise (CPU path, odd channel counts)."""
    use_hip = x.is_cuda and x.dim() in (2, 4) and x.size(1) % 8 == 0 and \
        x.size(1) <= MAX_BN_C and x.dtype in (h16(), torch.float32)
    if use_hip:
        return _FusedBN.apply(x, residual, weight, bias, running_mean, running_var, training,
                              momentum, eps, relu)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` (same parameters, buffers and state_dict keys) whose forward can also
    apply the residual add and the ReLU that follow it in the reference models."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, relu: bool = False, **kw):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, **kw)
        self.fuse_relu = relu

    def forward(self, x, residual=None):
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            if not getattr(self, "_shared_counter", False) or self.momentum is None:
                self.num_batches_tracked.add_(1)
            if self.momentum is None:
                momentum = 1.0 / float(self.num_batches_tracked)
        training = self.training or not self.track_running_stats
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return fused_batch_norm(x, self.weight, self.bias, rm, rv, training, momentum, self.eps,
                                relu=self.fuse_relu, residual=residual)

    def extra_repr(self):
        return super().extra_repr() + (", fused_relu=True" if self.fuse_relu else "") + \
            (f", fused_pool={self.fuse_pool}" if getattr(self, "fuse_pool", None) else "")


class FusedBNReluPool2d(FusedBatchNorm2d):
    """BN → ReLU → max-pool of a CIFAR graph net (``CIFAR10/dawn.py:23-33``: conv_bn then
    ``MaxPool2d(2)``) as ONE forward kernel after the statistics pass and one reduce + one apply
    kernel backward — the ``csrc/bn.hip`` k_stem_pool_* kernels, whose window slot byte routes the
    pooled gradient straight into the BN backward (neither the normalised activation nor the
    un-pooled gradient is ever written). Same parameters / buffers / state_dict as the BN; eval
    mode and unsupported inputs run BN+ReLU then ``F.max_pool2d``."""

    def forward(self, x, residual=None):
        k, s, p = self.fuse_pool
        if (residual is None and self.training and self.track_running_stats and x.is_cuda and
                x.dim() == 4 and x.dtype == h16() and x.size(1) % 8 == 0 and
                x.size(1) <= MAX_BN_C and self.affine and _stem_fits(*x.shape, self.fuse_pool)):
            return _StemPoolFn.apply(x, self.weight, self.bias, self, self.fuse_pool)
        y = super().forward(x, residual)
        return F.max_pool2d(y, k, s, p)


def share_bn_counters(model: nn.Module) -> nn.Module:
    """Make every BN's ``num_batches_tracked`` a view into one int64 vector, bumped by ONE kernel
    per training forward (a pre-forward hook) instead of one launch per BN layer. Call after the
    model is on its final device; buffer names / state_dict are unchanged."""
    bns = [m for m in model.modules() if isinstance(m, FusedBatchNorm2d)
           and m.track_running_stats and m.momentum is not None]
    if not bns:
        return model
    flat = torch.stack([m.num_batches_tracked.detach().reshape(()) for m in bns])
    for i, m in enumerate(bns):
        m._buffers["num_batches_tracked"] = flat[i]
        m._shared_counter = True

    def bump(mod, args):
        if mod.training:
            flat.add_(1)
    model._bn_counter = flat
    model.register_forward_pre_hook(bump)
    return model


def to_fused_bn(bn: nn.BatchNorm2d, relu: bool = False) -> FusedBatchNorm2d:
    """Re-class in place: the very same Parameter / buffer objects stay registered."""
    bn.__class__ = FusedBatchNorm2d
    bn.fuse_relu = relu
    return bn


# ----------------------------------------------------------------------------- fused ResNet
def _fused_bottleneck_forward(self, x):
    identity = x if self.downsample is None else self.downsample[1](self.downsample[0](x))
    out = self.bn1(self.conv1(x))
    out = self.bn2(self.conv2(out))
    return self.bn3(self.conv3(out), identity)


def _block_bottleneck_forward(self, x):
    """Training: the whole-block fused path (``ops/block.py``); eval / unsupported shapes: the
    per-layer fused path."""
    from . import block
    if block.block_supported(self, x):
        return block.bottleneck_forward(self, x)
    return _fused_bottleneck_forward(self, x)


def _fused_basic_forward(self, x):
    identity = x if self.downsample is None else self.downsample[1](self.downsample[0](x))
    out = self.bn1(self.conv1(x))
    return self.bn2(self.conv2(out), identity)


# The stem backward's BN statistics pass reads the pooled gradient and the pooled map (saved from
# the forward) instead of the 112x112 conv output and the slot bytes (csrc/bn.hip
# k_stem_pool_reduce_out); False (tests only) keeps the full-resolution reduce
STEM_POOLED = True


class _StemPoolFn(torch.autograd.Function):
    """conv1 output → BN (batch stats) → ReLU → max-pool as one forward kernel after the stats
    pass, and one reduce + one apply kernel backward (``csrc/bn.hip`` k_stem_pool_*)."""

    @staticmethod
    def forward(ctx, c, weight, bias, bn, geom):
        from . import block
        lib = load()
        c = c.to(h16()).contiguous(memory_format=torch.channels_last)
        block._bump(bn)
        mean, invstd, ss = lib.bn_stats(c, None, weight, bias, bn.running_mean, bn.running_var,
                                        block._bn_momentum(bn), bn.eps)
        out, idx = lib.stem_pool_fwd(c, ss, *geom)
        ctx.save_for_backward(c, idx, ss, weight, mean, invstd, out if STEM_POOLED else None)
        ctx.geom = geom
        ctx.params = (weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import block
        c, idx, ss, weight, mean, invstd, pooled = ctx.saved_tensors
        w, b = ctx.params
        dout = dout.to(h16()).contiguous(memory_format=torch.channels_last)
        outs = block._bn_grad_outs(w, b)
        dc, dg, db = load().stem_pool_bwd(dout, idx, c, ss, weight, mean, invstd, *ctx.geom,
                                          outs[0], outs[1], pooled)
        gw, gb = block._finish_bn(w, b, dg, db, outs)
        return dc, gw, gb, None, None


class _StemConvPoolFn(torch.autograd.Function):
    """The whole ResNet stem — 7x7/2 conv, BN (batch stats), ReLU, 3x3/2 max-pool — as the
    implicit-GEMM conv (4-channel image chunks, BN statistics in its epilogue) + one fused
    BN-apply/ReLU/pool kernel; backward: the fused pool/BN backward + the implicit-GEMM weight
    gradient (the image needs no gradient)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, conv, bn, geom):
        from . import block
        from .conv import conv_fwd
        lib = load()
        c, st = conv_fwd(x, block._bf16_weight(w), conv.stride, conv.padding, stats=True)
        block._bump(bn)
        mean, invstd, ss = lib.bn_stats(c, st, gamma, beta, bn.running_mean, bn.running_var,
                                        block._bn_momentum(bn), bn.eps)
        out, idx = lib.stem_pool_fwd(c, ss, *geom)
        ctx.save_for_backward(x, c, idx, ss, gamma, mean, invstd, out if STEM_POOLED else None)
        ctx.geom = geom
        ctx.conv = (tuple(conv.stride), tuple(conv.padding))
        ctx.params = (w, gamma, beta)
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import block
        from .conv import conv_dgrad, conv_wgrad
        x, c, idx, ss, gamma, mean, invstd, pooled = ctx.saved_tensors
        w, g, b = ctx.params
        dout = dout.to(h16()).contiguous(memory_format=torch.channels_last)
        outs = block._bn_grad_outs(g, b)
        if (block.FUSE_BNBWD and not ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and
                pooled is not None and ctx.geom == (3, 2, 1) and tuple(c.shape[1:]) ==
                (64, 112, 112) and tuple(x.shape[2:]) == (224, 224) and
                ctx.conv == ((2, 2), (3, 3)) and tuple(w.shape) == (64, 3, 7, 7)):
            # the pool / BN backward apply fused into the 7x7 conv's weight gradient
            # (csrc/stemfuse.hip): the 112x112 conv-output gradient is never written
            from .conv import _c4_input
            x4 = x if x.shape[1] == 4 else _c4_input(x)
            x4 = x4.to(h16()).contiguous(memory_format=torch.channels_last)
            dw, dg, db = load().stem_bwd_fused(dout, idx, c, ss, gamma, mean, invstd, *ctx.geom,
                                               outs[0], outs[1], pooled, x4)
            gg, gb = block._finish_bn(g, b, dg, db, outs)
            dw = dw.view(64, 7, 8, 4)[:, :, :7, :3].permute(0, 3, 1, 2)
            return None, block._finish_param(w, dw, block._direct(w)), gg, gb, None, None, None
        dc, dg, db = load().stem_pool_bwd(dout, idx, c, ss, gamma, mean, invstd, *ctx.geom,
                                          outs[0], outs[1], pooled)
        gg, gb = block._finish_bn(g, b, dg, db, outs)
        stride, padding = ctx.conv
        dx = None
        if ctx.needs_input_grad[0]:
            if x.shape[1] % 8 == 0:
                dx = conv_dgrad(dc, block._bf16_weight(w), tuple(x.shape[2:]), stride, padding)
            else:   # an image that requires grad (saliency maps): not a training path
                dx = torch.ops.aten.convolution_backward(
                    dc.float(), x[:, :w.shape[1]].float(), w.float(), None, list(stride),
                    list(padding), [1, 1], False, [0, 0], 1, [True, False, False])[0]
                if x.shape[1] != w.shape[1]:
                    dx = torch.cat([dx, torch.zeros_like(dx[:, :x.shape[1] - w.shape[1]])], 1)
                dx = dx.to(x.dtype)
        gw = None
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad(dc, x, tuple(w.shape), stride, padding)
            gw = block._finish_param(w, dw, block._direct(w))
        return dx, gw, gg, gb, None, None, None


def stem_conv_supported(model, x: torch.Tensor) -> bool:
    from .conv import supported
    conv, bn = model.conv1, model.bn1
    return (model.training and x.is_cuda and x.dim() == 4 and x.shape[1] in (3, 4) and
            conv.in_channels == 3 and conv.bias is None and conv.padding_mode == "zeros" and
            isinstance(conv.padding, tuple) and supported(3, conv.out_channels, conv.groups,
                                                          conv.dilation) and
            bn.affine and bn.track_running_stats and isinstance(model.maxpool, nn.MaxPool2d) and
            _pool_geom(model.maxpool) is not None and
            _stem_fits(x.shape[0], conv.out_channels,
                       (x.shape[2] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1,
                       (x.shape[3] + 2 * conv.padding[1] - conv.kernel_size[1]) // conv.stride[1] + 1,
                       _pool_geom(model.maxpool)))


def stem_conv_bn_relu_pool(x, conv: nn.Conv2d, bn: nn.BatchNorm2d, pool: nn.MaxPool2d):
    return _StemConvPoolFn.apply(x, conv.weight, bn.weight, bn.bias, conv, bn, _pool_geom(pool))


class _ReluPoolFn(torch.autograd.Function):
    """Max-pool of a post-ReLU map (``csrc/bn.hip`` k_stem_pool_fwd with an identity affine, and
    the apply pass of its backward): the backward routes the pooled gradient to the window's max
    AND applies the preceding ReLU's mask in the same kernel."""

    @staticmethod
    def forward(ctx, x, geom):
        out, idx = load().relu_pool_fwd(x, *geom)
        ctx.save_for_backward(x, idx)
        ctx.geom = geom
        return out

    @staticmethod
    def backward(ctx, dout):
        x, idx = ctx.saved_tensors
        dout = dout.to(h16()).contiguous(memory_format=torch.channels_last)
        return load().relu_pool_bwd(dout, idx, x, *ctx.geom), None


class ReluMaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` placed after a ReLU (``fuse_convs`` installs it behind a conv whose ReLU
    runs in the epilogue): HIP kernels on CUDA bf16 channels_last maps, torch otherwise."""

    def forward(self, x):
        geom = _pool_geom(self)
        if (geom is not None and x.is_cuda and x.dim() == 4 and x.dtype == h16() and
                x.size(1) % 8 == 0 and x.size(1) <= MAX_BN_C and
                x.is_contiguous(memory_format=torch.channels_last) and _stem_fits(*x.shape, geom)):
            return _ReluPoolFn.apply(x, geom)
        return super().forward(x)


def _pool_geom(pool: nn.MaxPool2d):
    def one(v):
        return v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)
    k, s, p, d = one(pool.kernel_size), one(pool.stride or pool.kernel_size), one(pool.padding), \
        one(pool.dilation)
    if None in (k, s, p) or d != 1 or pool.ceil_mode or pool.return_indices or 2 * p > k:
        return None
    return (k, s, p)


def _stem_fits(n: int, c: int, h: int, w: int, geom) -> bool:
    """The stem kernels index pixels / outputs in 32-bit arithmetic (bindings.cpp stem_geom):
    larger inputs take the unfused path instead of raising."""
    k, s, p = geom
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    return n * h * w < 2 ** 31 and n * ho * wo * (c // 8) < 2 ** 31


def stem_supported(model, c: torch.Tensor) -> bool:
    bn = model.bn1
    geom = _pool_geom(model.maxpool) if isinstance(model.maxpool, nn.MaxPool2d) else None
    return (model.training and c.is_cuda and c.dim() == 4 and c.dtype == h16() and
            c.size(1) % 8 == 0 and c.size(1) <= MAX_BN_C and bn.affine and
            bn.track_running_stats and geom is not None and _stem_fits(*c.shape, geom))


def stem_bn_relu_pool(c: torch.Tensor, bn: nn.BatchNorm2d, pool: nn.MaxPool2d) -> torch.Tensor:
    return _StemPoolFn.apply(c, bn.weight, bn.bias, bn, _pool_geom(pool))


class _GlobalAvgPoolFn(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) + flatten on a channels_last bf16 map (``csrc/nn.hip`` k_gap_*): the
    backward writes ``dy / HW`` straight into the channels_last gradient of the last block."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return load().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return load().gap_bwd(dy.contiguous(), *ctx.hw)


def global_avg_pool(x: torch.Tensor, pool: nn.Module) -> torch.Tensor:
    """``flatten(pool(x), 1)`` for ``AdaptiveAvgPool2d(1)``: the HIP kernels on a CUDA
    channels_last bf16 input with C % 8 == 0, torch otherwise."""
    if (isinstance(pool, nn.AdaptiveAvgPool2d) and pool.output_size in (1, (1, 1)) and x.is_cuda
            and x.dim() == 4 and x.dtype == h16() and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(pool(x), 1)


def _fused_resnet_forward(self, x):
    if getattr(self, "_lw_stem_c4", False) and stem_conv_supported(self, x):
        x = stem_conv_bn_relu_pool(x, self.conv1, self.bn1, self.maxpool)
    else:
        c = self.conv1(x)
        if getattr(self, "_lw_stem_fused", False) and stem_supported(self, c):
            x = stem_bn_relu_pool(c, self.bn1, self.maxpool)
        else:
            x = self.maxpool(self.bn1(c))
    x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
    return self.fc(global_avg_pool(x, self.avgpool))


def fuse_resnet(model: nn.Module, block: bool = True, mfma: bool = True) -> nn.Module:
    """Switch a ``models.resnet`` network to fused BN(+add)(+ReLU) and — with ``block`` — its
    bottlenecks to the whole-block fused MFMA path (``ops/block.py``). Parameter/buffer names and
    values are untouched; only forward changes."""
    from ..models import resnet as R
    import types
    for m in model.modules():
        if isinstance(m, R.Bottleneck):
            to_fused_bn(m.bn1, relu=True)
            to_fused_bn(m.bn2, relu=True)
            to_fused_bn(m.bn3, relu=True)
            if m.downsample is not None:
                to_fused_bn(m.downsample[1], relu=False)
            fwd = _block_bottleneck_forward if block else _fused_bottleneck_forward
            m.forward = types.MethodType(fwd, m)
        elif isinstance(m, R.BasicBlock):
            to_fused_bn(m.bn1, relu=True)
            to_fused_bn(m.bn2, relu=True)
            if m.downsample is not None:
                to_fused_bn(m.downsample[1], relu=False)
            m.forward = types.MethodType(_fused_basic_forward, m)
    if isinstance(model, R.ResNet):
        to_fused_bn(model.bn1, relu=True)
        model._lw_stem_fused = block
        model._lw_stem_c4 = block and mfma     # stem = implicit-GEMM conv on a 4-channel image
        model.forward = types.MethodType(_fused_resnet_forward, model)
    # every remaining conv (stem, eval-mode / BasicBlock paths) and the classifier on the
    # hand-written MFMA kernels (bf16 operands, fp32 accumulation); mfma=False keeps torch's
    # convs / Linear (fp32 parity checks of the BN fusion alone)
    if mfma:
        from .conv import fuse_convs
        from .gemm import fuse_linears
        fuse_convs(model)
        fuse_linears(model)
    return model


def fuse_graph_network(net: nn.Module, pool: bool = True) -> nn.Module:
    """Fuse ``bn -> relu`` node pairs of a dict-graph :class:`~..models.graph.Network` (ResNet-9,
    graph AlexNet): the BN becomes a FusedBatchNorm2d(relu=True), the ReLU node an Identity.
    Only pairs where the ReLU is the BN's sole consumer are fused; with ``pool``, a max-pool that
    is the ReLU's sole consumer is folded in too (:class:`FusedBNReluPool2d`)."""
    from ..models.graph import Identity
    graph = getattr(net, "graph", None)
    if graph is None:
        return net
    loss_of = {}                           # the loss node on the fused cross-entropy kernel
    for k, (mod, ins) in graph.items():
        if type(mod) is nn.CrossEntropyLoss:
            mod.__class__ = FusedCrossEntropyLoss
            loss_of[tuple(ins)] = mod
    # a top-1 "correct" node on the same (logits, target) as a fused loss reads the loss kernel's
    # correctness instead of its own max-reduce + compare
    from ..models.graph import Correct
    for k, (mod, ins) in list(graph.items()):
        if type(mod) is Correct and tuple(ins) in loss_of:
            cm = _XentCorrect(loss_of[tuple(ins)])
            graph[k] = (cm, ins)
            net._modules[k] = cm
    names = list(graph)
    consumers = {}
    for k, (_, ins) in graph.items():
        for i in ins:
            consumers.setdefault(i, []).append(k)
    for k in names:
        mod, _ = graph[k]
        if not isinstance(mod, nn.BatchNorm2d) or isinstance(mod, FusedBatchNorm2d):
            continue
        users = consumers.get(k, [])
        if len(users) != 1:
            continue
        r = users[0]
        rmod, rins = graph[r]
        if isinstance(rmod, nn.ReLU) and rins == [k]:
            to_fused_bn(mod, relu=True)
            ident = Identity()
            graph[r] = (ident, rins)
            net._modules[r] = ident
            # BN+ReLU whose only consumer is a max-pool: the pool joins the BN kernel pair
            pu = consumers.get(r, [])
            if pool and len(pu) == 1:
                pmod, pins = graph[pu[0]]
                geom = _pool_geom(pmod) if isinstance(pmod, nn.MaxPool2d) else None
                if geom is not None and pins == [r]:
                    mod.__class__ = FusedBNReluPool2d
                    mod.fuse_pool = geom
                    pid = Identity()
                    graph[pu[0]] = (pid, pins)
                    net._modules[pu[0]] = pid
    # a max-pool of a map that is already non-negative (post-ReLU, or a sum of post-ReLU maps:
    # the graph AlexNet's last pool after layer4's BN-ReLU-pool, ResNet-9's after its residual
    # add): the relu-pool kernels (their ReLU mask is a no-op on x >= 0) instead of ATen's
    # max-pool forward / backward and the zero fill the latter needs
    from ..models.graph import Add

    def nonneg(node, depth=0):
        if node not in graph or depth > 16:
            return False
        m, ins_ = graph[node]
        if isinstance(m, FusedBatchNorm2d):
            return bool(m.fuse_relu)
        if isinstance(m, (ReluMaxPool2d, nn.ReLU)):
            return True
        if isinstance(m, (Identity, nn.MaxPool2d)) and len(ins_) == 1:
            return nonneg(ins_[0], depth + 1)
        if isinstance(m, Add):
            return all(nonneg(i, depth + 1) for i in ins_)
        return False

    for k in names:
        mod, ins = graph[k]
        if type(mod) is nn.MaxPool2d and len(ins) == 1 and _pool_geom(mod) is not None and \
                nonneg(ins[0]):
            mod.__class__ = ReluMaxPool2d
    return net


# ----------------------------------------------------------------------------- fused loss
class _XentFn(torch.autograd.Function):
    """Softmax cross-entropy + top-1/top-5 correctness in one HIP kernel (``csrc/nn.hip`` k_xent):
    the forward already writes the unscaled logit gradient (softmax - onehot); backward only
    scales it by the incoming gradient / the valid-target count (device tensors: no host sync)."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, reduction):
        lg = logits.detach().float().contiguous()
        rows, corr, grad = load().xent(lg, target.contiguous(), 1.0, int(ignore_index),
                                       bool(logits.requires_grad))
        ctx.reduction = reduction
        ctx.dtype = logits.dtype
        if reduction == "mean":
            # mean and valid count in one launch (csrc/nn.hip k_xent_mean)
            loss, n = load().xent_mean(rows, target.contiguous(), int(ignore_index))
        elif reduction == "sum":
            n = None
            loss = rows.sum()
        else:
            n = None
            loss = rows
        ctx.save_for_backward(grad, n)
        ctx.mark_non_differentiable(corr)
        return loss, corr

    @staticmethod
    def backward(ctx, gl, _gc):
        grad, n = ctx.saved_tensors
        if ctx.reduction == "none":
            g = grad * gl.view(-1, 1)
        elif ctx.reduction == "mean":
            if gl.is_cuda and gl.dtype == torch.float32 and gl.numel() == 1:
                g = load().xent_scale(grad, gl.reshape(1), n)       # (k_xent_scale)
            else:
                g = grad * (gl / n)
        else:
            g = grad * gl
        return g.to(ctx.dtype), None, None, None


def fused_cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                        reduction: str = "mean"):
    """(loss, correct[B, 2]) — correct[:, 0] / [:, 1]: the target is the top-1 / within the
    top-5 logits (strictly-greater rank < k). GPU fp32/bf16 [B, C] logits with int64 targets;
    torch ops elsewhere."""
    if logits.is_cuda and logits.dim() == 2 and target.dim() == 1 and \
            target.dtype == torch.int64 and reduction in ("mean", "sum", "none"):
        return _XentFn.apply(logits, target, ignore_index, reduction)
    loss = F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction)
    k = min(5, logits.shape[1])
    top = logits.topk(k, 1).indices
    ok = top.eq(target.view(-1, 1))
    corr = torch.stack([ok[:, 0].float(), ok.any(1).float()], 1)
    return loss, corr


def fuse_dict_losses(model: nn.Module) -> nn.Module:
    """A CIFAR nn.Module model's ``loss = (CrossEntropyLoss, Correct)`` heads
    (models/cifar.py _DictLossMixin: VGG-16, the module AlexNet) on the fused cross-entropy
    kernel, the correctness read from it (as fuse_graph_network does for the graph nets)."""
    from ..models.graph import Correct
    heads = getattr(model, "loss", None)
    if isinstance(heads, tuple) and len(heads) == 2 and type(heads[0]) is nn.CrossEntropyLoss \
            and type(heads[1]) is Correct:
        heads[0].__class__ = FusedCrossEntropyLoss
        model.loss = (heads[0], _XentCorrect(heads[0]))
    return model


class _XentCorrect(nn.Module):
    """``Correct`` (argmax == target) of a graph whose loss node runs the fused kernel on the same
    inputs: that kernel's top-1 column (one compare launch instead of a max-reduce and an equality;
    the graph runs the loss node first). A tie at the maximum counts as correct here (no logit
    strictly greater than the target's), where argmax picks the first maximal index."""

    def __init__(self, loss: "FusedCrossEntropyLoss"):
        super().__init__()
        self.__dict__["_loss"] = loss      # (not a submodule: no second state_dict entry)

    def forward(self, classifier, target):
        corr = getattr(self._loss, "last_correct", None)
        if corr is None or corr.shape[0] != target.shape[0]:
            return classifier.max(dim=1)[1] == target
        return corr[:, 0] > 0


class FusedCrossEntropyLoss(nn.CrossEntropyLoss):
    """``nn.CrossEntropyLoss`` on the fused kernel (no class weights / label smoothing); the
    per-sample top-1/top-5 correctness of the last call is kept in ``last_correct`` ([B, 2]) so a
    training loop needs no separate ``topk`` pass."""

    def forward(self, input, target):
        if self.weight is None and self.label_smoothing == 0.0:
            loss, corr = fused_cross_entropy(input, target, self.ignore_index, self.reduction)
            self.last_correct = corr
            return loss
        self.last_correct = None
        return super().forward(input, target)
