"""MFMA GEMM (``csrc/gemm.hip``) and the layers built on it.

``MFMALinear`` is an ``nn.Linear`` (same parameters / state_dict) whose forward is
``relu?(x·Wᵀ + b)`` in ONE kernel (bias and ReLU in the epilogue) and whose backward runs the
data-gradient ``dy·W`` and the weight-gradient ``dyᵀ·x`` (split-K, fp32 output written straight
into the fp32 master gradient) on the same kernel family — no transpose copies: the kernel reads
M/N-contiguous operands through the gfx950 transposing LDS read.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from ._ext import h16, load
from .tuning import Tuner, with_mf32


def _splits(tiles: int, K: int) -> int:
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, K // 256 if K >= 512 else 1)))


TILES = {"auto": 0, "128x128x32": 1, "128x128x64": 2, "256x64x32": 3, "64x256x32": 4,
         "256x64x64": 5, "64x64x64": 6, "256x256x64": 21, "256x128x64": 22}
# the 32x32x16-MFMA twins of tiles 1..6 (csrc GemmTile id + 40), e.g. "128x128x64/mf32"
TILES.update({f"{k}/mf32": v + 40 for k, v in list(TILES.items()) if 1 <= v <= 6})


def gemm(A, lda, a_kc, B, ldb, b_kc, M, N, K, bias=None, relu=False, splits=1, out_bf16=True):
    return load().gemm(A, lda, a_kc, B, ldb, b_kc, M, N, K, bias, relu, splits, out_bf16)


def gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, bias=None, relu=False, splits=1, out_bf16=True,
            tile="auto", pro_scale=None, pro_shift=None, pro_on_a=True, stats=False):
    """Full-featured entry: explicit tile, prologue ``relu(v*scale+shift)`` (per-k of a
    K-contiguous A, or per-n of an N-contiguous B) and per-column output statistics
    ``[tiles_m][2][N]`` (Σv, Σv² of the stored values per M-tile). Returns ``(C, stats)``."""
    return load().gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, bias, relu, splits, out_bf16,
                          TILES[tile] if isinstance(tile, str) else int(tile), pro_scale,
                          pro_shift, pro_on_a, stats)


class LinearTuner(Tuner):
    """First sight of a Linear GEMM problem: time every (tile, split-K) candidate with HIP events
    on scratch outputs and keep the fastest (``LWAAAI_GEMM_TUNE=0``: the 128x128 heuristic;
    ``LWAAAI_TUNE_FILE`` pins the choices, ``ops/tuning.py``). The classifier GEMMs are skinny in
    M (batch 256-512) and span K = 1k-25k, so the right tile and split count differ per layer and
    pass (``profiles/r2_linear_vs_blas*.log``)."""

    TILES = with_mf32((1, 2, 3, 4, 5, 6))
    BIG = (21, 22)                    # 8-wave LDS-DMA tiles: K-/K-, K-/N- or M-/N-contiguous operands
    SPLITS = (1, 2, 4, 8, 16)

    def __init__(self):
        super().__init__("linear", "LWAAAI_GEMM_TUNE")

    def pick(self, key, tiles_of, K, run, big=False):
        default = (0, _splits(tiles_of(128, 128), K))
        cands = [(t, sp) for t in self.TILES + (self.BIG if big else ()) for sp in self.SPLITS
                 if sp == 1 or K // sp >= 256]
        return super().pick(key, lambda c: run(*c), cands, default)


TUNER = LinearTuner()


def _tiles(M: int, N: int):
    return lambda bm, bn: -(-M // bm) * -(-N // bn)


def _gemm_tuned(kind, A, lda, a_kc, B, ldb, b_kc, M, N, K, bias=None, relu=False,
                out_bf16=True, out=None, accumulate=False):
    """One Linear GEMM on the tuned (tile, splits); ``out``/``accumulate``: fp32 C += result
    (the tuner times on scratch outputs, never on ``out``)."""
    lib = load()

    def run(t, sp, dst=None, acc=False):
        return lib.gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, bias, relu, sp, out_bf16, t, None,
                           None, True, False, dst, None, acc, 0, None)[0]
    key = (kind, M, N, K, bias is not None, relu, out_bf16)
    big = (a_kc and b_kc and K % 8 == 0) or (not a_kc and not b_kc and M % 8 == 0 and N % 8 == 0) \
        or (a_kc and not b_kc and K % 8 == 0 and N % 8 == 0 and ldb % 8 == 0)
    t, sp = TUNER.pick(key, _tiles(M, N), K, run, big=big)
    return run(t, sp, out, accumulate)


def linear_fwd(x2, w, bias=None, relu=False, out_fp32=False):
    """x2 [M,K] bf16, w [N,K] bf16 -> [M,N] bf16 (or fp32) = relu?(x2·wᵀ + bias)."""
    M, K = x2.shape
    N = w.shape[0]
    return _gemm_tuned("fwd", x2, K, True, w, K, True, M, N, K, bias, relu, not out_fp32)


def linear_dgrad(dy2, w):
    """dy2 [M,N], w [N,K] -> dx [M,K] bf16 = dy2·w."""
    M, N = dy2.shape
    K = w.shape[1]
    return _gemm_tuned("dgrad", dy2, N, True, w, K, False, M, K, N)


def linear_wgrad(dy2, x2, out=None):
    """dy2 [M,N], x2 [M,K] -> dW [N,K] fp32 = dy2ᵀ·x2 (reduction over the batch, split-K);
    ``out``: accumulate into that fp32 [N,K] buffer (the gradient arena) instead."""
    M, N = dy2.shape
    K = x2.shape[1]
    return _gemm_tuned("wgrad", dy2, N, False, x2, K, False, N, K, M, out_bf16=False, out=out,
                       accumulate=out is not None)


def _pad_rows(w: torch.Tensor, n: int) -> torch.Tensor:
    """[N, K] → [n, K] with zero rows (the GEMM's N and its 16-byte stores need N % 8 == 0)."""
    if w.shape[0] == n:
        return w
    out = torch.zeros((n, w.shape[1]), dtype=w.dtype, device=w.device)
    out[:w.shape[0]].copy_(w)
    return out


def _relu_bias_native(ctx, dyf, y, dense_y: bool):
    """ReLU mask + bias gradient of a bf16 [M, N] linear output in one native pass
    (csrc/nn.hip k_relu_bias_bwd), an arena-managed bias accumulated in place (no AccumulateGrad
    add): (masked dy, db or None), or None where it does not apply (fp32 dy, odd widths, a sliced
    padded output) and the torch ops run instead."""
    from .conv import _bias_arena_view
    need_db = ctx.has_bias and ctx.needs_input_grad[2]
    N = dyf.shape[1]
    if not (ctx.relu or need_db) or not dyf.is_cuda or dyf.dtype != h16() or not dense_y or \
            N % 8 != 0 or not (N <= 2048 or N % 2048 == 0) or N > 16384:
        return None
    dyc = dyf.contiguous()
    b = ctx.bias
    dst = _bias_arena_view(b) if need_db else None
    dym, db = load().relu_bias_bwd(dyc, y.contiguous() if ctx.relu else None, dst)
    if dst is not None:
        b._lw_grad_ready(b)
        db = None
    elif not need_db:
        db = None
    return dym, db


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu, out_fp32=False):
        from .block import _bf16_weight
        shp = x.shape
        N, K = weight.shape
        Np = N + (-N) % 8                       # e.g. a 10-way classifier runs as 16 columns
        x2 = x.reshape(-1, shp[-1]).to(h16()).contiguous()
        w = _pad_rows(_bf16_weight(weight).contiguous(), Np)
        b = None
        if bias is not None:
            b = bias.float() if Np == N else torch.cat([bias.float(),
                                                        bias.new_zeros(Np - N).float()])
        y = linear_fwd(x2, w, b, relu, out_fp32)
        if Np != N:
            y = y[:, :N]
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu, ctx.has_bias, ctx.shape, ctx.N, ctx.Np = relu, bias is not None, shp, N, Np
        ctx.weight = weight
        ctx.bias = bias
        return y.reshape(*shp[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        N, Np = ctx.N, ctx.Np
        dyf = dy.reshape(-1, N)
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        done = _relu_bias_native(ctx, dyf, y, N == Np)
        if done is not None:
            dyf, db = done
        else:
            if ctx.relu:
                dyf = dyf * (y > 0)
            # the bias gradient from dy as it arrives (fp32 for an fp32-output classifier: a bf16
            # dy makes many logits' bias gradients exactly equal — Top-K ties at the threshold)
            db = dyf.float().sum(0) if need_db else None
        dy2 = dyf.to(h16())
        if Np != N:
            dy2 = torch.cat([dy2, dy2.new_zeros(dy2.shape[0], Np - N)], 1)
        dy2 = dy2.contiguous()
        dx = linear_dgrad(dy2, w).reshape(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = None
        p = ctx.weight
        if ctx.needs_input_grad[1]:
            g = p.grad if getattr(p, "_lw_grad_ready", None) is not None else None
            if g is not None and Np == N and g.dtype == torch.float32 and g.is_contiguous():
                # fp32 weight gradient accumulated straight into the gradient arena (split-K)
                linear_wgrad(dy2, x2, out=g)
                p._lw_grad_ready(p)
            else:
                dw = linear_wgrad(dy2, x2)[:N].to(p.dtype)
        return dx, dw, db, None, None


class _ReplicatedLinearFn(torch.autograd.Function):
    """``Linear(W)`` applied to an input whose every feature is repeated ``reps`` times, as
    ``flatten(AdaptiveAvgPool2d((7, 7))(x))`` makes it when ``x`` is 1x1 spatially (CIFAR VGG-16:
    ``CIFAR10/vgg16.py:10-94``; 512 features repeated 49 times into fc1's 25088 inputs). Exactly
    the same layer: ``W · rep(x) = (Σ_r W[:, c, r]) · x``, so the forward and data-gradient GEMMs run
    on the folded ``[O][C]`` weight (49x fewer FLOPs), and the weight gradient — ``dy ⊗ x``, the
    same for every repeat — is computed once and added to each repeat's slice of the arena."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu, reps):
        from .block import _bf16_weight
        O, K = weight.shape
        C = K // reps
        wb = _bf16_weight(weight)                                  # [O][C*reps] 16-bit mirror
        weff = load().sum_repeats(wb.contiguous(), reps).view(O, C)    # one HBM pass (nn.hip)
        x2 = x.reshape(-1, C).to(h16()).contiguous()
        b = bias.float() if bias is not None else None
        y = linear_fwd(x2, weff, b, relu)
        ctx.save_for_backward(x2, weff, y if relu else None)
        ctx.weight, ctx.reps, ctx.relu, ctx.has_bias = weight, reps, relu, bias is not None
        ctx.bias = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, weff, y = ctx.saved_tensors
        p, reps = ctx.weight, ctx.reps
        done = _relu_bias_native(ctx, dy, y, True)
        if done is not None:
            dyf, db = done
        else:
            dyf = dy * (y > 0) if ctx.relu else dy
            db = dyf.float().sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        dy2 = dyf.to(h16()).contiguous()
        dx = linear_dgrad(dy2, weff) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            g1 = linear_wgrad(dy2, x2)                             # [O][C] fp32
            O, C = g1.shape
            g = p.grad if getattr(p, "_lw_grad_ready", None) is not None else None
            if g is not None and g.dtype == torch.float32 and g.is_contiguous():
                claim = getattr(p, "_lw_grad_overwrite", None)
                # the only contribution this step and the arena slice was not zeroed: one write
                # pass instead of zero + read + write (engine.claim_overwrite); nn.hip
                # k_repeat_store either way (the broadcast add / copy ran ATen's generic
                # strided kernel)
                load().repeat_store(g1.reshape(-1), g.view(-1), reps,
                                    not (claim is not None and claim()))
                p._lw_grad_ready(p)
            else:
                dw = g1.unsqueeze(-1).expand(O, C, reps).reshape(O, C * reps).to(p.dtype)
        return dx, dw, db, None, None


def replicated_linear(x, lin, reps: int):
    """``lin(x.repeat_interleave(reps, dim=1))`` for an MFMALinear ``lin`` (see
    :class:`_ReplicatedLinearFn`); ``x`` is [B, C] with ``C * reps == lin.in_features``."""
    return _ReplicatedLinearFn.apply(x, lin.weight, lin.bias, bool(getattr(lin, "fuse_relu",
                                                                           False)), reps)


def mfma_linear(x, weight, bias=None, relu=False, out_fp32=False):
    """Every GPU Linear runs on the MFMA GEMM. The kernels move K in 16-byte chunks, so an
    in_features that is not a multiple of 8 is zero-padded on both operands (the padded products
    are exact zeros; autograd slices the padding off the gradients). The CPU path (tests, the
    CPU mirror of a model) is torch's."""
    if x.is_cuda:
        K = weight.shape[1]
        if K % 8:
            kp = -(-K // 8) * 8
            x = F.pad(x, (0, kp - K))
            weight = F.pad(weight, (0, kp - K))
        return _LinearFn.apply(x, weight, bias, relu, out_fp32)
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


class MFMALinear(nn.Linear):
    """nn.Linear on the hand-written MFMA GEMM; ``fuse_relu`` applies the following ReLU in the
    epilogue (VGG / AlexNet classifiers)."""

    def __init__(self, in_features, out_features, bias=True, fuse_relu=False, out_fp32=False,
                 **kw):
        super().__init__(in_features, out_features, bias, **kw)
        self.fuse_relu = fuse_relu
        self.out_fp32 = out_fp32

    def forward(self, x):
        return mfma_linear(x, self.weight, self.bias, self.fuse_relu,
                           getattr(self, "out_fp32", False))


def to_mfma_linear(m: nn.Linear, fuse_relu=False, out_fp32=False) -> MFMALinear:
    m.__class__ = MFMALinear
    m.fuse_relu = fuse_relu
    m.out_fp32 = out_fp32
    return m


def fuse_linears(model: nn.Module) -> nn.Module:
    """Switch every nn.Linear of ``model`` to MFMALinear; inside nn.Sequential, a Linear directly
    followed by a ReLU gets the ReLU fused (the ReLU becomes Identity)."""
    for mod in model.modules():
        if isinstance(mod, nn.Sequential):
            kids = list(mod._modules.items())
            for i, (name, child) in enumerate(kids):
                if type(child) is nn.Linear:
                    relu_next = i + 1 < len(kids) and isinstance(kids[i + 1][1], nn.ReLU)
                    to_mfma_linear(child, fuse_relu=relu_next)
                    if relu_next:
                        mod._modules[kids[i + 1][0]] = nn.Identity()
    for mod in model.modules():
        if type(mod) is nn.Linear:
            to_mfma_linear(mod)
    # the model's last Linear (the classifier) produces fp32 logits: the loss reads them in fp32
    # anyway, and its gradient — the classifier bias gradient — stays fp32
    last = [m for m in model.modules() if isinstance(m, MFMALinear)]
    if last and not last[-1].fuse_relu:
        last[-1].out_fp32 = True
    return model
