"""MFMA GEMM (``csrc/gemm.hip``) and the layers built on it.

``MFMALinear`` is an ``nn.Linear`` (same parameters / state_dict) whose forward is
``relu?(x·Wᵀ + b)`` in ONE kernel (bias and ReLU in the epilogue) and whose backward runs the
data-gradient ``dy·W`` and the weight-gradient ``dyᵀ·x`` (split-K, fp32 output written straight
into the fp32 master gradient) on the same kernel family — no transpose copies: the kernel reads
M/N-contiguous operands through the gfx950 transposing LDS read.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ._ext import load


def _splits(tiles: int, K: int) -> int:
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, K // 256 if K >= 512 else 1)))


TILES = {"auto": 0, "128x128x32": 1, "128x128x64": 2, "256x64x32": 3, "64x256x32": 4,
         "256x64x64": 5, "64x64x64": 6}


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


def linear_fwd(x2, w, bias=None, relu=False):
    """x2 [M,K] bf16, w [N,K] bf16 -> [M,N] bf16 = relu?(x2·wᵀ + bias)."""
    M, K = x2.shape
    N = w.shape[0]
    tiles = -(-M // 128) * -(-N // 128)
    return gemm(x2, K, True, w, K, True, M, N, K, bias, relu, _splits(tiles, K), True)


def linear_dgrad(dy2, w):
    """dy2 [M,N], w [N,K] -> dx [M,K] bf16 = dy2·w."""
    M, N = dy2.shape
    K = w.shape[1]
    tiles = -(-M // 128) * -(-K // 128)
    return gemm(dy2, N, True, w, K, False, M, K, N, None, False, _splits(tiles, N), True)


def linear_wgrad(dy2, x2):
    """dy2 [M,N], x2 [M,K] -> dW [N,K] fp32 = dy2ᵀ·x2 (reduction over the batch, split-K)."""
    M, N = dy2.shape
    K = x2.shape[1]
    tiles = -(-N // 128) * -(-K // 128)
    return gemm(dy2, N, False, x2, K, False, N, K, M, None, False, _splits(tiles, M), False)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(torch.bfloat16).contiguous()
        w = weight.to(torch.bfloat16).contiguous()
        y = linear_fwd(x2, w, bias.float() if bias is not None else None, relu)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu, ctx.has_bias, ctx.shape = relu, bias is not None, shp
        ctx.wdtype = weight.dtype
        return y.reshape(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).to(torch.bfloat16)
        if ctx.relu:
            dy2 = dy2 * (y > 0)
        dy2 = dy2.contiguous()
        dx = linear_dgrad(dy2, w).reshape(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(dy2, x2).to(ctx.wdtype) if ctx.needs_input_grad[1] else None
        db = dy2.float().sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None


def _gemm_ok(x, weight):
    K, N = weight.shape[1], weight.shape[0]
    return x.is_cuda and K % 8 == 0 and N % 8 == 0


def mfma_linear(x, weight, bias=None, relu=False):
    if _gemm_ok(x, weight):
        return _LinearFn.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


class MFMALinear(nn.Linear):
    """nn.Linear on the hand-written MFMA GEMM; ``fuse_relu`` applies the following ReLU in the
    epilogue (VGG / AlexNet classifiers)."""

    def __init__(self, in_features, out_features, bias=True, fuse_relu=False, **kw):
        super().__init__(in_features, out_features, bias, **kw)
        self.fuse_relu = fuse_relu

    def forward(self, x):
        return mfma_linear(x, self.weight, self.bias, self.fuse_relu)


def to_mfma_linear(m: nn.Linear, fuse_relu=False) -> MFMALinear:
    m.__class__ = MFMALinear
    m.fuse_relu = fuse_relu
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
    return model
