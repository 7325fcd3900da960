"""Reference-semantics compressor oracles (pure PyTorch, dense in -> dense out).

These are executable restatements of the per-tensor compressors of the AAAI-20 reference
(``CIFAR10/core.py:178-215`` and the copy in ``IMAGENET/training/train_imagenet_nv.py:258-295``),
kept bit-for-bit faithful in *selection* semantics so that the HIP kernels and the sparse /
quantised wire formats of this framework can be tested against them.

Every oracle takes a flat 1-D tensor ``g`` (one layer in layer-wise mode, the concatenated model
in entire-model mode) and returns a dense tensor of the same length whose dropped entries are 0.
The all-reduce that follows in the reference (``core.py:217-225``) means the final gradient is the
mean over ranks of these per-rank dense vectors; :func:`mean_over_ranks` states that.

Deliberate, documented deviations from the reference:
  * TernGrad / RandomDithering of an all-zero tensor return zeros instead of NaN (0/0).
  * ``Topk`` with ``K >= 1`` keeps everything instead of raising (``kthvalue(0)``).
  * Random numbers come from an explicit ``torch.Generator`` so tests are reproducible; the
    kernels use counter-based Philox and are therefore compared statistically, not bitwise.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

METHODS = ("none", "Topk", "Randomk", "Thresholdv", "AdaptiveThreshold", "TernGrad",
           "RandomDithering")

# Spellings used by the reference READMEs and notebooks.
ALIASES = {
    "topk": "Topk", "TopK": "Topk", "top_k": "Topk",
    "randomk": "Randomk", "RandomK": "Randomk", "randk": "Randomk",
    "thresholdv": "Thresholdv", "ThresholdV": "Thresholdv", "threshold": "Thresholdv",
    "adaptivethreshold": "AdaptiveThreshold", "adaptive": "AdaptiveThreshold",
    "terngrad": "TernGrad", "Terngrad": "TernGrad",
    "randomdithering": "RandomDithering", "QSGD": "RandomDithering", "qsgd": "RandomDithering",
    "None": "none", "": "none", None: "none",
}


def canonical_method(method) -> str:
    """Map a user spelling to a canonical method name; unknown names raise (D17)."""
    if method in METHODS:
        return method
    if method in ALIASES:
        return ALIASES[method]
    raise ValueError(f"unknown compression method {method!r}; expected one of {METHODS} "
                     f"or an alias {sorted(k for k in ALIASES if isinstance(k, str))}")


def topk_keep_count(n: int, K: float) -> int:
    """Guaranteed number of kept elements of the reference Top-K rule.

    The reference computes ``thr = kthvalue(|g|, ceil(n(1-K)))`` and keeps ``|g| >= thr``
    (``core.py:180-183``). Without ties that keeps ``n - ceil(n(1-K)) + 1`` elements, which is
    ``nK + 1`` when ``nK`` is integral and is always >= 1.
    """
    if n <= 0:
        return 0
    if K >= 1.0:
        return n
    kk = math.ceil(n * (1.0 - K))
    kk = min(max(kk, 1), n)
    return n - kk + 1


def randomk_keep_count(n: int, K: float) -> int:
    """``randperm(n).lt(n*K)`` keeps exactly ``ceil(n*K)`` elements (``core.py:186``)."""
    if n <= 0:
        return 0
    return min(n, max(0, math.ceil(n * K)))


def topk(g: torch.Tensor, K: float) -> torch.Tensor:
    n = g.numel()
    if n == 0:
        return g.clone()
    if K >= 1.0:
        return g.clone()
    a = g.abs()
    kk = min(max(math.ceil(n * (1.0 - K)), 1), n)
    thr, _ = a.float().kthvalue(kk)
    out = g.clone()
    out[a < thr.to(a.dtype)] = 0
    return out


def randomk(g: torch.Tensor, K: float, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    n = g.numel()
    mask = torch.randperm(n, generator=generator, device="cpu").to(g.device).lt(n * K)
    return g * mask.to(g.dtype)


def thresholdv(g: torch.Tensor, V: float) -> torch.Tensor:
    out = g.clone()
    out[g.abs() < V] = 0
    return out


def adaptive_threshold(g: torch.Tensor) -> torch.Tensor:
    if g.numel() == 0:
        return g.clone()
    H = g * 2
    gmax = g.abs().max()
    out = g.clone()
    out[H.abs() < gmax] = 0
    return out


def terngrad(g: torch.Tensor, generator: Optional[torch.Generator] = None,
             uniform: Optional[torch.Tensor] = None) -> torch.Tensor:
    if g.numel() == 0:
        return g.clone()
    a = g.abs()
    maxval = a.max()
    if maxval == 0:
        return torch.zeros_like(g)
    prob = a / maxval
    if uniform is None:
        uniform = torch.rand(g.shape, generator=generator, dtype=torch.float32).to(g.device)
    b = (uniform.to(prob.dtype) < prob).to(g.dtype)
    return g.sign() * maxval * b


def random_dithering(g: torch.Tensor, qstates: int, generator: Optional[torch.Generator] = None,
                     uniform: Optional[torch.Tensor] = None) -> torch.Tensor:
    if g.numel() == 0:
        return g.clone()
    norm = torch.norm(g.float())
    if norm == 0:
        return torch.zeros_like(g)
    if uniform is None:
        uniform = torch.rand(g.shape, generator=generator, dtype=torch.float32).to(g.device)
    level = torch.floor(g.abs().float() / norm * qstates + uniform)
    out = g.float().sign() * norm * (level / qstates)
    out = torch.where(torch.isinf(out), torch.zeros_like(out), out)
    return out.to(g.dtype)


def compress(g: torch.Tensor, method, K=None, V=None, qstates=None,
             generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Dispatch exactly like the reference ``if/elif`` chain (``core.py:178-215``).

    Note the reference's falsy guards: ``Topk``/``Randomk`` with ``K`` falsy, ``Thresholdv`` with
    ``V`` falsy and ``RandomDithering`` with ``qstates`` falsy all mean "no compression".
    """
    method = canonical_method(method)
    if method == "Topk" and K:
        return topk(g, K)
    if method == "Randomk" and K:
        return randomk(g, K, generator)
    if method == "Thresholdv" and V:
        return thresholdv(g, V)
    if method == "AdaptiveThreshold":
        return adaptive_threshold(g)
    if method == "TernGrad":
        return terngrad(g, generator)
    if method == "RandomDithering" and qstates:
        return random_dithering(g, qstates, generator)
    return g.clone()


def mean_over_ranks(per_rank: list) -> torch.Tensor:
    """What ``all_reduce(SUM)`` then ``/= world_size`` produces (``core.py:217-225``)."""
    acc = per_rank[0].clone()
    for t in per_rank[1:]:
        acc += t
    return acc / float(len(per_rank))
