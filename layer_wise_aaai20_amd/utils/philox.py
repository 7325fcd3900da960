"""Philox4x32-10 in numpy, bit-identical to ``csrc/common.h::philox4x32_10``.

Used by the CPU (gloo) implementation of the Random-K selection and of the TernGrad / QSGD dither so
that CPU and GPU choose the same masks / codes for the same (seed, step, segment, index). The
reference instead draws ``torch.randperm`` / ``torch.rand`` from the global generator
(``CIFAR10/core.py:186, 204, 210``), which is only rank-coherent when every rank is seeded alike
(``train_imagenet_nv.py:118``); counter-based draws make coherence a property of the key.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

TAG_RANDK = 1 << 24
TAG_TERNGRAD = 2 << 24
TAG_QSGD = 3 << 24


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised over arrays of counters; returns four uint32 arrays."""
    x = [np.asarray(c, dtype=np.uint64) & MASK32 for c in (c0, c1, c2, c3)]
    x = list(np.broadcast_arrays(*x))
    x = [a.copy() for a in x]
    ka = np.uint64(k0 & 0xFFFFFFFF)
    kb = np.uint64(k1 & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * x[0]
        p1 = M1 * x[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        x = [(hi1 ^ x[1] ^ ka) & MASK32, lo1, (hi0 ^ x[3] ^ kb) & MASK32, lo0]
        ka = (ka + np.uint64(W0)) & MASK32
        kb = (kb + np.uint64(W1)) & MASK32
    return [a.astype(np.uint32) for a in x]


def stream_words(n: int, gid: int, step: int, tag: int, seed: int) -> np.ndarray:
    """Word i of the stream = output (i % 4) of philox(counter=(i//4, gid, step, tag))."""
    if n == 0:
        return np.zeros(0, dtype=np.uint32)
    q = np.arange((n + 3) // 4, dtype=np.uint64)
    r = philox4x32_10(q, gid, step, tag, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return np.stack(r, axis=1).reshape(-1)[:n]


def randk_keys(n: int, gid: int, step: int, seed: int) -> np.ndarray:
    """31-bit odd selection keys of Random-K (``compress.hip::randk_key4``)."""
    w = stream_words(n, gid, step, TAG_RANDK, seed)
    return (w >> np.uint32(1)) | np.uint32(1)


def uniforms(n: int, gid: int, step: int, tag: int, seed: int) -> np.ndarray:
    """fp32 uniforms in [0,1) with 24 random bits (``common.h::u01``)."""
    w = stream_words(n, gid, step, tag, seed)
    return (w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
