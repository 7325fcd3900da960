"""Shared kernel-choice tuner with an optional persisted table.

The GEMM (``ops/block.py``), Linear (``ops/gemm.py``) and convolution (``ops/conv.py``) tuners
time every candidate kernel (tile, or (tile, split-K)) the first time a problem shape is seen and
keep the fastest, as MIOpen's find mode does for the reference's cuDNN/MIOpen convolutions
(``IMAGENET/training/train_imagenet_nv.py:36`` sets ``cudnn.benchmark``). Timing noise can make
two processes pick different kernels for the same shape, and different kernels round differently.
``LWAAAI_TUNE_FILE=path`` pins the choices:

* at import the table is read (JSON: ``{"<tuner>|<key repr>": choice}``) and every entry in it
  is used instead of timing;
* a new decision is added to the table and, on rank 0 (``RANK`` unset or 0), written back
  atomically, so a second run — or every rank of a multi-process run pointed at a file tuned
  beforehand — makes exactly the same choices.
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, Sequence

import torch

_FILE = os.environ.get("LWAAAI_TUNE_FILE", "")
_TABLE: Dict[str, object] = {}
if _FILE and os.path.exists(_FILE):
    with open(_FILE) as f:
        _TABLE = json.load(f)


def _encode(v):
    return list(v) if isinstance(v, tuple) else v


def _decode(v):
    return tuple(v) if isinstance(v, list) else v


def _save() -> None:
    if not _FILE or os.environ.get("RANK", "0") != "0":
        return
    tmp = f"{_FILE}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(_TABLE, f, indent=0, sort_keys=True)
    os.replace(tmp, _FILE)


def table() -> Dict[str, object]:
    """The persisted choices (read-only view for tests / tools)."""
    return dict(_TABLE)


class Tuner:
    """Time each candidate ``run(c)`` (one warm-up call, then ``reps`` timed calls with HIP
    events) on first sight of ``key`` and keep the fastest; ``env`` names the switch that turns
    timing off (the ``default`` choice is used then)."""

    def __init__(self, name: str, env: str, reps: int = 3):
        self.name = name
        self.reps = reps
        self.best: Dict[tuple, object] = {}
        self.enabled = os.environ.get(env, "1") != "0"

    def _tkey(self, key) -> str:
        return f"{self.name}|{key!r}"

    def pick(self, key, run: Callable, candidates: Sequence, default):
        c = self.best.get(key)
        if c is not None:
            return c
        pinned = _TABLE.get(self._tkey(key))
        if pinned is not None:
            c = _decode(pinned)
            self.best[key] = c
            return c
        if torch.cuda.is_current_stream_capturing():
            return default            # no timing inside a graph capture; tune on the next eager call
        if not self.enabled or len(candidates) <= 1:
            self.best[key] = default
            return default
        times = []
        for cand in candidates:
            run(cand)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(self.reps):
                run(cand)
            e.record()
            e.synchronize()
            times.append((s.elapsed_time(e), cand))
        c = min(times, key=lambda t: t[0])[1]
        self.best[key] = c
        if _FILE:
            _TABLE[self._tkey(key)] = _encode(c)
            _save()
        return c
