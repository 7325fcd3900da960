"""Shared kernel-choice tuner with an optional persisted table.

The GEMM (``ops/block.py``), Linear (``ops/gemm.py``) and convolution (``ops/conv.py``) tuners
time every candidate kernel (tile, or (tile, split-K)) the first time a problem shape is seen and
keep the fastest, as MIOpen's find mode does for the reference's cuDNN/MIOpen convolutions
(``IMAGENET/training/train_imagenet_nv.py:36`` sets ``cudnn.benchmark``). Timing noise can make
two processes pick different kernels for the same shape, and different kernels round differently.
Three mechanisms make the choices reproducible and identical on every rank:

* **Shipped gfx950 table** (``ops/tune_gfx950.json``): the choices for the benchmark / recipe
  shapes, measured on MI355X. It is read at import unless ``LWAAAI_TUNE_FILE`` names another
  table (``LWAAAI_TUNE_FILE=none`` disables both), so two runs of ``bench.py`` pick the same
  kernels and train bit-identically.
* ``LWAAAI_TUNE_FILE=path``: that table is read at import and a new decision is added to it and,
  on rank 0 (``RANK`` unset or 0), written back atomically.
* **Cross-rank agreement**: inside :func:`rank_agreement` (the trainers wrap their eager
  training steps in it, where every rank runs the same shapes in the same order) the candidate
  times are summed over ranks with one all-reduce before the minimum is taken, so every rank
  picks the same kernel and the step is not paced by one rank's unlucky choice.

A pinned entry is used only if it is one of the current candidates (a table written with other
kernel switches, or before a kernel was removed, is stale for that key): otherwise the shape is
timed as usual and a warning names the stale entry.
"""
from __future__ import annotations

import contextlib
import json
import os
import warnings
from typing import Callable, Dict, Sequence

import torch

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tune_gfx950.json")
_FILE = os.environ.get("LWAAAI_TUNE_FILE", "")
if _FILE.lower() == "none":
    _FILE, _READ = "", ""
else:
    _READ = _FILE or SHIPPED
_TABLE: Dict[str, object] = {}
if _READ and os.path.exists(_READ):
    with open(_READ) as f:
        _TABLE = json.load(f)
# The shipped table pins choices timed on gfx950 (MI355X): on any other device they were never
# timed, so it is used only where the device is gfx950 (checked on the first pick); a table named
# by LWAAAI_TUNE_FILE is the user's own and always used.
_ARCH_OK = None if (_READ == SHIPPED and _TABLE) else True


def _pinned(key: str):
    global _ARCH_OK
    if _ARCH_OK is None:
        arch = ""
        try:
            if torch.cuda.is_available():
                arch = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
        except Exception:                  # noqa: BLE001 — no device / no property: not gfx950
            arch = ""
        _ARCH_OK = arch.startswith("gfx950")
        if not _ARCH_OK and _TABLE:
            warnings.warn(f"shipped tuning table (gfx950) ignored on device arch {arch!r}: "
                          f"every kernel choice is timed instead", stacklevel=3)
    return _TABLE.get(key) if _ARCH_OK else None

_AGREE: list = []          # stack of (process group, device) set by rank_agreement()

# The GEMM tiles 1..6 also exist on v_mfma_f32_32x32x16 (csrc GemmTile id + 40: gemm_core.h k_gemm
# MF = 32); every tuner times them as further candidates (profiles/r5/mf32_ab.txt: they win
# on some shapes and lose overall, so the tuner decides per shape).
MF32 = 40
MF32_ON = True


def with_mf32(tiles) -> tuple:
    """``tiles`` plus the 32x32x16-MFMA twins of those among ids 1..6, when enabled."""
    tiles = tuple(tiles)
    return tiles + (tuple(MF32 + t for t in tiles if 1 <= t <= 6) if MF32_ON else ())


@contextlib.contextmanager
def rank_agreement(group=None, device=None):
    """Within this context every new tuning decision is taken on the candidate times summed over
    the ranks of ``group`` (one all-reduce per decision), so all ranks pick the same kernel. Use
    it only where every rank reaches the same tuner calls in the same order (a training step)."""
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    if on:
        _AGREE.append((group, device))
    try:
        yield
    finally:
        if on:
            _AGREE.pop()


def _agree_times(times):
    if not _AGREE:
        return times
    import torch.distributed as dist
    group, device = _AGREE[-1]
    dev = torch.device("cpu")
    if dist.get_backend(group) == "nccl":
        dev = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([x for x, _ in times], dtype=torch.float64, device=dev)
    dist.all_reduce(t, group=group)
    return [(float(v), c) for v, (_, c) in zip(t.tolist(), times)]


def _encode(v):
    return list(v) if isinstance(v, tuple) else v


def _decode(v):
    return tuple(v) if isinstance(v, list) else v


def _save() -> None:
    if not _FILE or os.environ.get("RANK", "0") != "0":   # (the shipped table is read-only)
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
        pinned = _pinned(self._tkey(key))
        if pinned is not None:
            c = _decode(pinned)
            if any(c == _decode(_encode(x)) for x in candidates) or \
                    (len(candidates) <= 1 and c == default):
                self.best[key] = c
                return c
            warnings.warn(f"stale tuning entry {self._tkey(key)} = {pinned!r}: not among the "
                          f"current candidates {list(candidates)!r}; timing instead",
                          stacklevel=2)
        if torch.cuda.is_current_stream_capturing():
            return default            # no timing inside a graph capture; tune on the next eager call
        if not self.enabled or len(candidates) <= 1:
            self.best[key] = default
            return default
        from ._ext import splitk_paused
        times = []
        with splitk_paused():          # (every candidate timed with its split-K reduce)
            for cand in candidates:
                run(cand)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(self.reps):
                    run(cand)
                e.record()
                e.synchronize()
                times.append((s.elapsed_time(e), cand))
        times = _agree_times(times)
        c = min(times, key=lambda t: t[0])[1]
        self.best[key] = c
        if _FILE:
            _TABLE[self._tkey(key)] = _encode(c)
            _save()
        return c
