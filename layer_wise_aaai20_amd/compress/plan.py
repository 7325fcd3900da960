"""Static per-bucket launch plans for the compression / optimizer kernels.

A bucket is a contiguous slice of the gradient arena holding S segments (layers). Everything the
kernels need that does not change from step to step — segment offsets and sizes, Top-K keep
counts, payload slot offsets, the workgroup task tables (which 8192-element block of which
segment each workgroup owns) — is computed once here, uploaded once, and reused every step.
This replaces the reference's per-step, per-tensor Python loop over ``model.parameters()``
(``CIFAR10/core.py:176``) with one launch chain per bucket.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

LARGE_EPB = 8192     # must match csrc/lw_kernels.h kLargeEPB
SMALL_MAX = 4096     # kSmallMax
UNPACK_CHUNK = 4096  # kUnpackChunk
GROUP = 32           # quantiser group (elements per thread)


def hdr_words(nseg: int) -> int:
    return (nseg + 3) // 4 * 4


class SegPlan:
    def __init__(self, offsets: Sequence[int], sizes: Sequence[int], gid_base: int = 0):
        self.offsets = np.asarray(offsets, dtype=np.int64)
        self.sizes = np.asarray(sizes, dtype=np.int64)
        assert len(self.offsets) == len(self.sizes)
        self.S = len(self.sizes)
        self.gid_base = int(gid_base)
        self.numel = int(self.offsets[-1] + self.sizes[-1]) if self.S else 0
        self._dev: Dict = {}

    # -------------------------------------------------------------- host tables
    def seg_off_ext(self) -> np.ndarray:
        return np.concatenate([self.offsets, [self.offsets[-1] + self.sizes[-1]]]).astype(np.int64)

    def split(self, small_max: int):
        small = [s for s in range(self.S) if self.sizes[s] <= small_max]
        large = [s for s in range(self.S) if self.sizes[s] > small_max]
        return small, large

    @staticmethod
    def block_tasks(sizes: np.ndarray, segs: List[int], epb: int):
        tasks, lo = [], [0]
        for li, s in enumerate(segs):
            nb = max(1, -(-int(sizes[s]) // epb))
            tasks.extend((li, b * epb) for b in range(nb))
            lo.append(len(tasks))
        t = np.asarray(tasks, dtype=np.int32).reshape(-1, 2)
        return t, np.asarray(lo, dtype=np.int32)

    def unpack_tasks(self) -> np.ndarray:
        t = [(s, c) for s in range(self.S) for c in range(0, max(1, int(self.sizes[s])),
                                                           UNPACK_CHUNK)]
        return np.asarray(t, dtype=np.int32).reshape(-1, 2)

    def groups(self) -> np.ndarray:
        return -(-self.sizes // GROUP)

    def rec_off(self) -> np.ndarray:
        return np.concatenate([[0], np.cumsum(self.groups())]).astype(np.int64)

    # -------------------------------------------------------------- device tables
    def dev(self, device: torch.device, key: str, build) -> torch.Tensor:
        k = (str(device), key)
        t = self._dev.get(k)
        if t is None:
            t = build()
            t = torch.as_tensor(t).to(device) if not isinstance(t, torch.Tensor) else t.to(device)
            self._dev[k] = t
        return t

    def common(self, device):
        d = torch.device(device)
        return dict(
            seg_off=self.dev(d, "seg_off", lambda: torch.from_numpy(self.seg_off_ext())),
            seg_n=self.dev(d, "seg_n", lambda: torch.from_numpy(self.sizes.astype(np.int32))),
        )

    def select_tables(self, device):
        d = torch.device(device)
        small, large = self.split(SMALL_MAX)

        def tasks():
            return torch.from_numpy(self.block_tasks(self.sizes, large, LARGE_EPB)[0])

        def lo():
            return torch.from_numpy(self.block_tasks(self.sizes, large, LARGE_EPB)[1])
        t = dict(self.common(d))
        t.update(
            small_segs=self.dev(d, "small", lambda: torch.tensor(small, dtype=torch.int32)),
            large_segs=self.dev(d, "large", lambda: torch.tensor(large, dtype=torch.int32)),
            tasks=self.dev(d, "tasks", tasks),
            task_lo=self.dev(d, "task_lo", lo),
        )
        return t

    def all_large_tables(self, device):
        d = torch.device(device)
        segs = list(range(self.S))
        t = dict(self.common(d))
        t.update(
            segs=self.dev(d, "all_segs", lambda: torch.tensor(segs, dtype=torch.int32)),
            tasks=self.dev(d, "all_tasks", lambda: torch.from_numpy(
                self.block_tasks(self.sizes, segs, LARGE_EPB)[0])),
            task_lo=self.dev(d, "all_task_lo", lambda: torch.from_numpy(
                self.block_tasks(self.sizes, segs, LARGE_EPB)[1])),
            rec_off=self.dev(d, "rec_off", lambda: torch.from_numpy(self.rec_off())),
        )
        return t

    def max_large_tasks(self) -> int:
        """The most 8192-element tasks of one large (> SMALL_MAX) segment (0: none)."""
        if not hasattr(self, "_max_large_tasks"):
            _, large = self.split(SMALL_MAX)
            self._max_large_tasks = max([-(-int(self.sizes[s]) // LARGE_EPB) for s in large],
                                        default=0)
        return self._max_large_tasks

    def utasks(self, device):
        return self.dev(torch.device(device), "utasks", lambda: torch.from_numpy(self.unpack_tasks()))

    def n_tasks(self, small_max: int) -> int:
        _, large = self.split(small_max)
        return int(sum(max(1, -(-int(self.sizes[s]) // LARGE_EPB)) for s in large))
