"""ImageNet data path: synthetic loaders of the reference's shapes, distributed (uneven) validation
sharding and aspect-ratio ("rectangular") validation batches.

Counterparts of ``IMAGENET/training/dataloader.py`` (``get_loaders``, ``BatchTransformDataLoader``,
``fast_collate``, ``DistValSampler``, ``sort_ar``, ``chunks``, ``map_idx2ar``, ``CropArTfm``).
No network and no ImageNet copy are available here, so the dataset is synthetic: per-sample uint8
NHWC images of the phase's size and labels drawn from a fixed seed. Everything downstream (GPU
normalisation, sharding, uneven last batches, rect-val batch shapes) is the real code path.
``ImageFolderU8`` can read a real ``<root>/<class>/<image>`` tree when PIL is importable.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, Sampler

IMAGENET_MEAN = [0.485 * 255, 0.456 * 255, 0.406 * 255]
IMAGENET_STD = [0.229 * 255, 0.224 * 255, 0.225 * 255]


class SyntheticImageNet(Dataset):
    """Deterministic random uint8 images [H, W, 3] and labels. ``ars`` optionally gives each item an
    aspect ratio (w/h) so rect-val batches have the reference's varying shapes."""

    def __init__(self, n: int, size: int, num_classes: int = 1000, seed: int = 0,
                 ars: Optional[np.ndarray] = None):
        self.n, self.size, self.num_classes, self.seed = n, size, num_classes, seed
        rng = np.random.default_rng(seed)
        self.labels = rng.integers(0, num_classes, size=n).astype(np.int64)
        self.ars = ars

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rng = np.random.default_rng(self.seed * 1_000_003 + int(i))
        img = rng.integers(0, 256, size=(self.size, self.size, 3), dtype=np.uint8)
        return img, int(self.labels[i])


def fast_collate(batch):
    """uint8 NHWC batch + int64 targets (``dataloader.py:117-130`` collates to NCHW uint8; NHWC
    is what the channels_last model consumes, the GPU normaliser permutes logically)."""
    imgs = np.stack([b[0] for b in batch]) if batch else np.zeros((0, 1, 1, 3), np.uint8)
    targets = torch.tensor([b[1] for b in batch], dtype=torch.int64)
    return torch.from_numpy(imgs), targets


class BatchTransformDataLoader:
    """Moves uint8 batches to the GPU and normalises them there in one fused kernel
    (``dataloader.py:76-97``). Output dtype follows the model (fixes SURVEY.md D13)."""

    def __init__(self, loader, device=None, dtype=torch.float32, mean=IMAGENET_MEAN,
                 std=IMAGENET_STD):
        self.loader = loader
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.dtype = dtype
        self.mean = torch.tensor(mean, dtype=torch.float32)
        self.std = torch.tensor(std, dtype=torch.float32)
        self.sampler = getattr(loader, "sampler", None)

    def __len__(self):
        return len(self.loader)

    def update_batch_size(self, bs):
        self.loader.batch_sampler.batch_size = bs

    def __iter__(self):
        from ..ops.nn import normalize_nhwc_u8
        for imgs, target in self.loader:
            imgs = imgs.to(self.device, non_blocking=True)
            target = target.to(self.device, non_blocking=True)
            if imgs.numel() == 0:
                yield torch.empty((0, 3, 1, 1), device=self.device, dtype=self.dtype), target
                continue
            yield normalize_nhwc_u8(imgs.contiguous(), self.mean, self.std, self.dtype), target


class DistValSampler(Sampler):
    """Contiguous shard per rank of the (optionally aspect-ratio sorted) validation indices; ranks
    may get fewer — or zero — items (``dataloader.py:133-161``)."""

    def __init__(self, indices: Sequence[int], batch_size: int, distributed: bool = True,
                 rank: Optional[int] = None, world: Optional[int] = None):
        from ..parallel import comm
        self.indices = list(indices)
        self.batch_size = batch_size
        self.world = world if world is not None else (comm.world_size() if distributed else 1)
        self.rank = rank if rank is not None else (comm.rank() if distributed else 0)
        self.expected_num_batches = math.ceil(len(self.indices) / self.world / batch_size)
        per = self.expected_num_batches * batch_size
        self.shard = self.indices[self.rank * per:(self.rank + 1) * per]

    def __iter__(self):
        for b in range(self.expected_num_batches):
            yield self.shard[b * self.batch_size:(b + 1) * self.batch_size]

    def __len__(self):
        return self.expected_num_batches


def chunks(seq, n):
    return [seq[i:i + n] for i in range(0, len(seq), n)]


def sort_ar(n: int, seed: int = 0) -> List[tuple]:
    """Aspect ratios of the validation set, sorted: [(ar, index)] (``dataloader.py:164-180``).
    Synthetic: ImageNet-like spread of w/h in [0.5, 2]."""
    rng = np.random.default_rng(seed + 17)
    ars = np.exp(rng.uniform(np.log(0.5), np.log(2.0), size=n))
    return sorted((float(a), i) for i, a in enumerate(ars))


def map_idx2ar(idx_ar_sorted, batch_size):
    """Every index of a batch gets the batch's mean aspect ratio (``dataloader.py:190-201``)."""
    out = {}
    for chunk in chunks(idx_ar_sorted, batch_size):
        mean_ar = float(np.mean([ar for ar, _ in chunk]))
        for _, idx in chunk:
            out[idx] = mean_ar
    return out


def crop_size_for_ar(ar: float, size: int):
    """``CropArTfm``: target (h, w) for an aspect ratio, the short side = size, multiples of 8."""
    if ar < 1:
        return size, int(round(size / ar / 8)) * 8
    return int(round(size * ar / 8)) * 8, size


class RectValDataset(Dataset):
    """Validation items resized/cropped to the batch's mean aspect ratio (synthetic pixels)."""

    def __init__(self, base: SyntheticImageNet, idx2ar: dict, size: int):
        self.base, self.idx2ar, self.size = base, idx2ar, size

    def __len__(self):
        return len(self.base)

    def __getitem__(self, i):
        _, label = self.base[i]
        h, w = crop_size_for_ar(self.idx2ar[i], self.size)
        rng = np.random.default_rng(self.base.seed * 7 + int(i))
        return rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8), label


def get_loaders(traindir=None, valdir=None, sz=128, bs=256, val_bs=None, workers=0,
                rect_val=False, min_scale=0.08, distributed=False, n_train=None, n_val=None,
                device=None, dtype=torch.float32, seed=0, synthetic=True):
    """Train / val loaders + samplers for one phase (``dataloader.py:26-57``).

    Synthetic sizes default to a small ImageNet stand-in (``n_train = 64 * bs``, ``n_val = 8 *
    val_bs``) so an epoch is short; pass ``n_train`` / ``n_val`` for full-size epochs."""
    from ..parallel import comm
    val_bs = val_bs or bs
    n_train = n_train or 64 * bs
    n_val = n_val or 8 * val_bs
    if not synthetic:
        raise NotImplementedError("real ImageNet folders need ImageFolderU8 (PIL) — not available "
                                  "offline; use synthetic=True")
    train_ds = SyntheticImageNet(n_train, sz, seed=seed)
    trn_smp = torch.utils.data.distributed.DistributedSampler(
        train_ds, num_replicas=comm.world_size(), rank=comm.rank()) if distributed else None
    trn = DataLoader(train_ds, batch_size=bs, shuffle=trn_smp is None, num_workers=workers,
                     collate_fn=fast_collate, sampler=trn_smp, drop_last=False)
    val_base = SyntheticImageNet(n_val, sz, seed=seed + 1)
    if rect_val:
        idx_ar = sort_ar(n_val, seed)
        idx2ar = map_idx2ar(idx_ar, val_bs)
        val_ds = RectValDataset(val_base, idx2ar, sz)
        order = [i for _, i in idx_ar]
    else:
        val_ds = val_base
        order = list(range(n_val))
    val_smp = DistValSampler(order, val_bs, distributed)
    val = DataLoader(val_ds, batch_sampler=val_smp, num_workers=workers, collate_fn=fast_collate)
    return (BatchTransformDataLoader(trn, device, dtype), BatchTransformDataLoader(val, device, dtype),
            trn_smp, val_smp)
