"""ImageNet data path: synthetic loaders of the reference's shapes, distributed (uneven) validation
sharding and aspect-ratio ("rectangular") validation batches.

Counterparts of ``IMAGENET/training/dataloader.py`` (``get_loaders``, ``BatchTransformDataLoader``,
``fast_collate``, ``DistValSampler``, ``sort_ar``, ``chunks``, ``map_idx2ar``, ``CropArTfm``).
No network and no ImageNet copy are available here, so the dataset is synthetic: per-sample uint8
NHWC images of the phase's size and labels drawn from a fixed seed. Everything downstream (GPU
normalisation, sharding, uneven last batches, rect-val batch shapes) is the real code path.
``ImageFolderU8`` reads a real ``<root>/<class>/<image>`` tree with PIL (decode in DataLoader
workers; uint8 HWC out, normalised on the GPU): ``RandomResizedCropFlip`` for training,
``ResizeCenterCrop`` / ``CropArTfm`` (rect-val) for validation, aspect ratios cached as JSON.
"""
from __future__ import annotations

import json
import math
import os
import random
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops._ext import h16
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
            yield normalize_nhwc_u8(imgs.contiguous(), self.mean, self.std, self.dtype,
                                    pad4=getattr(self, "pad4", False)), target


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
    """``CropArTfm`` (``dataloader.py:164-175``): target (h, w) for an aspect ratio ar = w / h,
    the short side = ``size``, the long side truncated to a multiple of 8. A tall image (ar < 1)
    gets a tall crop (h > w), a wide one a wide crop."""
    if ar < 1:
        return int(size / ar) // 8 * 8, size
    return size, int(size * ar) // 8 * 8


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


# ----------------------------------------------------------------------------- real folders
IMG_EXTS = (".jpg", ".jpeg", ".png", ".bmp", ".webp", ".ppm", ".tif", ".tiff")


def find_classes(root: str) -> Tuple[List[str], dict]:
    classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
    if not classes:
        raise FileNotFoundError(f"no class sub-directories under {root}")
    return classes, {c: i for i, c in enumerate(classes)}


def make_samples(root: str) -> List[Tuple[str, int]]:
    classes, idx = find_classes(root)
    out = []
    for c in classes:
        for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
            for f in sorted(files):
                if f.lower().endswith(IMG_EXTS):
                    out.append((os.path.join(dirpath, f), idx[c]))
    return out


def _rng() -> random.Random:
    """Per-worker RNG seeded from torch's per-worker seed (numpy is not reseeded by DataLoader)."""
    seed = torch.initial_seed()
    r = getattr(_rng, "_r", None)
    if r is None or getattr(_rng, "_seed", None) != seed:
        _rng._r, _rng._seed = random.Random(seed), seed
    return _rng._r


class RandomResizedCropFlip:
    """Inception-style crop: area in ``scale`` of the image, log-uniform aspect ratio in
    ``ratio``, 10 tries then a centre crop; bilinear resize to ``size``; horizontal flip with
    p = 0.5 (``dataloader.py:28-31``)."""

    def __init__(self, size: int, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), flip: bool = True):
        self.size, self.scale, self.ratio, self.flip = size, scale, ratio, flip

    def box(self, w: int, h: int, r: random.Random):
        area = w * h
        lr = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            target = area * r.uniform(*self.scale)
            ar = math.exp(r.uniform(*lr))
            cw, ch = int(round(math.sqrt(target * ar))), int(round(math.sqrt(target / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                x0, y0 = r.randint(0, w - cw), r.randint(0, h - ch)
                return x0, y0, cw, ch
        in_ar = w / h
        if in_ar < self.ratio[0]:
            cw, ch = w, int(round(w / self.ratio[0]))
        elif in_ar > self.ratio[1]:
            ch, cw = h, int(round(h * self.ratio[1]))
        else:
            cw, ch = w, h
        return (w - cw) // 2, (h - ch) // 2, cw, ch

    def __call__(self, img, index: int = 0):
        from PIL import Image
        r = _rng()
        x0, y0, cw, ch = self.box(img.width, img.height, r)
        img = img.resize((self.size, self.size), Image.BILINEAR, box=(x0, y0, x0 + cw, y0 + ch))
        if self.flip and r.random() < 0.5:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        return img


class ResizeCenterCrop:
    """Validation: shorter side → ``int(size * 1.14)``, centre crop ``size`` (``dataloader.py:
    60-74``)."""

    def __init__(self, size: int, resize: Optional[int] = None):
        self.size, self.resize = size, resize or int(size * 1.14)

    def __call__(self, img, index: int = 0):
        from PIL import Image
        w, h = img.size
        s = self.resize / min(w, h)
        nw, nh = max(self.size, int(round(w * s))), max(self.size, int(round(h * s)))
        img = img.resize((nw, nh), Image.BILINEAR)
        x0, y0 = (nw - self.size) // 2, (nh - self.size) // 2
        return img.crop((x0, y0, x0 + self.size, y0 + self.size))


class CropArTfm:
    """Rect-val: resize the shorter side to ``size`` and centre-crop to the batch's mean aspect
    ratio (``crop_size_for_ar``), so a batch shares one (h, w) (``dataloader.py:164-201``)."""

    def __init__(self, idx2ar: dict, size: int):
        self.idx2ar, self.size = idx2ar, size

    def __call__(self, img, index: int = 0):
        from PIL import Image
        th, tw = crop_size_for_ar(self.idx2ar[index], self.size)
        w, h = img.size
        s = max(tw / w, th / h)
        nw, nh = max(tw, int(round(w * s))), max(th, int(round(h * s)))
        img = img.resize((nw, nh), Image.BILINEAR)
        x0, y0 = (nw - tw) // 2, (nh - th) // 2
        return img.crop((x0, y0, x0 + tw, y0 + th))


class ImageFolderU8(Dataset):
    """``<root>/<class>/<image>`` → (uint8 [H, W, 3], class index); decoding and augmentation run
    in the DataLoader workers, normalisation on the GPU (``BatchTransformDataLoader``)."""

    def __init__(self, root: str, transform: Optional[Callable] = None,
                 samples: Optional[List[Tuple[str, int]]] = None):
        self.root = root
        self.samples = samples if samples is not None else make_samples(root)
        self.transform = transform

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image
        path, label = self.samples[i]
        with Image.open(path) as im:
            img = im.convert("RGB")
        if self.transform is not None:
            img = self.transform(img, i)
        return np.asarray(img, dtype=np.uint8), label


def sort_ar_folder(valdir: str, cache: Optional[str] = None) -> List[tuple]:
    """[(w/h, index)] of a real validation folder, sorted; image headers only (no decode). Cached
    as JSON next to the data (the reference pickles ``sorted_idxar.p``; nothing is unpickled
    here)."""
    cache = cache or os.path.join(os.path.dirname(os.path.normpath(valdir)), "sorted_idxar.json")
    samples = make_samples(valdir)
    if os.path.exists(cache):
        with open(cache) as f:
            data = json.load(f)
        if len(data) == len(samples):
            return [(float(a), int(i)) for a, i in data]
    from PIL import Image
    ars = []
    for i, (path, _) in enumerate(samples):
        with Image.open(path) as im:
            w, h = im.size
        ars.append((w / h, i))
    out = sorted(ars)
    try:
        with open(cache, "w") as f:
            json.dump(out, f)
    except OSError:
        pass
    return out


def _folder_loaders(traindir, valdir, sz, bs, val_bs, workers, rect_val, min_scale,
                    distributed, device, dtype):
    from ..parallel import comm
    train_ds = ImageFolderU8(traindir, RandomResizedCropFlip(sz, scale=(min_scale, 1.0)))
    trn_smp = torch.utils.data.distributed.DistributedSampler(
        train_ds, num_replicas=comm.world_size(), rank=comm.rank()) if distributed else None
    trn = DataLoader(train_ds, batch_size=bs, shuffle=trn_smp is None, num_workers=workers,
                     collate_fn=fast_collate, sampler=trn_smp, pin_memory=True,
                     persistent_workers=workers > 0)
    if rect_val:
        idx_ar = sort_ar_folder(valdir)
        val_ds = ImageFolderU8(valdir, CropArTfm(map_idx2ar(idx_ar, val_bs), sz))
        order = [i for _, i in idx_ar]
    else:
        val_ds = ImageFolderU8(valdir, ResizeCenterCrop(sz))
        order = list(range(len(val_ds)))
    val_smp = DistValSampler(order, val_bs, distributed)
    val = DataLoader(val_ds, batch_sampler=val_smp, num_workers=workers, collate_fn=fast_collate,
                     pin_memory=True)
    return (BatchTransformDataLoader(trn, device, dtype),
            BatchTransformDataLoader(val, device, dtype), trn_smp, val_smp)


class GPUSyntheticLoader:
    """Synthetic training batches generated on the GPU (uint8 noise plus a per-class colour
    offset, so the model has a signal to learn) and normalised by the same fused kernel as real
    batches: the training loop of the CLI runs at the model's speed instead of the speed of a
    host-side numpy generator. Each rank draws its own shard of an epoch (``n // world`` items),
    deterministically from (seed, epoch, batch, rank)."""

    def __init__(self, n, size, bs, device, dtype=torch.float32, seed=0, distributed=False,
                 pad4=False, num_classes=1000):
        from ..parallel import comm
        self.n, self.size, self.bs, self.dtype, self.seed = n, size, bs, dtype, seed
        self.device = torch.device(device)
        self.world = comm.world_size() if distributed else 1
        self.rank = comm.rank() if distributed else 0
        self.pad4, self.num_classes, self.epoch = pad4, num_classes, 0
        self.mean = torch.tensor(IMAGENET_MEAN, dtype=torch.float32)
        self.std = torch.tensor(IMAGENET_STD, dtype=torch.float32)
        g = torch.Generator(device=self.device).manual_seed(seed + 17)
        self.bias = torch.randint(0, 128, (num_classes, 3), dtype=torch.int16, device=self.device,
                                  generator=g)
        self.sampler = self

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def update_batch_size(self, bs):
        self.bs = bs

    def __len__(self):
        return max(1, -(-(self.n // self.world) // self.bs))

    def __iter__(self):
        from ..ops.nn import normalize_nhwc_u8
        per = self.n // self.world
        for b in range(len(self)):
            nb = min(self.bs, per - b * self.bs)
            g = torch.Generator(device=self.device).manual_seed(
                (self.seed * 1_000_003 + self.epoch * 10_007 + b) * 8191 + self.rank)
            t = torch.randint(0, self.num_classes, (nb,), device=self.device, generator=g)
            x = torch.randint(0, 128, (nb, self.size, self.size, 3), dtype=torch.int16,
                              device=self.device, generator=g)
            x = (x + self.bias[t].view(nb, 1, 1, 3)).to(torch.uint8)
            yield normalize_nhwc_u8(x, self.mean, self.std, self.dtype,
                                    pad4=self.pad4 and self.dtype == h16()), t


def get_loaders(traindir=None, valdir=None, sz=128, bs=256, val_bs=None, workers=0,
                rect_val=False, min_scale=0.08, distributed=False, n_train=None, n_val=None,
                device=None, dtype=torch.float32, seed=0, synthetic=True, gpu_synthetic=False,
                pad4=False):
    """Train / val loaders + samplers for one phase (``dataloader.py:26-57``).

    Synthetic sizes default to a small ImageNet stand-in (``n_train = 64 * bs``, ``n_val = 8 *
    val_bs``) so an epoch is short; pass ``n_train`` / ``n_val`` for full-size epochs."""
    from ..parallel import comm
    val_bs = val_bs or bs
    n_train = n_train or 64 * bs
    n_val = n_val or 8 * val_bs
    if not synthetic:
        return _folder_loaders(traindir, valdir, sz, bs, val_bs, workers, rect_val, min_scale,
                               distributed, device, dtype)
    if gpu_synthetic:
        trn = GPUSyntheticLoader(n_train, sz, bs, device, dtype, seed, distributed, pad4)
        trn_smp = trn
    else:
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
    trn_dl = trn if gpu_synthetic else BatchTransformDataLoader(trn, device, dtype)
    val_dl = BatchTransformDataLoader(val, device, dtype)
    val_dl.pad4 = pad4
    return trn_dl, val_dl, trn_smp, val_smp
