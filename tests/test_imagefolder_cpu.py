"""Real-folder ImageNet path (PIL decode, crops, rect-val aspect ratios, distributed val shards)
on a tiny generated JPEG tree."""
import numpy as np
import pytest
import torch

from layer_wise_aaai20_amd.data import imagenet as D

PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = tmp_path_factory.mktemp("imnet")
    rng = np.random.default_rng(0)
    for split, n in (("train", 6), ("validation", 5)):
        for c in ("n01", "n02", "n03"):
            d = root / split / c
            d.mkdir(parents=True)
            for i in range(n):
                w, h = int(rng.integers(40, 90)), int(rng.integers(40, 90))
                arr = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
                PIL.fromarray(arr).save(d / f"img{i}.JPEG", quality=90)
    return root


def test_folder_dataset_and_transforms(tree):
    ds = D.ImageFolderU8(str(tree / "train"), D.RandomResizedCropFlip(32, scale=(0.35, 1)))
    assert len(ds) == 18 and sorted({lbl for _, lbl in ds.samples}) == [0, 1, 2]
    img, lbl = ds[3]
    assert img.shape == (32, 32, 3) and img.dtype == np.uint8
    val = D.ImageFolderU8(str(tree / "validation"), D.ResizeCenterCrop(24))
    assert val[0][0].shape == (24, 24, 3)


def test_rect_val_batches_share_shape(tree):
    idx_ar = D.sort_ar_folder(str(tree / "validation"))
    assert [a for a, _ in idx_ar] == sorted(a for a, _ in idx_ar) and len(idx_ar) == 15
    assert (tree / "sorted_idxar.json").exists()
    idx2ar = D.map_idx2ar(idx_ar, 4)
    ds = D.ImageFolderU8(str(tree / "validation"), D.CropArTfm(idx2ar, 32))
    for chunk in D.chunks(idx_ar, 4):
        shapes = {ds[i][0].shape for _, i in chunk}
        assert len(shapes) == 1
        h, w, _ = shapes.pop()
        assert min(h, w) == 32
        ar = np.mean([a for a, _ in chunk])        # ar = w / h
        assert (h > w) == (ar < 1) or h == w, (ar, h, w)


def test_crop_size_for_ar_orientation():
    """Tall images (ar = w/h < 1) get tall crops, like dataloader.py:164-175."""
    assert D.crop_size_for_ar(0.5, 128) == (256, 128)
    assert D.crop_size_for_ar(0.75, 224) == (296, 224)
    assert D.crop_size_for_ar(4 / 3, 224) == (224, 296)
    assert D.crop_size_for_ar(1.0, 224) == (224, 224)


def test_cifar10_missing_dataset_raises(tmp_path):
    from layer_wise_aaai20_amd.data import cifar as C
    with pytest.raises(FileNotFoundError):
        C.cifar10(str(tmp_path))
    with pytest.warns(UserWarning):
        d = C.cifar10(str(tmp_path), synthetic_fallback=True, n_train=16, n_test=8)
    assert d["train"]["data"].shape == (16, 32, 32, 3)


def test_get_loaders_real_folders(tree):
    trn, val, trn_smp, val_smp = D.get_loaders(str(tree / "train"), str(tree / "validation"),
                                               sz=32, bs=4, val_bs=4, workers=0, rect_val=True,
                                               min_scale=0.35, distributed=False, device="cpu",
                                               synthetic=False)
    x, y = next(iter(trn))
    assert x.shape == (4, 3, 32, 32) and x.dtype == torch.float32 and y.shape == (4,)
    seen = 0
    for xb, yb in val:
        assert xb.shape[0] == yb.shape[0]
        seen += yb.shape[0]
    assert seen == 15
