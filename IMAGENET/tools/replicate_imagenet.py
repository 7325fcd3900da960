#!/usr/bin/env python
"""Dataset staging (reference ``IMAGENET/tools/replicate_imagenet.py`` replicated an EBS volume per
AWS zone). On an MI355X node the equivalent is getting an ImageNet-layout tree onto local NVMe:

  * ``--src DIR``: copy an existing ``<root>/{train,validation}/<class>/<img>`` tree (parallel,
    skip-if-same-size) to ``--dst``;
  * ``--synthetic``: write a synthetic tree of random JPEGs (same layout, configurable size) so the
    real-folder loader (``ImageFolderU8``) can be exercised without the dataset.
"""
import argparse
import os
import shutil
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def copy_tree(src: str, dst: str, workers: int = 16) -> int:
    jobs = []
    for dirpath, _, files in os.walk(src):
        rel = os.path.relpath(dirpath, src)
        os.makedirs(os.path.join(dst, rel), exist_ok=True)
        for f in files:
            s, d = os.path.join(dirpath, f), os.path.join(dst, rel, f)
            if not (os.path.exists(d) and os.path.getsize(d) == os.path.getsize(s)):
                jobs.append((s, d))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(lambda sd: shutil.copyfile(*sd), jobs))
    return len(jobs)


def write_synthetic(dst: str, classes: int, per_class_train: int, per_class_val: int,
                    size: int = 160, seed: int = 0) -> int:
    from PIL import Image
    rng = np.random.default_rng(seed)
    n = 0
    for split, per in (("train", per_class_train), ("validation", per_class_val)):
        for c in range(classes):
            d = os.path.join(dst, split, f"n{c:08d}")
            os.makedirs(d, exist_ok=True)
            for i in range(per):
                w = int(size * rng.uniform(0.75, 1.33))
                arr = rng.integers(0, 256, size=(size, w, 3), dtype=np.uint8)
                Image.fromarray(arr).save(os.path.join(d, f"img_{i:06d}.JPEG"), quality=85)
                n += 1
    return n


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--dst", required=True)
    p.add_argument("--src", default=None)
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--classes", type=int, default=10)
    p.add_argument("--per-class-train", type=int, default=32)
    p.add_argument("--per-class-val", type=int, default=8)
    p.add_argument("--size", type=int, default=160)
    p.add_argument("--workers", type=int, default=16)
    a = p.parse_args(argv)
    if a.synthetic:
        n = write_synthetic(a.dst, a.classes, a.per_class_train, a.per_class_val, a.size)
    elif a.src:
        n = copy_tree(a.src, a.dst, a.workers)
    else:
        p.error("need --src or --synthetic")
    print(f"{n} files written under {a.dst}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
