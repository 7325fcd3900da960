#!/usr/bin/env python
"""Dataset snapshot (reference ``IMAGENET/tools/create_imagenet_snapshot.py`` documented an EBS
snapshot). Here: a manifest (relative path, size, class) plus optional tar shards of an
ImageNet-layout tree, so a node can verify or restore its local copy."""
import argparse
import json
import os
import sys
import tarfile


def manifest(root: str):
    out = []
    for dirpath, _, files in sorted(os.walk(root)):
        for f in sorted(files):
            p = os.path.join(dirpath, f)
            out.append({"path": os.path.relpath(p, root), "bytes": os.path.getsize(p)})
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("root")
    p.add_argument("--out", required=True, help="output directory")
    p.add_argument("--shard-mb", type=float, default=0, help="also write tar shards of this size")
    a = p.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    m = manifest(a.root)
    with open(os.path.join(a.out, "manifest.json"), "w") as f:
        json.dump({"root": os.path.abspath(a.root), "files": m}, f)
    if a.shard_mb > 0:
        cap, k, acc, tf = a.shard_mb * 2 ** 20, 0, 0, None
        for e in m:
            if tf is None or acc >= cap:
                if tf is not None:
                    tf.close()
                tf = tarfile.open(os.path.join(a.out, f"shard_{k:05d}.tar"), "w")
                k, acc = k + 1, 0
            tf.add(os.path.join(a.root, e["path"]), arcname=e["path"])
            acc += e["bytes"]
        if tf is not None:
            tf.close()
    print(f"{len(m)} files, {sum(e['bytes'] for e in m) / 2**20:.1f} MiB -> {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
