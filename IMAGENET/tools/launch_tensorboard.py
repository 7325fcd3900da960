#!/usr/bin/env python
"""Start TensorBoard on the run directory (reference ``IMAGENET/tools/launch_tensorboard.py``
created an AWS instance for it). Uses the ``tensorboard`` executable when installed; otherwise
prints the scalars the runs logged (``TensorboardLogger`` also writes ``scalars.jsonl``)."""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--logdir", default="runs")
    p.add_argument("--port", type=int, default=6006)
    a = p.parse_args(argv)
    exe = shutil.which("tensorboard")
    if exe:
        return subprocess.call([exe, "--logdir", a.logdir, "--port", str(a.port), "--bind_all"])
    files = sorted(glob.glob(os.path.join(a.logdir, "**", "*.jsonl"), recursive=True))
    if not files:
        print(f"tensorboard is not installed and no *.jsonl scalar logs under {a.logdir}")
        return 1
    for fn in files:
        last = {}
        with open(fn) as f:
            for line in f:
                try:
                    r = json.loads(line)
                except ValueError:
                    continue
                last[r.get("tag", "?")] = r
        print(f"== {fn}")
        for tag, r in sorted(last.items()):
            print(f"  {tag:40s} step {r.get('step')}: {r.get('value')}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
