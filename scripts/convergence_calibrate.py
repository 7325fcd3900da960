#!/usr/bin/env python
"""Calibration of tests/test_convergence_gpu.py: held-out accuracy of the convergence smoke's
short ResNet-9 run on the calibrated texture task (data/cifar.py synthetic_cifar10
task="textures") for every (method, granularity), over seeds, plus a broken-compressor control
(Top-K at K = 1e-6: one element per tensor) that a useful threshold must reject.

usage: python scripts/convergence_calibrate.py [--seeds 0,1] [--steps 300]
Prints one JSON line per run."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1")
    ap.add_argument("--steps", type=int, default=0, help="0: the test's own step count")
    a = ap.parse_args()
    import test_convergence_gpu as T
    cases = [(m, kw, mode) for m, kw in T.METHODS for mode in ("layerwise", "entiremodel")
             if not (m == "none" and mode == "entiremodel")]
    cases.append(("Topk", {"K": 1e-6}, "layerwise"))             # broken-compressor control
    for seed in [int(s) for s in a.seeds.split(",")]:
        for method, kw, mode in cases:
            t0 = time.time()
            acc, first, last = T.run_short(method, kw, mode, seed=seed,
                                           steps=a.steps or T.STEPS)
            print(json.dumps(dict(method=method, mode=mode, kw=kw, seed=seed,
                                  acc=round(acc, 4), loss_first=round(first, 4),
                                  loss_last=round(last, 4), wall_s=round(time.time() - t0, 1),
                                  task=f"textures amp={T.AMP}")), flush=True)


if __name__ == "__main__":
    main()
