#!/usr/bin/env python
"""Held-out top-1 of a short ResNet-50 run on the bench's learnable synthetic task.

This is the accuracy half of the headline metric
("images/sec/node + top-1 acc, ResNet-50 Top-K k=0.1% layer-wise").

Each method trains the same random-init ResNet-50 through the full MI355X path: fused MFMA
convolutions, CompressedDDP compression inline in the HIP-graph step, and FlatSGD. The run is:

* data: bench.py's class-conditional synthetic ImageNet (uint8 noise plus a per-class colour
  offset, 1000 classes), 128 px;
* schedule: a linear LR warm-up (the reference's first phase, ``train_imagenet_nv.py:204-218``)
  to a peak of 1.0 at batch 512, then a linear decay to 0 — calibrated so that the uncompressed
  run is the ceiling (``train/accuracy.py`` PEAK_LR_512 / DECAY,
  ``profiles/r5/acc_schedule_sweep.jsonl``), the same for every method;
* evaluation: held-out top-1 / top-5 on fresh batches of the same distribution.

The methods are compared at the same step budget:

* no compression;
* Top-K 0.1 % layer-wise (the headline config);
* Top-K 0.1 % + error feedback.

Real-ImageNet parity is unpinned (no dataset on this machine).

usage: python scripts/accuracy_r50.py [--steps 300] [--size 128] [--batch 256]
Prints one JSON line per method.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

METHODS = {"none": dict(compress="none", method="none"),
           "topk0.1%": dict(compress="layerwise", method="Topk", K=0.001),
           "topk0.1%+ef": dict(compress="layerwise", method="Topk", K=0.001, error_feedback=True),
           # opt-in EF variants (profiles/r4/ef_root_cause.md)
           "topk0.1%+ef+dense4k": dict(compress="layerwise", method="Topk", K=0.001,
                                       error_feedback=True, dense_below=4096),
           "topk0.1%+ef+mc+dense4k": dict(compress="layerwise", method="Topk", K=0.001,
                                          error_feedback=True, dense_below=4096,
                                          momentum_correction=True),
           "topk0.1%+ef+mc": dict(compress="layerwise", method="Topk", K=0.001,
                                  error_feedback=True, momentum_correction=True),
           "topk0.1%+dense4k": dict(compress="layerwise", method="Topk", K=0.001,
                                    dense_below=4096),
           "randk1%+ef": dict(compress="layerwise", method="Randomk", K=0.01,
                              error_feedback=True),
           "randk1%+ef+mc+dense4k": dict(compress="layerwise", method="Randomk", K=0.01,
                                         error_feedback=True, dense_below=4096,
                                         momentum_correction=True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256)
    from layer_wise_aaai20_amd.train.accuracy import DECAY, PEAK_LR_512
    ap.add_argument("--lr", type=float, default=PEAK_LR_512, help="peak LR at batch 512")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--decay", default=DECAY, choices=["none", "linear"],
                    help="after the warm-up: constant LR, or a linear decay to 0")
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--eval-batches", type=int, default=8)
    ap.add_argument("--methods", default="none,topk0.1%,topk0.1%+ef")
    ap.add_argument("--seeds", default="0", help="comma list: model-init seeds")
    args = ap.parse_args()
    from layer_wise_aaai20_amd.train.accuracy import short_run_top1
    runs = [(seed, name) for seed in [int(v) for v in args.seeds.split(",")]
            for name in args.methods.split(",")]
    for seed, name in runs:
        t0 = time.time()
        r = short_run_top1("cuda:0", steps=args.steps, size=args.size, batch=args.batch,
                           peak_lr_512=args.lr, warmup=args.warmup, decay=args.decay,
                           momentum=args.momentum,
                           eval_batches=args.eval_batches, seed=seed, **METHODS[name])
        print(json.dumps(dict(method=name, seed=seed, chance_top1=0.1,
                              wall_s=round(time.time() - t0, 1),
                              data="synthetic class-conditional (bench.py distribution), "
                                   "random init", **r)), flush=True)

if __name__ == "__main__":
    main()
