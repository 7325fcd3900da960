#!/usr/bin/env python
"""Per-method held-out accuracy on the synthetic CIFAR-10 texture task.

This reproduces the kind of comparison the reference paper makes between compressors
(``CIFAR10/dawn.py:98-155``, whose top-1 goes to ``logs.tsv``). For each method and each
granularity, a ResNet-9 is trained with the dawn recipe and its held-out accuracy reported:

* data: 50 k images, batch 512, crop / flip / cutout augmentation;
* schedule: ``PiecewiseLinear([0, 5, E], [0, 0.4, 0])`` per-sample LR; Nesterov momentum 0.9;
  weight decay ``5e-4 · bs``;
* epochs: 24, or 40 for Randomk / Thresholdv (``dawn.py:105-108``).

Everything runs on the MI355X path: MFMA convolutions, CompressedDDP, FlatSGD, and the HIP-graph
step. Data is synthetic (``data/cifar.py synthetic_cifar10``); parity with real CIFAR-10 is
unpinned.

usage:
  python scripts/cifar_accuracy_table.py --amps 0.2,0.3,0.45   # calibration (no compression)
  python scripts/cifar_accuracy_table.py                        # every method, both modes
One JSON line per run.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

RUNS = [
    ("none", "none", {}, False),
    ("Topk", "layerwise", {"K": 0.01}, False), ("Topk", "layerwise", {"K": 0.01}, True),
    ("Topk", "entiremodel", {"K": 0.01}, False), ("Topk", "entiremodel", {"K": 0.01}, True),
    ("Topk", "layerwise", {"K": 0.001}, False), ("Topk", "layerwise", {"K": 0.001}, True),
    ("Randomk", "layerwise", {"K": 0.01}, False), ("Randomk", "layerwise", {"K": 0.01}, True),
    ("Randomk", "entiremodel", {"K": 0.01}, True),
    ("Thresholdv", "layerwise", {"V": 1e-3}, False),
    ("AdaptiveThreshold", "layerwise", {}, False), ("AdaptiveThreshold", "entiremodel", {}, False),
    ("TernGrad", "layerwise", {}, False), ("TernGrad", "entiremodel", {}, False),
    ("RandomDithering", "layerwise", {"qstates": 127}, False),
    ("RandomDithering", "layerwise", {"qstates": 255}, False),
    ("RandomDithering", "entiremodel", {"qstates": 255}, False),
    ("RandomDithering", "layerwise", {"qstates": 32767}, True),
]


def one(method, mode, kw, ef, amp, epochs_override, n_train, net):
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    epochs = epochs_override or (40 if method in ("Randomk", "Thresholdv") else 24)
    torch.manual_seed(0)
    tr = CifarTrainer(net, compress=mode, method=method, error_feedback=ef, epochs=epochs,
                      n_train=n_train, n_test=10000, amp=amp, **kw)
    steps = epochs * tr.steps_per_epoch
    t0 = time.time()
    losses = []
    for i in range(steps):
        losses.append(tr.step())
        if (i + 1) % tr.steps_per_epoch == 0 and (i + 1) // tr.steps_per_epoch % 8 == 0:
            print(f"  [{method} {mode}] epoch {(i + 1) // tr.steps_per_epoch}: "
                  f"train loss {float(losses[-1]) / tr.bs:.4f}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    wall = time.time() - t0
    acc = tr.evaluate()
    last = sum(float(v) for v in losses[-tr.steps_per_epoch:]) / tr.steps_per_epoch / tr.bs
    return {"network": net, "method": method, "mode": mode, **kw, "error_feedback": ef,
            "epochs": epochs, "test_acc": round(100 * acc, 2), "final_train_loss": round(last, 4),
            "amp": amp, "train_s": round(wall, 1), "graph_replays": tr.graphed.replays,
            "wire_bytes_per_step": tr.ddp.sync_stats().payload_bytes}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--amps", default="", help="calibration: uncompressed runs at these amps")
    ap.add_argument("--amp", type=float, default=None)
    ap.add_argument("--epochs", type=int, default=0)
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--network", default="resnet9")
    ap.add_argument("--only", default="", help="comma list of run indices")
    args = ap.parse_args()
    if args.amps:
        for a in args.amps.split(","):
            print(json.dumps(one("none", "none", {}, False, float(a), args.epochs,
                                 args.n_train, args.network)), flush=True)
        return
    idx = [int(i) for i in args.only.split(",")] if args.only else range(len(RUNS))
    for i in idx:
        m, mode, kw, ef = RUNS[i]
        print(json.dumps(one(m, mode, kw, ef, args.amp, args.epochs, args.n_train,
                             args.network)), flush=True)


if __name__ == "__main__":
    main()
