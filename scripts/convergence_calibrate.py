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
    ap.add_argument("--amp", default="", help="comma list of texture amplitudes (test's: AMP)")
    ap.add_argument("--peak", default="", help="comma list of peak LRs (test's: PEAK)")
    ap.add_argument("--methods", default="", help="comma list (default: every test method)")
    ap.add_argument("--modes", default="layerwise,entiremodel")
    a = ap.parse_args()
    import test_convergence_gpu as T
    want = set(a.methods.split(",")) if a.methods else None
    cases = [(m, kw, mode) for m, kw in T.METHODS for mode in a.modes.split(",")
             if not (m == "none" and mode == "entiremodel") and (want is None or m in want)]
    cases.append(("Topk", {"K": 1e-6}, "layerwise"))             # broken-compressor control
    amps = [float(x) for x in a.amp.split(",")] if a.amp else [T.AMP]
    peaks = [float(x) for x in a.peak.split(",")] if a.peak else [T.PEAK]
    for amp in amps:
        for peak in peaks:
            for seed in [int(s) for s in a.seeds.split(",")]:
                for method, kw, mode in cases:
                    t0 = time.time()
                    acc, first, last = T.run_short(method, kw, mode, seed=seed,
                                                   steps=a.steps or T.STEPS, amp=amp, peak=peak)
                    print(json.dumps(dict(method=method, mode=mode, kw=kw, seed=seed,
                                          acc=round(acc, 4), loss_first=round(first, 4),
                                          loss_last=round(last, 4),
                                          wall_s=round(time.time() - t0, 1),
                                          steps=a.steps or T.STEPS, peak=peak,
                                          task=f"textures amp={amp}")), flush=True)


if __name__ == "__main__":
    main()
