#!/usr/bin/env python
"""Which layer-wise Top-K / Random-K settings learn the convergence smoke's texture task, and in
how many steps (tests/test_convergence_gpu.py run_short). One JSON line per run."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tests"))


def main():
    import test_convergence_gpu as T
    cases = [("Topk", {"K": 0.01}, "layerwise"),
             ("Randomk", {"K": 0.1}, "layerwise"),
             ("Randomk", {"K": 0.1}, "entiremodel"),
             ("Randomk", {"K": 0.25, "dense_below": 4096}, "layerwise"),
             ("Randomk", {"K": 0.25, "dense_below": 4096}, "entiremodel"),
             ("Topk", {"K": 0.01, "dense_below": 4096}, "layerwise")]
    for steps in (600, 2000):
        for method, kw, mode in cases:
            for ef in (True, False):
                if method == "none" and not ef:
                    continue
                t0 = time.time()
                acc, first, last = T.run_short(method, kw, mode, seed=0, steps=steps, ef=ef)
                print(json.dumps(dict(method=method, mode=mode, kw=kw, ef=ef, steps=steps,
                                      acc=round(acc, 4), loss_first=round(first, 4),
                                      loss_last=round(last, 4),
                                      wall_s=round(time.time() - t0, 1))), flush=True)


if __name__ == "__main__":
    main()
