#!/usr/bin/env python
"""Fold scripts/accuracy_r50.py output (one JSON line per (seed, method)) into the reference-point
table bench.py quotes next to its top-1 (layer_wise_aaai20_amd/train/accuracy_reference.json: package
data, so it ships to the GPU box; profiles/ does not).
usage: python scripts/acc_reference.py RUNS.jsonl [OUT.json]"""
import json
import statistics
import sys


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "layer_wise_aaai20_amd/train/accuracy_reference.json"
    by, steps, sched = {}, None, None
    for line in open(src):
        d = json.loads(line)
        steps = d["steps"] if steps is None else steps
        sc = {k: d.get(k) for k in ("peak_lr_512", "warmup", "decay", "momentum")}
        sched = sc if sched is None else sched
        assert sc == sched, "one schedule per table"
        assert d["steps"] == steps, "one step budget per table"
        by.setdefault(d["method"], []).append((d.get("seed", 0), d["top1"]))
    methods = {}
    for m, runs in by.items():
        top = [t for _, t in sorted(runs)]
        methods[m] = {"mean": round(statistics.mean(top), 3),
                      "stdev": round(statistics.stdev(top), 3) if len(top) > 1 else 0.0,
                      "seeds": [s for s, _ in sorted(runs)], "top1": top}
    with open(dst, "w") as f:
        json.dump({"steps": steps, "source": src, "schedule": sched, "methods": methods}, f,
                  indent=1)
    print(json.dumps(methods, indent=1))


if __name__ == "__main__":
    main()
