#!/usr/bin/env python
"""Sum rocprofv3 counter-collection CSVs per kernel (name prefix) and print per-dispatch means
plus derived ratios. usage: python scripts/pmc_summ.py a.csv [b.csv ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:90]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, d in agg.items():
    n = max(1, len(disp[k]))
    print(f"{k}  (dispatches {n})")
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v / n:16.0f}")
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in d:
                print(f"   {c + ' / wave cycles':44s} {d[c] / wc:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "SQ_BUSY_CYCLES" in d:
        print(f"   {'MFMA busy / busy cycles':44s} {d['SQ_VALU_MFMA_BUSY_CYCLES'] / d['SQ_BUSY_CYCLES']:.3f}")
