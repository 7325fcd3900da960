#!/usr/bin/env python
"""Sum a rocprofv3 counter_collection.csv per kernel name (last 2 steps' worth of dispatches are
what a short bench run mostly contains; warm-up dispatches are included) and print one row per
kernel, largest SQ_WAVE_CYCLES / FETCH_SIZE first."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
rows = list(csv.DictReader(open(sys.argv[1])))
if "--last-step" in sys.argv:
    # only the dispatches of the last step: after the second-to-last fused-SGD dispatch (the tile
    # tuners' timing runs of the first eager step are excluded)
    did = lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", "0")) or 0)  # noqa: E731
    # one step = from one input-normalise dispatch (the step's first kernel) to the next
    st = sorted({did(r) for r in rows if "k_normalize_u8" in r["Kernel_Name"]})
    if len(st) >= 2:
        lo, hi = st[-2], st[-1]
        rows = [r for r in rows if lo <= did(r) < hi]
for r in rows:
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
names = sorted({n for d in agg.values() for n in d})
key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in names else names[0]
print("kernel".ljust(92), "disp", " ".join(n[:16].rjust(16) for n in names))
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get(key, 0))[:60]:
    print(k.ljust(92), str(len(disp[k])).rjust(4), " ".join(f"{d.get(n, 0):16.0f}" for n in names))
# --dispatches PATTERN: one line per matching dispatch of the selected step, in order (which layer
# a BatchNorm call belongs to follows from its grid size and position)
if "--dispatches" in sys.argv:
    pat = sys.argv[sys.argv.index("--dispatches") + 1]
    per = collections.OrderedDict()
    for r in rows:
        if pat not in r["Kernel_Name"]:
            continue
        d = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
        e = per.setdefault(d, {"name": r["Kernel_Name"][:60], "grid": r.get("Grid_Size", "")})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(f"\n# dispatches matching {pat!r}")
    for d, e in per.items():
        print(d.rjust(8), e["name"].ljust(62), str(e["grid"]).rjust(10),
              " ".join(f"{n}={e[n]:.0f}" for n in names if n in e))
