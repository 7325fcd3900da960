#!/usr/bin/env python
"""Steady-state per-step breakdown from a rocprofv3 kernel_trace.csv: step boundaries are a
kernel launched once per step — the arena SGD (`k_sgd<`), or, when every bucket's step is fused
into its decode (k_unpack_sgd), the input kernel (CIFAR augmentation / ImageNet normalisation);
only the last N steps are summarised, so MIOpen's find-mode search in the warm-up does not
pollute the numbers."""
import csv
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import CATS  # noqa: E402


def main(path, last=5, verbose=False):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if re.search(r"lw::k_sgd<", r["Kernel_Name"])]
    if len(sgd) < last + 1:
        # every bucket's step fused into its decode: the step is the period of the replayed
        # graph's kernel-name sequence (the smallest P whose last `last` periods are identical)
        # (the run may end with a few non-step kernels: trim up to 1000 from the end)
        names = [r["Kernel_Name"] for r in rows]
        for trim in range(0, min(1001, len(names) // 2), 25):
            n = len(names) - trim
            for P in range(16, n // (last + 1) + 1):
                if names[n - 1] != names[n - 1 - P]:
                    continue
                tail = names[n - P:n]
                # (a step, not a repeated block inside one: the period holds the optimizer step)
                if not any("k_unpack_sgd" in x or "lw::k_sgd<" in x for x in tail) or \
                        not any("k_gemm" in x for x in tail):
                    continue
                if all(names[n - (k + 1) * P:n - k * P] == tail for k in range(1, last + 1)):
                    sgd = [n - 1 - k * P for k in range(last, -1, -1)]
                    break
            if sgd:
                break
    if len(sgd) < last + 1:
        raise SystemExit(f"only {len(sgd)} steps in trace")
    lo, hi = sgd[-last - 1] + 1, sgd[-1] + 1
    sel = rows[lo:hi]
    wall = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e6 / last
    tot, names, busy = {}, {}, 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        busy += d
        n = r["Kernel_Name"]
        cat = next((c for c, p in CATS if re.search(p, n)), "other")
        tot[cat] = tot.get(cat, 0.0) + d
        key = n[:100]
        names.setdefault(cat, {}).setdefault(key, [0.0, 0])
        names[cat][key][0] += d
        names[cat][key][1] += 1
    print(f"steps={last}  wall/step={wall:.3f} ms  kernel-busy/step={busy / last:.3f} ms  "
          f"kernels/step={len(sel) / last:.0f}")
    for c, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {c:28s} {t / last:8.3f} ms  {100 * t / busy:5.1f}%")
        if verbose:
            for k, (t2, n2) in sorted(names[c].items(), key=lambda x: -x[1][0])[:int(__import__("os").environ.get("TOPK", "14"))]:
                print(f"      {t2 / last:7.3f}  x{n2 // last:<4d} {k}")
    seq = __import__("os").environ.get("SEQ")
    if seq:                       # the last step's kernels in launch order (what precedes a copy)
        one = rows[sgd[-2] + 1:sgd[-1] + 1]
        with open(seq, "w") as f:
            for r in one:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
                f.write(f"{d:9.1f} us  grid={grid:>8}  {r['Kernel_Name'][:110]}\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5, "-v" in sys.argv)
