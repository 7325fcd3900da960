#!/bin/bash
# rocprofv3 kernel statistics of the CIFAR benches (bench_cifar.py, one run per config): top
# kernels by total time, vendor (non lw::) kernels marked.   usage: scripts/prof_cifar.sh [configs]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cifar_prof
for c in ${@:-anchor vgg16 alexnet}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/cprof/$c -o run --output-format csv \
    -- python bench_cifar.py --config $c --steps 10 --warmup 5 > gpurun_out/cifar_prof/$c.log 2>&1 || exit $?
  ST=$(find /tmp/cprof/$c -name '*kernel_stats.csv' | head -1)
  python - "$ST" > gpurun_out/cifar_prof/${c}_top.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.3f} ms (15 steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    n = r["Name"]
    tag = "   " if "lw::" in n else "[V]"
    print(f"{tag} {float(r['TotalDurationNs']) / 1e6:8.3f} ms {float(r['Percentage']):5.1f}% x{r['Calls']:>5} {n[:110]}")
PY
done
