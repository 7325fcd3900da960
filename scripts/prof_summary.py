#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats.csv into per-category time (optionally per step)."""
import csv
import re
import sys

CATS = [
    ("lwaaai compress/unpack", r"lw::k_(small_select|hist|select|count|scan|write|fill_tail|unpack|thresh|set_caps|partial|finalize|quant|dequant)"),
    ("lwaaai sgd", r"lw::k_sgd"),
    ("lwaaai gemm", r"lw::k_(gemm|splitk)"),
    ("lwaaai nn", r"lw::k_(normalize|bn|relu|add|pool|ce)"),
    ("conv fwd", r"igemm_fwd|conv_fwd|ConvFwd|grouped_conv_fwd|naive_conv_fwd"),
    ("conv bwd-data", r"igemm_bwd|bwd_data|ConvBwdData"),
    ("conv bwd-weight", r"igemm_wrw|bwd_weight|ConvBwdWeight|wrw"),
    ("gemm", r"Cijk_|gemm|Gemm"),
    ("batchnorm (MIOpen)", r"BatchNorm"),
    ("miopen tensor ops", r"SubTensorOp|OpTensor|TensorOp"),
    ("relu/threshold", r"threshold|clamp"),
    ("elementwise add", r"CUDAFunctor_add|add_kernel"),
    ("casts/copies", r"copy_kernel|copyBuffer|bfloat16_copy|float32_copy|fillBuffer|FillBuffer"),
    ("pooling", r"pool"),
    ("reduce/softmax/loss", r"reduce|softmax|nll|cross_entropy|log_softmax"),
    ("rccl", r"ncclDevKernel|nccl|rccl"),
]


def main(path, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = {}
    names = {}
    grand = 0.0
    for r in rows:
        n = r["Name"]
        t = float(r["TotalDurationNs"]) / 1e6
        grand += t
        cat = "other"
        for c, pat in CATS:
            if re.search(pat, n):
                cat = c
                break
        tot[cat] = tot.get(cat, 0.0) + t
        names.setdefault(cat, []).append((t, n[:90], int(r["Calls"])))
    div = float(steps) if steps else 1.0
    unit = "ms/step" if steps else "ms total"
    print(f"{'category':28s} {unit:>10s} {'share':>7s}")
    for c, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{c:28s} {t / div:10.3f} {100 * t / grand:6.1f}%")
    print(f"{'TOTAL GPU busy':28s} {grand / div:10.3f}")
    if "-v" in sys.argv:
        for c in tot:
            print("\n#", c)
            for t, n, k in sorted(names[c], reverse=True)[:8]:
                print(f"  {t / div:8.3f}  x{k:<5d} {n}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-v" else None)
