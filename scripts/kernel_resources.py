#!/usr/bin/env python
"""Per-kernel VGPR / AGPR / scratch / occupancy of one HIP source, from hipcc's
``-Rpass-analysis=kernel-resource-usage`` remarks (no GPU needed).

usage: python scripts/kernel_resources.py layer_wise_aaai20_amd/csrc/conv.hip [--spills]
"""
import os
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    only_spill = "--spills" in sys.argv
    inc = os.path.dirname(os.path.abspath(src))
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
                        src, "-o", "/tmp/_kr.o", f"-I{inc}",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (?:\S+: )?\s*(.*?) \[-Rpass", line)
        if not m:
            continue
        body = m.group(1)
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            cur[k.strip()] = v.strip()
    names = subprocess.run(["c++filt"], input="\n".join(r_["name"] for r_ in rows),
                           capture_output=True, text=True).stdout.splitlines()
    for r_, n in zip(rows, names):
        scratch = int(r_.get("ScratchSize [bytes/lane]", "0"))
        if only_spill and scratch == 0:
            continue
        n = n.replace("(lw::GemmK)", "").replace("void lw::", "")
        print(f"{n[:70]:70s} vgpr={r_.get('VGPRs', '?'):>4} agpr={r_.get('AGPRs', '?'):>3} "
              f"scratch={scratch:>4} occ={r_.get('Occupancy [waves/SIMD]', '?')}")
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)


if __name__ == "__main__":
    main()
