import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sgd = [i for i, r in enumerate(rows) if "k_sgd" in r["Kernel_Name"]]
sel = rows[sgd[-2] + 1:sgd[-1] + 1]
ov = 0; tot = 0; maxend = 0; n_ov = 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < maxend:
        n_ov += 1; ov += min(e, maxend) - s
    maxend = max(maxend, e); tot += e - s
print(f"kernels {len(sel)} overlapping starts {n_ov} overlap_us {ov/1e3:.1f} busy_us {tot/1e3:.1f} wall_us {(int(sel[-1]['End_Timestamp'])-int(sel[0]['Start_Timestamp']))/1e3:.1f}")
