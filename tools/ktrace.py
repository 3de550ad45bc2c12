"""Summarise a rocprofv3 kernel trace: per-kernel totals and the last step's launches in order."""
import csv, sys
path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = [r for r in csv.DictReader(open(path)) if "zgpu" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tot = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("zgpu::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    t = tot.setdefault(k, [0, 0.0])
    t[0] += 1; t[1] += d
for k, (n, s) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"{k:40s} n={n:5d} total={s:10.3f} ms avg={s/n:8.3f} ms")
print("-- last launches")
for r in rows[-last:]:
    k = r["Kernel_Name"].split("(")[0].replace("zgpu::", "")
    print(f'{k:40s} grid={int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"]):7d} lds={r["LDS_Block_Size"]:>6s} vgpr={r["VGPR_Count"]:>4s} {(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6:9.3f} ms')
