"""Timeline of the last step of a multi-stream rocprofv3 kernel trace (C5's four lanes): per stream,
each kernel's start / end in ms from the step's first launch. Usage: c5_timeline.py trace.csv [n_last]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "zgpu" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
# the last step: launches after the largest gap between consecutive kernel starts in the last 300
tail = rows[-300:]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), i + 1) for i, (a, b) in enumerate(zip(tail, tail[1:]))]
cut = max(gaps)[1] if not n_last else len(tail) - n_last
step = tail[cut:]
t0 = min(int(r["Start_Timestamp"]) for r in step)
key = "Stream_Id" if "Stream_Id" in step[0] else "Queue_Id"
by = {}
for r in step:
    by.setdefault(r[key], []).append(r)
end_all = max(int(r["End_Timestamp"]) for r in step)
print(f"step: {len(step)} launches, {(end_all - t0) / 1e6:.2f} ms")
for s, rs in sorted(by.items(), key=lambda kv: int(kv[1][0]["Start_Timestamp"])):
    print(f"-- {key} {s}: ends at {(max(int(r['End_Timestamp']) for r in rs) - t0) / 1e6:.2f} ms")
    for r in rs:
        k = r["Kernel_Name"].split("(")[0].replace("zgpu::", "").replace("void ", "")
        a, b = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
        print(f"   {k:28s} {a:8.2f} -> {b:8.2f}  ({b - a:7.2f} ms)")
