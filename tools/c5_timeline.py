"""Timeline of the last bench step in a rocprofv3 kernel trace (bench.py --workload c5 under
`tools/gpu.sh prof:c5`): every zgpu kernel of the step with its stream, start and end (ms from the
step's first dispatch) - which plan's kernels make the step's critical path."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "zgpu::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# argv[2]: the step's start (ms after the trace's first zgpu dispatch; the scans of one step start
# together), argv[3]: its length bound (ms)
at, span = float(sys.argv[2]), float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
T = int(rows[0]["Start_Timestamp"])
step = [r for r in rows if at <= (int(r["Start_Timestamp"]) - T) / 1e6 < at + span]
t0 = int(step[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in step)
print(f"step: {len(step)} zgpu dispatches, {(end - t0) / 1e6:.2f} ms")
busy = {}
for r in step:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    name = r["Kernel_Name"].split("(")[0].replace("zgpu::", "")
    q = r["Stream_Id"]
    busy[q] = busy.get(q, 0) + e - s
    print(f"  stream {q:>3}  {name:<28} grid {int(r['Grid_Size_X']):>8}  {s:8.2f} -> {e:8.2f}  ({e - s:7.2f} ms)")
for q, b in sorted(busy.items()):
    print(f"stream {q}: kernels busy {b:.2f} ms")
