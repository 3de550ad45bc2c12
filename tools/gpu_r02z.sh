#!/bin/bash
# r02 session Z: C5 kernel timeline on concurrent streams (which level's kernels finish last).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || { echo "rocprof rc=$?"; tail -5 $O/c5.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r02z/kt/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "zgpu" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step: the last 1/4 of the zgpu dispatches (steps: warmup 1 + 3 timed + roundtrip checks...)
t_end = int(rows[-1]["End_Timestamp"])
# find step boundaries by k_zstd_scan dispatches per stream: take the last 16 zgpu scan... simply print the last 60 dispatches
last = rows[-64:]
t0 = min(int(r["Start_Timestamp"]) for r in last)
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{r["Kernel_Name"].split("(")[0][6:]:22s} q{r.get("Queue_Id","?"):>3} s{r.get("Stream_Id","?"):>3} grid {r["Grid_Size_X"]:>8} start {(s-t0)/1e6:8.2f} end {(e-t0)/1e6:8.2f} dur {(e-s)/1e6:7.2f} ms')
PY
