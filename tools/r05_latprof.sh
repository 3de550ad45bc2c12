#!/bin/bash
# round 5: kernel trace of the drop-in latency cases (tools/dropin_latency.py) to split a lone call
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-latprof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o lat -- python3 -u tools/dropin_latency.py > $O/latency.txt 2> $O/lat.err || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
rm -rf $O/prof
python3 - "$O/kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 20 calls of the one-inner-chunk case: the trailing k_gzip dispatches with grid 128 (one stream)
tail = rows[-400:]
prev = None
for r in tail[-60:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    print("%-40s grid %8s  dur %8.1f us  gap %8.1f us" % (r["Kernel_Name"].split("(")[0][-40:], r.get("Grid_Size_X", r.get("Grid_Size", "?")), (e - s) / 1e3, gap))
    prev = e
PY
