#!/bin/bash
# r02 session R: blosc / blosc-zstd kernel breakdowns (rocprof) on the current build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02r
mkdir -p $O
for w in blosc-zstd blosc; do
  echo "== rocprof $w"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu --no-pmc --no-host-leg --steps 10 --warmup 2 > $O/prof_$w.json 2> $O/prof_$w.err || { echo "rocprof rc=$?"; exit 1; }
  python3 - <<PY
import csv
for r in list(csv.DictReader(open("$O/prof_$w/run_kernel_stats.csv")))[:10]:
    print(" ", r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e3,1), "us", r["Percentage"][:5])
PY
done
echo "== done"
