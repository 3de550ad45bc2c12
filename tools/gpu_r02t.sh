#!/bin/bash
# r02 session T: C5 record (bench with PMC + CPU baseline), serialised-lanes kernel split, blosc
# lines with PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02t
mkdir -p $O
for w in c5 blosc blosc-zstd; do
  echo "== bench $w"
  timeout -k 10 900 python bench.py --workload $w --no-host-leg --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], r['alg_bytes_per_launch'], (d['cpu_baseline'] or {}).get('value'))"
done
echo "== rocprof c5 serial lanes"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5s -o run --output-format csv -- python3 bench.py --workload c5 --serial-lanes --no-pmc --no-host-leg --no-cpu --steps 5 --warmup 1 > $O/prof_c5s.json 2> $O/prof_c5s.err || { echo "rocprof c5 rc=$?"; tail -5 $O/prof_c5s.err; exit 1; }
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r02t/prof_c5s/run_kernel_stats.csv")))[:9]:
    print(" ", r["Name"][:40], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms", r["Percentage"][:5])
PY
echo "== done"
