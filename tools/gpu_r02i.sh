#!/bin/bash
# r02 session I: gzip lab A/B (window-word fast path, word copies); C5 bench with PMC; C5 rocprof
# with serialised lanes (per-kernel split at full scale); C2 rocprof including the encode leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
for v in pj1 bw bw_x8 bw_x16 pj1 bw bw_x8; do
  echo "== lab $v"
  timeout -k 10 120 zarrs_amd/lib_variants/gz/$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$v.txt; exit 1; }
  grep k_gzip $O/lab_$v.txt
done
echo "== bench c5 (PMC)"
timeout -k 10 900 python bench.py --workload c5 --no-host-leg --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || { echo "rc=$?"; tail -3 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], str(r['traffic_detail'])[:300])"
echo "== rocprof c5 serial lanes"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5s -o run --output-format csv -- python3 bench.py --workload c5 --serial-lanes --no-pmc --no-host-leg --no-cpu --steps 5 --warmup 1 > $O/prof_c5s.json 2> $O/prof_c5s.err || { echo "rocprof c5 rc=$?"; tail -5 $O/prof_c5s.err; exit 1; }
echo "== rocprof c2 incl. encode leg"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 10 --warmup 2 > $O/prof_c2.json 2> $O/prof_c2.err || { echo "rocprof c2 rc=$?"; tail -5 $O/prof_c2.err; exit 1; }
echo "== done"
