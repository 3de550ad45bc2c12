#!/bin/bash
# r02 session F: gzip lab phase profile; blosc tests (cached layout); C3 bench with PMC + rocprof;
# blosc / blosc-zstd / C5 bench lines with PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
for v in prof_cur prof_x16 x0 x8 x16; do
  echo "== lab $v"
  timeout -k 10 120 zarrs_amd/lib_variants/gz/$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$v.txt; exit 1; }
  grep -A6 k_gzip $O/lab_$v.txt
done
echo "== pytest blosc"
timeout -k 10 600 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in c3 blosc blosc-zstd c5; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w --no-host-leg --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], r['alg_bytes_per_launch'], d['cpu_baseline']['value'])"
done
echo "== rocprof c3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== done"
