#!/bin/bash
# r02 session M: zstd/blosc/C3C5 GPU tests on the final zstd defaults, then C5 (with PMC), blosc-zstd,
# C3 (with PMC) bench lines and a C3 rocprof summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
echo "== gzip lab profile"
timeout -k 10 120 zarrs_amd/lib_variants/gz/prof 15625 1 > $O/lab_prof.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_prof.txt; exit 1; }
grep -A8 k_gzip $O/lab_prof.txt
echo "== pytest zstd paths"
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_c3c5.py tests/test_gpu_blosc.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in c5 blosc-zstd c3; do
  echo "== bench $w"
  timeout -k 10 900 python bench.py --workload $w --no-host-leg --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], r['alg_bytes_per_launch'], (d['cpu_baseline'] or {}).get('value'))"
done
echo "== rocprof c3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== done"
