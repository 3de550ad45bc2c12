#!/bin/bash
# r02 session 2, call G2: prefetched CRC segments: GPU tests, lab, C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2g2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./lab_bin/gzip_lab_crc2 15625 1 > $O/lab_crc.txt 2>&1 || { echo "lab rc=$?"; cat $O/lab_crc.txt; exit 1; }
grep k_gzip $O/lab_crc.txt
timeout -k 10 500 python bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench rc=$?"; tail -5 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== done"
