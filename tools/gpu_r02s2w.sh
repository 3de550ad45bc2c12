#!/bin/bash
# r02 session 2, call W: gzip 1 KiB ring in the product: GPU tests, C3 line (PMC + CPU), rocprof.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2w
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench rc=$?"; tail -5 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['traffic']/r['alg_bytes_per_launch'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --workload blosc-zstd --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/bz.json 2> $O/bz.err || { echo "bz rc=$?"; exit 1; }
python -c "import json; d=json.load(open('$O/bz.json')); print('blosc-zstd', d['value'], d['ms_per_step'], d['roundtrip_ok'])"
echo "== done"
