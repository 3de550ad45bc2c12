#!/bin/bash
# r02 session 2, call T: gzip scatter fused into the flush (direct output for whole chunks): GPU
# tests, C3 with and without it (ZGPU_GZIP_DIRECT=0), the C3 line with PMC traffic, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in 0 1 0 1; do
  ZGPU_GZIP_DIRECT=$f timeout -k 10 400 python bench.py --workload c3 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/c3_d$f.json 2> $O/c3_d$f.err || { echo "rc=$?"; tail -3 $O/c3_d$f.err; exit 1; }
  echo "direct=$f $(python -c "import json; d=json.load(open('$O/c3_d$f.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
done
timeout -k 10 500 python bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench rc=$?"; tail -5 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['traffic']/r['alg_bytes_per_launch'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== done"
