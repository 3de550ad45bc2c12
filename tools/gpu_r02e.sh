#!/bin/bash
# r02 session E: gzip lab A/B (lookahead rewrite, ring/occupancy), then gzip/zstd GPU tests with the
# rebuilt library and C3/C5 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
G=zarrs_amd/lib_variants/gz
for v in old_r4096 new_r4096 new_r2048 new_r2048w5 new_r1024w6; do
  echo "== $v"
  timeout -k 10 120 $G/$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$v.txt; exit 1; }
  tail -1 $O/lab_$v.txt
done
echo "== pytest gzip/zstd/c3c5"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3c5.py tests/test_gpu_parity.py tests/test_gpu_codecs.py tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in c3 c5 blosc-zstd; do
  echo "== bench $w"
  timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
done
echo "== done"
