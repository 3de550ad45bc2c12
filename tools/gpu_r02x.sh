#!/bin/bash
# r02 session X: full GPU suite + smoke on the current build; bench records (PMC + CPU baseline) for
# C5, blosc-zstd, blosc lz4, C3 and the default C2 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in c5 blosc-zstd blosc c3 c2; do
  echo "== bench $w"
  timeout -k 10 900 python bench.py --workload $w --cpu-seconds 10 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['frac'], r['traffic'], r['alg_bytes_per_launch'], (d['cpu_baseline'] or {}).get('value'))"
done
echo "== done"
