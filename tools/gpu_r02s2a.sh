#!/bin/bash
# r02 session 2, call A: state check after the container re-creation (full GPU tests, smoke, bench lines).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2a
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo "== smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in c2 c3 c5; do
  echo "== bench $w"
  timeout -k 10 400 python bench.py --workload $w --no-pmc > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w rc=$?"; tail -5 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
done
echo "== done"
