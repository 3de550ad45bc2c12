#!/bin/bash
# Full GPU session: parity tests, then bench lines (+ rocprof kernel stats) for the given workloads.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> [workloads...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}; shift
WL=${@:-c2 c3 c5}
O=gpurun_out/$TAG
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in $WL; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w rc=$?"; tail -5 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
  echo "== rocprof $w"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_$w.json 2> $O/prof_$w.err || { echo "rocprof $w rc=$?"; exit 1; }
done
echo "== done"
