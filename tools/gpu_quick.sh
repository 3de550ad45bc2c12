#!/bin/bash
# Targeted GPU iteration: selected parity tests, then one workload's bench line + rocprof kernel stats.
# Usage: gpurun --timeout 900 -- bash tools/gpu_quick.sh <tag> <pytest -k expr|all> <workload|none>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-quick}; K=${2:-all}; W=${3:-none}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$K" = "all" ]; then KA=""; else KA="-k $K"; fi
echo "== pytest -m gpu $KA"
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread $KA > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
[ "$W" = "none" ] && exit 0
echo "== bench $W"
timeout -k 10 400 python bench.py --workload $W --no-pmc --no-host-leg --cpu-seconds 5 > $O/bench_$W.json 2> $O/bench_$W.err || { echo "bench rc=$?"; tail -5 $O/bench_$W.err; exit 1; }
cat $O/bench_$W.json
echo "== rocprof $W"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python3 bench.py --workload $W --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_$W.json 2> $O/prof_$W.err || { echo "rocprof rc=$?"; exit 1; }
echo "== done"
