#!/bin/bash
# Bench lines for every workload + rocprofv3 kernel stats of each. Usage: gpurun -- bash tools/gpu_bench.sh <tag> [workloads...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}; shift
WL=${@:-c2 c3}
O=gpurun_out/$TAG
mkdir -p $O
for w in $WL; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w rc=$?"; tail -5 $O/bench_$w.err; exit 1; }
  cat $O/bench_$w.json
  echo "== rocprof $w"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu --no-pmc --no-host-leg --steps 10 > $O/prof_$w.json 2> $O/prof_$w.err || { echo "rocprof $w rc=$?"; exit 1; }
done
echo "== done"
