#!/bin/bash
# One GPU-box session: parity tests, the default bench line (CPU baseline + PMC traffic passes +
# host leg), and a rocprofv3 kernel-trace summary of the same bench command.
# Usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_full.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 420 python -m pytest tests -q -m gpu -x > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== bench" && \
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
echo "== rocprof stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --no-host-leg > $O/bench_prof.json 2> $O/bench_prof.err && \
cat $O/bench_prof.json && echo "== done"
