#!/bin/bash
# r02 session 2, call I: C5 kernel trace on the concurrent lanes (critical path of one step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2i
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --steps 2 --warmup 1 > $O/c5.json 2> $O/c5.err || { echo "rocprof rc=$?"; tail -5 $O/c5.err; exit 1; }
cat $O/c5.json
echo "== done"
