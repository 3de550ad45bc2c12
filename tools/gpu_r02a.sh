#!/bin/bash
# r02 session A: full GPU parity suite, default C2 bench line, C5 bench + rocprof with plans serialised
# on one stream (true per-kernel durations) and the zstd path counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== bench c2"
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench c2 rc=$?"; tail -5 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
echo "== rocprof c5 (serial lanes)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --serial-lanes --no-pmc --no-host-leg --cpu-seconds 5 --steps 5 --warmup 1 > $O/prof_c5.json 2> $O/prof_c5.err || { echo "rocprof c5 rc=$?"; tail -5 $O/prof_c5.err; exit 1; }
cat $O/prof_c5.json
echo "== done"
