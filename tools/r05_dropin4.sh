#!/bin/bash
# round 5: coalescer traces (ZGPU_TRACE=1, tools/co_trace.py) of two drop-in policies
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin4}; mkdir -p $O
for cfg in "16 2000 ZGPU_CTX_LANES=2" "4 200 ZGPU_CTX_LANES=8"; do
  set -- $cfg
  mc=$1 win=$2; shift 2
  echo "== mc=$mc win=$win $*"
  env ZGPU_TRACE=1 "$@" timeout -k 10 240 python -u tools/dropin_sweep.py $mc $win 2> $O/trace_$mc.txt | tail -1 || exit 1
  python3 tools/co_trace.py $O/trace_$mc.txt | tail -14
done
