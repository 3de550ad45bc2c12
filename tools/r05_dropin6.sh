#!/bin/bash
# round 5: C3 drop-in with a cap on concurrent coalesced batches (ZGPU_CO_INFLIGHT), 8 lanes, 4 HIP queues
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin6}; mkdir -p $O
run() {  # MC WIN env...
  local mc=$1 win=$2; shift 2
  echo "== mc=$mc win=$win $*"
  env "$@" timeout -k 10 240 python -u tools/dropin_sweep.py $mc $win 2>> $O/err.txt | tail -1 || exit 1
}
run 8 200 ZGPU_CO_INFLIGHT=3
run 16 200 ZGPU_CO_INFLIGHT=3
run 16 200 ZGPU_CO_INFLIGHT=2
run 16 200 ZGPU_CO_INFLIGHT=4
run 16 1000 ZGPU_CO_INFLIGHT=3
run 4 200 ZGPU_CO_INFLIGHT=8
