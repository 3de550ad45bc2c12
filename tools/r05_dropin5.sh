#!/bin/bash
# round 5: C3 drop-in policy sweep with the 3-D DMA pack (default 4 HIP queues)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin5}; mkdir -p $O
run() {  # MC WIN env...
  local mc=$1 win=$2; shift 2
  echo "== mc=$mc win=$win $*"
  env "$@" timeout -k 10 240 python -u tools/dropin_sweep.py $mc $win 2>> $O/err.txt | tail -1 || exit 1
}
run 4 200 ZGPU_CTX_LANES=8
run 8 500 ZGPU_CTX_LANES=8
run 8 1000 ZGPU_CTX_LANES=4
run 16 2000 ZGPU_CTX_LANES=3
run 16 2000 ZGPU_CTX_LANES=2
run 16 4000 ZGPU_CTX_LANES=2
run 4 200 ZGPU_CTX_LANES=8 ZGPU_CO_HIPRIO=0
