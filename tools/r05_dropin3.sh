#!/bin/bash
# round 5: C3 drop-in policy sweep at the default 4 HIP queues (each configuration a fresh process)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin3}; mkdir -p $O
run() {  # MC WIN env...
  local mc=$1 win=$2; shift 2
  echo "== mc=$mc win=$win $*"
  env "$@" timeout -k 10 240 python -u tools/dropin_sweep.py $mc $win 2>> $O/err.txt | tail -1 || exit 1
}
run 4 200 ZGPU_CTX_LANES=8
run 4 200 ZGPU_CTX_LANES=4 ZGPU_CO_HIPRIO=0
run 16 2000 ZGPU_CTX_LANES=4
run 16 2000 ZGPU_CTX_LANES=2
run 8 1000 ZGPU_CTX_LANES=3 ZGPU_CO_HIPRIO=0
