#!/bin/bash
# round 5: C3 drop-in sweep (lanes x HIP queues x coalescing), each configuration a fresh process
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin}; mkdir -p $O
run() {  # env..., args
  echo "== $*"
  env "$@" timeout -k 10 240 python -u tools/dropin_sweep.py $MC $WIN 2>> $O/err.txt | tail -1 || exit 1
}
MC=4 WIN=200
run ZGPU_CTX_LANES=8
run ZGPU_CTX_LANES=4
run ZGPU_CTX_LANES=16
MC=16 WIN=1000 run ZGPU_CTX_LANES=4
run GPU_MAX_HW_QUEUES=8 ZGPU_CTX_LANES=8
echo "== trace lanes 8"
ZGPU_TRACE=1 ZGPU_CTX_LANES=8 timeout -k 10 240 python -u tools/dropin_sweep.py 4 200 2> $O/trace.txt | tail -1 || exit 1
python3 tools/co_trace.py $O/trace.txt
