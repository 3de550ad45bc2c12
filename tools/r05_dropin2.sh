#!/bin/bash
# round 5: C3 drop-in with lanes on CU-mask streams (own hardware queues) at the default queue count
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin2}; mkdir -p $O
for cfg in "ZGPU_LANE_QUEUES=1 ZGPU_CTX_LANES=8" "ZGPU_LANE_QUEUES=1 ZGPU_CTX_LANES=16" "ZGPU_LANE_QUEUES=1 ZGPU_CTX_LANES=8 ZGPU_CO_HIPRIO=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 240 python -u tools/dropin_sweep.py 4 200 2>> $O/err.txt | tail -1 || exit 1
done
