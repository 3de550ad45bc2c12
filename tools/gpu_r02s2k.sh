#!/bin/bash
# r02 session 2, call K: C5 stream-lane priorities (lanes: L0 half A, L0 half B, L1, L2-L4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2k
mkdir -p $O
i=0
for p in "-1,-1,0,0" "0,0,-1,0" "-1,-1,-1,0" "0,-1,-1,0" "0,0,-1,-1" "-1,-1,0,0" "0,0,-1,0"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 --lane-priorities=$p > $O/c5_$i.json 2> $O/c5_$i.err || { echo "rc=$?"; tail -3 $O/c5_$i.err; exit 1; }
  echo "prio $p $(python -c "import json; d=json.load(open('$O/c5_$i.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
done
echo "== done"
