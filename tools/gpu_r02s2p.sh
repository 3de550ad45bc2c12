#!/bin/bash
# r02 session 2, call P: gzip match readiness by source index range (no LDS read per round) A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02s2p
mkdir -p $O
for v in r0 r1 r0 r1; do
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "$v rc=$?"; cat $O/lab_$v.txt; exit 1; }
  echo "$v $(grep k_gzip $O/lab_$v.txt)"
done
