#!/bin/bash
# r02 session N: gzip lab A/B of exact match dependencies (xdep1) vs the first-pending frontier.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
for v in xdep1 sink xdep1 sink; do
  echo "== lab $v"
  timeout -k 10 120 zarrs_amd/lib_variants/gz/$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$v.txt; exit 1; }
  grep -A8 k_gzip $O/lab_$v.txt | grep -v " 0 cycles"
done
echo "== done"
