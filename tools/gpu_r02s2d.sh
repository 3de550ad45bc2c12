#!/bin/bash
# r02 session 2, call D: gzip lab A/B — subtable sizes / literal root 9 vs 10 / PJ doublings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02s2d
mkdir -p $O
for v in base a a3 b b3 b4 a b3; do
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "$v rc=$?"; tail -5 $O/lab_$v.txt; exit 1; }
  echo "$v $(grep k_gzip $O/lab_$v.txt)"
done
