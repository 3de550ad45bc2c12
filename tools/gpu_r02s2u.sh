#!/bin/bash
# r02 session 2, call U: gzip 1 KiB ring at 6 waves/SIMD (smaller subtable spaces) vs 2 KiB at 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02s3a
mkdir -p $O
for v in c3 c2 c4 c3 c2; do
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "$v rc=$?"; cat $O/lab_$v.txt; exit 1; }
  echo "$v $(grep k_gzip $O/lab_$v.txt)"
done
