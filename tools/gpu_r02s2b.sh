#!/bin/bash
# r02 session 2, call B: gzip lab A/B — wide lookahead windows (WIDE=2/3/4) + subtables vs HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2b
mkdir -p $O
for v in base nw0 nw2 nw3 nw4 w0 w4 w3; do
  echo "== $v"
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -5 $O/lab_$v.txt; exit 1; }
  cat $O/lab_$v.txt
done
echo "== done"
