#!/bin/bash
# r02 session 2, call F: blosc zlib streams (GPU tests), full GPU suite, gzip PJL 2 vs 3 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_blosc.log 2>&1 || { echo "pytest blosc rc=$?"; tail -40 $O/pytest_blosc.log; exit 1; }
tail -1 $O/pytest_blosc.log
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in p3 p2 p3 p2; do
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "$v rc=$?"; exit 1; }
  echo "$v $(grep k_gzip $O/lab_$v.txt)"
done
echo "== done"
