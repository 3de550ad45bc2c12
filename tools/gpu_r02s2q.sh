#!/bin/bash
# r02 session 2, call Q: gzip pipelined lookahead blocks (next block's lane symbols decoded while the
# current block is chained) A/B, then the gzip GPU tests on the product build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2q
mkdir -p $O
for v in q0 q1 q0 q1; do
  timeout -k 10 120 ./lab_bin/gzip_lab_$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "$v rc=$?"; cat $O/lab_$v.txt; exit 1; }
  echo "$v $(grep k_gzip $O/lab_$v.txt)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_c3c5.py tests/test_gpu_parity.py tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
