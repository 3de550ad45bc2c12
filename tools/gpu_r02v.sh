#!/bin/bash
# r02 session V: gzip parity (block types / strategies, periodic content) on the current build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py -v -m gpu -x -k gzip --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -15; echo "pytest rc=$rc"
exit $rc
