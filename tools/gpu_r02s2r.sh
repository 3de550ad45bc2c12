#!/bin/bash
# r02 session 2, call R: transpose codecs before sharding_indexed (parity vs the oracle), full suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "transpose" > $O/pytest_t.log 2>&1 || { echo "pytest t rc=$?"; tail -40 $O/pytest_t.log; exit 1; }
tail -1 $O/pytest_t.log
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
