#!/bin/bash
# r02 session 2, call L: blosc snappy streams (GPU tests), then C5 stream-lane priorities A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_blosc.log 2>&1 || { echo "pytest blosc rc=$?"; tail -40 $O/pytest_blosc.log; exit 1; }
tail -1 $O/pytest_blosc.log
bash tools/gpu_r02s2k.sh
