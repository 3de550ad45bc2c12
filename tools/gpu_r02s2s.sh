#!/bin/bash
# r02 session 2, call S: nested sharding (parity vs the oracle, fill / checksum / OOB errors), full suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -k "nested or transpose_then or sharded" > $O/pytest_n.log 2>&1 || { echo "pytest n rc=$?"; tail -40 $O/pytest_n.log; exit 1; }
tail -1 $O/pytest_n.log
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --workload c3 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -3 $O/c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['value'], d['ms_per_step'], d['roundtrip_ok'])"
