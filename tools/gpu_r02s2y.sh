#!/bin/bash
# r02 session 2, call Y: precomputed x^(2^k) CRC tables: GPU tests, C3 10-step line + kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2y
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 10 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
python -c "import json; d=json.load(open('$O/prof_c3.json')); print('c3', d['value'], d['ms_per_step'], d['roundtrip_ok'])"
