#!/bin/bash
# r02 session C: blosc / blosclz parity, then the zstd LDS-size A/B (session B's script).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== bench blosc (lz4)"
timeout -k 10 300 python bench.py --workload blosc --no-pmc --no-host-leg --cpu-seconds 5 > $O/bench_blosc.json 2> $O/bench_blosc.err || { echo "rc=$?"; tail -3 $O/bench_blosc.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_blosc.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'], d['cpu_baseline']['value'])"
bash tools/gpu_r02b.sh
