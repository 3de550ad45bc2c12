#!/bin/bash
# r02 session 2, call M: zstd sequence decoder forked onto a side stream beside the literal kernels:
# GPU tests, then C5 / blosc-zstd with the fork on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02s2m}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in 1 0 1; do
  for w in c5 blosc-zstd; do
    ZGPU_ZSTD_FORK=$f timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_f$f.json 2> $O/${w}_f$f.err || { echo "rc=$?"; tail -3 $O/${w}_f$f.err; exit 1; }
    echo "fork=$f $w $(python -c "import json; d=json.load(open('$O/${w}_f$f.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
  done
done
echo "== done"
