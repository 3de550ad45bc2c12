#!/bin/bash
# r02 session 2, call O: executor segments per item adaptive to the batch size (ZGPU_ZSTD_XSEG=4: fixed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3c5.py tests/test_gpu_codecs.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for x in "" 4 "" 4 8; do
  ZGPU_ZSTD_XSEG=$x timeout -k 10 400 python bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/c5_x$x.json 2> $O/c5_x$x.err || { echo "rc=$?"; tail -3 $O/c5_x$x.err; exit 1; }
  echo "xseg=${x:-adaptive} $(python -c "import json; d=json.load(open('$O/c5_x$x.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
done
echo "== done"
