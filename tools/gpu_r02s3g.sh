#!/bin/bash
# r02 session 3, call G: unshuffle fast path for u16 / u32 — blosc GPU tests, A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blosc.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_blosc.log 2>&1 || { echo "pytest blosc rc=$?"; tail -40 $O/pytest_blosc.log; exit 1; }
tail -1 $O/pytest_blosc.log
for v in fast base fast base; do
  L=zarrs_amd/lib_variants/u$v/libzgpu.so
  for c in blosc blosc-zstd; do
    ZGPU_LIB=$L timeout -k 10 200 python bench.py --workload $c --no-pmc --no-cpu --no-host-leg > $O/b_${c}_$v.json 2> $O/b_${c}_$v.err || { echo "bench $c $v rc=$?"; tail -5 $O/b_${c}_$v.err; exit 1; }
    echo "$c $v $(python -c "import json; d=json.load(open('$O/b_${c}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
  done
done
echo "== done"
