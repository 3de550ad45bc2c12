#!/bin/bash
# r02 session Y: zstd tests on the packed sequence tables; C5 / blosc-zstd A/B of the sequence
# decoder's table format and occupancy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_c3c5.py tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in pack0 pack1 pack1w6 pack0 pack1w6; do
  for w in c5 blosc-zstd; do
    echo "== $v $w"
    ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$v.json 2> $O/${w}_$v.err || { echo "rc=$?"; tail -3 $O/${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== done"
