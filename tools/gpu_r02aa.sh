#!/bin/bash
# r02 session AA: zstd tests; C5 / blosc-zstd A/B of the literal decoder's global read window
# (16-B vs 32-B with prefetch) and its grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_c3c5.py tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
run() {  # name lib lgrid
  for w in c5 blosc-zstd; do
    echo "== $1 $w"
    ZGPU_LIB=zarrs_amd/lib_variants/$2/libzgpu.so ZGPU_ZSTD_LGRID=$3 timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$1.json 2> $O/${w}_$1.err || { echo "rc=$?"; tail -3 $O/${w}_$1.err; return 1; }
    python -c "import json; d=json.load(open('$O/${w}_$1.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
}
run gw1 gw1 768 && run gw2 gw2 768 && run gw2g1024 gw2 1024 && run gw1b gw1 768 && run gw2g1024b gw2 1024
echo "== done"
