#!/bin/bash
# r02 session S: blosc lz4/blosclz LDS output ring A/B; blosc tests on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
echo "== pytest blosc"
timeout -k 10 600 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in ring0 ring4k ring8k ring0 ring4k; do
  echo "== $v blosc"
  ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 300 python bench.py --workload blosc --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/blosc_$v.json 2> $O/blosc_$v.err || { echo "rc=$?"; tail -3 $O/blosc_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/blosc_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
done
echo "== done"
