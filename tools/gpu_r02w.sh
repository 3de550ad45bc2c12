#!/bin/bash
# r02 session W: gzip parity (block types); C5 / blosc-zstd A/B of the executor ring and far-source
# staging sizes on the current build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py -v -m gpu -x -k gzip --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -12; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in x16 x8s256 x8 x16 x8s256; do
  for w in c5 blosc-zstd; do
    echo "== $v $w"
    ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$v.json 2> $O/${w}_$v.err || { echo "rc=$?"; tail -3 $O/${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== done"
