#!/bin/bash
# r02 session 2, call Z: LZ stream decoders (lz4 / blosclz / snappy) copy 1 / 4 / 8 bytes per lane per
# step: blosc GPU tests on the default build, then blosc lz4 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2z
mkdir -p $O
make -s -C zarrs_amd/csrc >/dev/null 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_blosc.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_blosc.log; exit 1; }
tail -1 $O/pytest_blosc.log
for v in u1 u4 u8 u1 u4; do
  ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload blosc --no-pmc --no-host-leg --no-cpu --steps 20 --warmup 3 > $O/blosc_$v.json 2> $O/blosc_$v.err || { echo "rc=$?"; tail -3 $O/blosc_$v.err; exit 1; }
  echo "$v $(python -c "import json; d=json.load(open('$O/blosc_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
done
echo "== done"
