#!/bin/bash
# r02 session 2, call J: zstd executor segments per item (XSEG 4 / 8 / 16) on C5 and blosc-zstd.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02s2j
mkdir -p $O
for v in x8 x4 x16 x8; do
  for w in c5; do
    ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$v.json 2> $O/${w}_$v.err || { echo "rc=$?"; tail -3 $O/${w}_$v.err; exit 1; }
    echo "$v $w $(python -c "import json; d=json.load(open('$O/${w}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])")"
  done
done
echo "== done"
