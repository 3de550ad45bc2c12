#!/bin/bash
# r02 session L: C5 A/B of the Huffman-table split and the literal decoder's occupancy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
for v in nosplit split2 split3 nosplit split3; do
  for w in c5 blosc-zstd; do
    echo "== $v $w"
    ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$v.json 2> $O/${w}_$v.err || { echo "rc=$?"; tail -3 $O/${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== done"
