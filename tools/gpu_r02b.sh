#!/bin/bash
# r02 session B: A/B of zstd kernel LDS sizes (exec ring, literal staging, literal grid) on C5 and
# blosc-zstd; each variant is a separate build of libzgpu.so selected with ZGPU_LIB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
run() {  # name lib lgrid workload
  echo "== $1 $4"
  ZGPU_LIB=$2 ZGPU_ZSTD_LGRID=$3 timeout -k 10 400 python bench.py --workload $4 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/$1_$4.json 2> $O/$1_$4.err || { echo "rc=$?"; tail -3 $O/$1_$4.err; return 1; }
  python -c "import json; d=json.load(open('$O/$1_$4.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'], d.get('zstd_items_per_step'))"
}
L=zarrs_amd/lib/libzgpu.so
V=zarrs_amd/lib_variants
for w in blosc-zstd c5; do
  run base $L 512 $w || exit 1
  run r32 $V/r32/libzgpu.so 512 $w || exit 1
  run r16 $V/r16/libzgpu.so 512 $w || exit 1
  run r32l16 $V/r32l16/libzgpu.so 2048 $w || exit 1
  run r16l16 $V/r16l16/libzgpu.so 2048 $w || exit 1
done
echo "== done"
