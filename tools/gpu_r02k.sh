#!/bin/bash
# r02 session K: C5 A/B of the literal-decoder grid (ZGPU_ZSTD_LGRID) and the FSE table layout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
for lib in zarrs_amd/lib/libzgpu.so zarrs_amd/lib_variants/oldseq/libzgpu.so; do
  for lg in 512 1024 2048; do
    n=$(basename $(dirname $lib))_$lg
    echo "== $n"
    ZGPU_LIB=$lib ZGPU_ZSTD_LGRID=$lg timeout -k 10 400 python bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/c5_$n.json 2> $O/c5_$n.err || { echo "rc=$?"; tail -3 $O/c5_$n.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c5_$n.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== done"
