#!/bin/bash
# A/B of libzgpu.so variants (tools/lab/build_variants.sh) on one workload: each variant's bench line
# (no CPU baseline, no PMC, no host leg, no secondary legs), interleaved twice.
# Usage: gpurun -- bash tools/ab.sh <tag> <workload> <steps> base <variant> [<variant> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; W=$2; N=$3; shift 3
O=gpurun_out/$TAG
mkdir -p "$O"
for rep in 1 2; do
  for v in "$@"; do
    # a variant is a library under zarrs_amd/lib_variants/, or NAME=VALUE: the base library with that
    # environment variable set
    lib=""; ev=""
    case "$v" in base) ;; *=*) ev=$v ;; *) lib=zarrs_amd/lib_variants/$v/libzgpu.so ;; esac
    ( [ -n "$ev" ] && export "$ev"; ZGPU_LIB=$lib timeout -k 10 400 python -u bench.py --workload "$W" --no-cpu \
      --no-pmc --no-host-leg --secondary= --steps "$N" --warmup 2 ) > "$O/$v.$rep.json" 2> "$O/$v.$rep.err" \
      || { echo "$v rc=$?"; tail -5 "$O/$v.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/$v.$rep.json')); print('$v', $rep, d['value'], d['unit'], d['ms_per_step'], 'ms', 'ok' if d['roundtrip_ok'] else 'MISMATCH')"
  done
done
