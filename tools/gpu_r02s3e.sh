#!/bin/bash
# r02 session 3, call E: blosclz workload record (tests, smoke, bench with PMC + CPU, rocprof), then
# the lz4 decoder's instruction mix / wait counters (two --pmc passes of their own).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_r02final.sh r02s3blz blosc-blosclz || exit 1
O=gpurun_out/r02s3e
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p --output-format csv -- python3 bench.py --workload blosc --no-cpu --no-pmc --no-host-leg --steps 2 --warmup 1 > $O/p1.txt 2>&1 || { echo "pmc1 rc=$?"; tail -5 $O/p1.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d $O/p2 -o p --output-format csv -- python3 bench.py --workload blosc --no-cpu --no-pmc --no-host-leg --steps 2 --warmup 1 > $O/p2.txt 2>&1 || { echo "pmc2 rc=$?"; tail -5 $O/p2.txt; exit 1; }
echo "== done"
