#!/bin/bash
# r02 session G: blosc tests (cached layout); C3 bench with PMC + rocprof; blosc / blosc-zstd / C5
# bench lines with PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
echo "== pytest blosc"
timeout -k 10 600 python -u -m pytest tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in c3 blosc blosc-zstd c5; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w --no-host-leg --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], r['alg_bytes_per_launch'], d['cpu_baseline']['value'])"
done
echo "== rocprof c3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== gzip lab PMC"
G=zarrs_amd/lib_variants/gz/cur
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/gzpmc1 -o p --output-format csv -- $G 15625 1 > $O/gzpmc1.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d $O/gzpmc2 -o p --output-format csv -- $G 15625 1 > $O/gzpmc2.txt 2>&1
echo "pmc rc=$?"
echo "== done"
