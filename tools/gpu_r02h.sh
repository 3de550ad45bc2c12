#!/bin/bash
# r02 session H: gzip lab A/B of the pointer-jumping symbol chain; C5 PMC (device memory released
# before the profiled child).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
for v in pj0 pj1 prof_pj1 pj0 pj1; do
  echo "== lab $v"
  timeout -k 10 120 zarrs_amd/lib_variants/gz/$v 15625 1 > $O/lab_$v.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$v.txt; exit 1; }
  grep -A6 k_gzip $O/lab_$v.txt | grep -v " 0 cycles"
done
G=zarrs_amd/lib_variants/gz/pj1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/gzpmc1 -o p --output-format csv -- $G 15625 1 > $O/gzpmc1.txt 2>&1
echo "pmc rc=$?"
echo "== bench c5 (PMC)"
timeout -k 10 900 python bench.py --workload c5 --no-host-leg --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || { echo "rc=$?"; tail -3 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], str(r['traffic_detail'])[:300])"
echo "== done"
