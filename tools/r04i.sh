# round-4 session: full GPU tests, C3 drop-in leg, literal-window A/B on C5 (scale 2) with FETCH_SIZE
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit $rc; }
timeout -k 10 600 python -u bench.py --workload c3 --no-pmc --no-cpu --secondary= --steps 3 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
for rep in 1 2; do for v in base gwin3; do
  lib=""; [ $v != base ] && lib=zarrs_amd/lib_variants/$v/libzgpu.so
  ZGPU_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --c5-scale 2 --no-cpu --no-pmc --no-host-leg --secondary= --steps 5 --warmup 2 > $O/c5_$v.$rep.json 2> $O/c5_$v.$rep.err || { echo "$v failed"; tail -5 $O/c5_$v.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], d['roundtrip_ok'])"
done; done
for v in base gwin3; do
  lib=""; [ $v != base ] && lib=$PWD/zarrs_amd/lib_variants/$v/libzgpu.so
  ZGPU_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_zstd_lits -d $O/pmc_$v -o pmc --output-format csv -- python3 bench.py --workload c5 --c5-scale 2 --child --no-cpu --no-pmc --no-host-leg --steps 2 --warmup 1 > /dev/null 2> $O/pmc_$v.err || { echo "pmc $v failed"; tail -5 $O/pmc_$v.err; exit 1; }
  python3 - $O/pmc_$v <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f)) if "k_zstd_lits" in r["Kernel_Name"]]
print(sys.argv[1], "k_zstd_lits FETCH_SIZE KiB per step (raw counter):", sum(v) / 3)
PY
done
timeout -k 10 200 ./labx/gzip_lab_prof 15625 > $O/gzip_lab_prof.txt 2>&1 || { echo "gzip_lab_prof failed"; tail -5 $O/gzip_lab_prof.txt; exit 1; }
cat $O/gzip_lab_prof.txt
echo done
