#!/bin/bash
# r02 session U: gzip tail effect (15360 = 3 full rounds of 5120 resident waves vs 15625 streams)
# and the PMC instruction mix of the current k_gzip.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02u
mkdir -p $O
G=zarrs_amd/lib_variants/gz/xdep1
for n in 15625 15360 10240 5120 15625; do
  echo "== lab n=$n"
  timeout -k 10 120 $G $n 1 > $O/lab_$n.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lab_$n.txt; exit 1; }
  grep k_gzip $O/lab_$n.txt
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/gzpmc1 -o p --output-format csv -- $G 15625 1 > $O/gzpmc1.txt 2>&1
echo "pmc rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d $O/gzpmc2 -o p --output-format csv -- $G 15625 1 > $O/gzpmc2.txt 2>&1
echo "pmc rc=$?"
python3 - <<'PY'
import csv, collections, glob
for d in ("gzpmc1", "gzpmc2"):
    for f in glob.glob(f"gpurun_out/r02u/{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float); n = collections.Counter()
        for row in csv.DictReader(open(f)):
            if "k_gzip" in row["Kernel_Name"]:
                agg[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
        for k, v in sorted(agg.items()):
            print(k, round(v / n[k] / 15625))
PY
echo "== done"
