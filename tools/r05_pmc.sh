#!/bin/bash
# round-5: SQ counter passes over the gzip lab kernel (one rocprofv3 --pmc run per counter set)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}; mkdir -p $O
B=${2:-new}; N=${3:-15625}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/p$i -o pmc --output-format csv -- tools/labbin/gzip_lab_$B $N 1 > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
tot = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gzip" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:24s} {v:16.0f}")
PY
