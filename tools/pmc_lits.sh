#!/bin/bash
# Lab (not product): HBM bytes of k_zstd_lits on 64 C5 L0 chunks (FETCH_SIZE / WRITE_SIZE passes,
# one counter each), with the literal record slots on and off (LAB_NOREC=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06zn
mkdir -p $O
for rec in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    E=(); [ $rec = 1 ] && E=(LAB_NOREC=1)
    env "${E[@]}" LAB_REPS=1 timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_zstd_lits|k_zstd_huf" \
      -d $O/p_${rec}_$c -o p --output-format csv -- tools/labbin/zstd_lab 64 16 3 c5 > $O/lab_${rec}_$c.txt 2>&1 || { echo "pass $rec $c rc=$?"; exit 1; }
    f=$(ls $O/p_${rec}_$c/*counter_collection.csv $O/p_${rec}_$c/*/*counter_collection.csv 2>/dev/null | head -1)
    python3 - "$f" "$c" "$rec" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == sys.argv[2]:
        acc[r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"])
for k, v in acc.items():
    mult = 2 if sys.argv[2] == "FETCH_SIZE" else 1
    print(f"norec={sys.argv[3]} {sys.argv[2]} {k}: {v * 1024 * mult / 1e6:.1f} MB")
PY
  done
done
grep -h "encoded\|lits " $O/lab_0_FETCH_SIZE.txt | head -3
