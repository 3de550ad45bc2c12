#!/bin/bash
# round 5: zstd lab variants under one rocprofv3 FETCH_SIZE pass each (512 C5 L0 chunks, 3 reps)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-zpmc}; shift; mkdir -p $O
for b in "$@"; do
  echo "== $b"
  timeout -k 5 300 tools/labbin/$b 512 16 3 c5 | grep -E "lits|exec_item|blocks |total" || exit 1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/$b -o pmc --output-format csv -- tools/labbin/$b 512 16 3 c5 > /dev/null 2>&1 || exit 1
  python3 - "$O/$b" <<'PY'
import csv, glob, os, sys, collections
acc = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE":
            k = r["Kernel_Name"].split("(")[0]; acc[k] += float(r["Counter_Value"]); cnt[k] += 1
for k, v in sorted(acc.items(), key=lambda kv: -kv[1])[:6]:
    print(f"   FETCH x2 per launch {k[:40]:40s} {2 * v * 1024 / cnt[k] / 1e6:10.1f} MB")
PY
done
