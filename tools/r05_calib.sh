#!/bin/bash
# round 5: FETCH_SIZE / WRITE_SIZE calibration per access width (tools/lab/fetch_calib.hip)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-calib}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- tools/labbin/fetch_calib || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- tools/labbin/fetch_calib || exit 1
python3 - "$O" <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for ctr, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    for f in glob.glob(os.path.join(O, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != ctr:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "flush" in k:
                continue
            print(f"{ctr:10s} {k:40s} {float(r['Counter_Value']) * 1024 / 2**30:8.3f} GiB (raw, of 1 GiB moved; wr_plane 0.5)")
PY
