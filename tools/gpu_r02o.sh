#!/bin/bash
# r02 session O: full GPU suite + smoke on the exact-dependency gzip executor; C3 bench (PMC) and
# rocprof; the default C2 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench c3"
timeout -k 10 900 python bench.py --workload c3 --no-host-leg --cpu-seconds 5 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "rc=$?"; tail -3 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['traffic'], r['avg_launch_ms_hip_events'])"
echo "== rocprof c3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof rc=$?"; exit 1; }
echo "== bench c2"
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "rc=$?"; tail -3 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['frac'], r['traffic'])"
echo "== C5 per-kernel WRITE_SIZE / FETCH_SIZE (one step)"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_zstd|k_scatter" -d $O/c5w -o pmc --output-format csv -- python3 bench.py --child --workload c5 --steps 1 --warmup 0 --no-cpu > $O/c5w.log 2>&1
echo "rc=$?"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_zstd|k_scatter" -d $O/c5f -o pmc --output-format csv -- python3 bench.py --child --workload c5 --steps 1 --warmup 0 --no-cpu > $O/c5f.log 2>&1
echo "rc=$?"
python3 - <<'PY'
import csv, glob, collections
for tag in ("c5w", "c5f"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"gpurun_out/r02o/{tag}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            agg[k] += float(row["Counter_Value"]) * 1024; n[k] += 1
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(tag, k, n[k], round(v / 1e9, 2), "GB")
PY
echo "== done"
