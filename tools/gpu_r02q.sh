#!/bin/bash
# r02 session Q: zstd literal-store packing / global-read window A/B (C5, blosc-zstd), zstd tests on
# the default build, then the C5 per-kernel traffic of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
echo "== pytest zstd"
timeout -k 10 600 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_c3c5.py tests/test_gpu_blosc.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in p8 p16 p8l32 p16l32 p8 p16l32; do
  for w in c5 blosc-zstd; do
    echo "== $v $w"
    ZGPU_LIB=zarrs_amd/lib_variants/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/${w}_$v.json 2> $O/${w}_$v.err || { echo "rc=$?"; tail -3 $O/${w}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_$v.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== C5 per-kernel WRITE_SIZE / FETCH_SIZE (one step, default build)"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_zstd|k_scatter" -d $O/c5w -o pmc --output-format csv -- python3 bench.py --child --workload c5 --steps 1 --warmup 0 --no-cpu > $O/c5w.log 2>&1
echo "rc=$?"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_zstd|k_scatter" -d $O/c5f -o pmc --output-format csv -- python3 bench.py --child --workload c5 --steps 1 --warmup 0 --no-cpu > $O/c5f.log 2>&1
echo "rc=$?"
python3 - <<'PY'
import csv, glob, collections
for tag in ("c5w", "c5f"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"gpurun_out/r02q/{tag}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            agg[k] += float(row["Counter_Value"]) * 1024; n[k] += 1
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:6]:
        print(tag, k, n[k], round(v / 1e9, 2), "GB")
PY
echo "== done"
