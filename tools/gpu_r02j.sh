#!/bin/bash
# r02 session J: full GPU suite on the rebuilt library (gzip pointer-jumping chain + word copies,
# zstd Huffman-table kernel + 4-wave literal decoder), then C3 / C5 / blosc-zstd bench lines and the
# C5 serialised-lanes kernel split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for w in c3 c5 blosc-zstd; do
  echo "== bench $w"
  timeout -k 10 500 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "rc=$?"; tail -3 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['roundtrip_ok'], r['avg_launch_ms_hip_events'])"
done
echo "== rocprof c5 serial lanes"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5s -o run --output-format csv -- python3 bench.py --workload c5 --serial-lanes --no-pmc --no-host-leg --no-cpu --steps 5 --warmup 1 > $O/prof_c5s.json 2> $O/prof_c5s.err || { echo "rocprof c5 rc=$?"; tail -5 $O/prof_c5s.err; exit 1; }
V=zarrs_amd/lib_variants
for v in base x8 x8s256; do
  for w in c5 blosc-zstd; do
    echo "== A/B $v $w"
    ZGPU_LIB=$V/$v/libzgpu.so timeout -k 10 400 python bench.py --workload $w --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/ab_${v}_$w.json 2> $O/ab_${v}_$w.err || { echo "rc=$?"; tail -3 $O/ab_${v}_$w.err; exit 1; }
    python -c "import json; d=json.load(open('$O/ab_${v}_$w.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
  done
done
echo "== done"
