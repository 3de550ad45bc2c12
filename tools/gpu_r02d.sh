#!/bin/bash
# r02 session D: sharding-encode parity + C1 bench line, then A/B round 2 of the zstd LDS sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
echo "== pytest encode"
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
echo "== bench c1"
timeout -k 10 300 python bench.py --workload c1 --no-pmc --cpu-seconds 5 > $O/bench_c1.json 2> $O/bench_c1.err || { echo "rc=$?"; tail -3 $O/bench_c1.err; exit 1; }
cat $O/bench_c1.json
run() {  # name lib workload
  echo "== $1 $3"
  ZGPU_LIB=$2 timeout -k 10 400 python bench.py --workload $3 --no-pmc --no-host-leg --no-cpu --steps 10 --warmup 2 > $O/$1_$3.json 2> $O/$1_$3.err || { echo "rc=$?"; tail -3 $O/$1_$3.err; return 1; }
  python -c "import json; d=json.load(open('$O/$1_$3.json')); print(d['value'], d['ms_per_step'], d['roundtrip_ok'])"
}
V=zarrs_amd/lib_variants
for w in blosc-zstd c5; do
  for v in r16l16 r8l16 r8l8 r16l8 r16l16s256 r8l16s256; do
    run $v $V/$v/libzgpu.so $w || exit 1
  done
done
echo "== done"
