#!/bin/bash
# Round-2 records on the current build: full GPU tests + smoke, every workload's bench line (CPU
# baseline + PMC traffic) and rocprofv3 kernel stats, and the torchrun launcher path at N=1.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r02final.sh <tag> [workloads...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02final}; shift
WL=${@:-c2 c3 c5 blosc blosc-zstd c1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in $WL; do
  timeout -k 10 600 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w rc=$?"; tail -5 $O/bench_$w.err; exit 1; }
  echo "$w $(python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print(d['value'], d['unit'], d['ms_per_step'], 'frac', r['frac'], 'traffic', r['traffic'], 'cpu', d['cpu_baseline']['value'])")"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --no-cpu --no-pmc --no-host-leg --steps 5 --warmup 1 > $O/prof_$w.json 2> $O/prof_$w.err || { echo "rocprof $w rc=$?"; exit 1; }
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu --no-pmc --no-host-leg > $O/torchrun_n1.json 2> $O/torchrun_n1.err || { echo "torchrun rc=$?"; tail -5 $O/torchrun_n1.err; exit 1; }
tail -1 $O/torchrun_n1.json
echo "== done"
