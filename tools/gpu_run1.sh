set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "not gzip and not zstd" > gpurun_out/pytest1.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest1.log
tail -5 gpurun_out/pytest1.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke1.log 2>&1 && cat gpurun_out/smoke1.log &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && cat gpurun_out/bench1.json
