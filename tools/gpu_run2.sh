set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -k "not gzip and not zstd" > gpurun_out/pytest2.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest2.log
tail -15 gpurun_out/pytest2.log
mkdir -p gpurun_out/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench2.json 2> gpurun_out/bench2.err
echo "rocprof rc=$?"
cat gpurun_out/bench2.json
find gpurun_out/prof2 -name "*stats*" | head
