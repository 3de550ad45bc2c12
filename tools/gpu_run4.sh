set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -k "zstd" > gpurun_out/pytest4.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest4.log
tail -40 gpurun_out/pytest4.log
