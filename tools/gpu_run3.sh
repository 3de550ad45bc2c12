set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -k "not zstd" -x > gpurun_out/pytest3.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest3.log
tail -30 gpurun_out/pytest3.log
