set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/gzpmc1 -o p --output-format csv -- ./tools/lab/gzip_lab 4096 1 > gpurun_out/gzpmc1.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_FLAT -d gpurun_out/gzpmc2 -o p --output-format csv -- ./tools/lab/gzip_lab 4096 1 > gpurun_out/gzpmc2.txt 2>&1
echo rc=$?
tail -3 gpurun_out/gzpmc1.txt gpurun_out/gzpmc2.txt
