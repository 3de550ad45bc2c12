set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex exec_item -d gpurun_out/zpmc1 -o p --output-format csv -- ./tools/lab/zstd_lab 8 16 3 c5 > gpurun_out/zpmc1.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex exec_item -d gpurun_out/zpmc2 -o p --output-format csv -- ./tools/lab/zstd_lab 8 16 3 c5 > gpurun_out/zpmc2.txt 2>&1
echo rc=$?
tail -3 gpurun_out/zpmc1.txt gpurun_out/zpmc2.txt
