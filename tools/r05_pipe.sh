#!/bin/bash
# round 5: pipelined k_gzip (two waves per stream) vs one wave, gzip lab (15625 / 2048 / 512 / 1 streams)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pipe}; mkdir -p $O
for pm in 0 2048; do
  for n in 15625 2048 512 1; do
    echo "== ZGPU_GZIP_PIPE_MAX=$pm n=$n"
    ZGPU_GZIP_PIPE_MAX=$pm timeout -k 5 120 tools/labbin/gzip_lab_pipe $n 1 | grep -E "k_gzip|bad" || exit 1
  done
done 2>&1 | tee $O/pipe.txt
