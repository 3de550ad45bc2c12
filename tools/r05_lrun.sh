#!/bin/bash
# round 5: literal runs packed into the gzip seg path's symbol records (ZG_INFLATE_LRUN 0/1), gzip lab A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-lrun}; mkdir -p $O
for v in lr0 lr1; do
  for n in 15625 512 1; do
    for pm in 0 2048; do
      echo "== $v n=$n ZGPU_GZIP_PIPE_MAX=$pm"
      ZGPU_GZIP_PIPE_MAX=$pm timeout -k 5 120 tools/labbin/gzip_lab_$v $n 1 | grep -E "k_gzip|bad" || exit 1
    done
  done
  echo "== ${v}p n=15625 (profile build)"
  ZGPU_GZIP_PIPE_MAX=0 timeout -k 5 120 tools/labbin/gzip_lab_${v}p 15625 1 || exit 1
done 2>&1 | tee $O/lrun.txt
