#!/bin/bash
# round-5 lab session: gzip lab A/B (throughput grid, a lone shard's 512 streams, one stream)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-lab}; mkdir -p $O
for b in base new; do
  for n in 15625 512 1; do
    echo "== $b n=$n"; timeout -k 5 120 tools/labbin/gzip_lab_$b $n 1 || exit 1
  done
  echo "== ${b}_prof n=15625"; timeout -k 5 120 tools/labbin/gzip_lab_${b}_prof 15625 1 || exit 1
  echo "== ${b}_prof n=512"; timeout -k 5 120 tools/labbin/gzip_lab_${b}_prof 512 1 || exit 1
done 2>&1 | tee $O/gzip_lab.txt
