#!/bin/bash
# round-5 zstd lab session: sequence decoder A/B on C5-like chunks (tools/labbin/zlab*, built on the CPU side)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-zlab}; shift; mkdir -p $O
for spec in "$@"; do
  b=${spec%%:*}; lg=${spec#*:}
  echo "== $b LAB_SEQLG=$lg"
  LAB_SEQLG=$lg timeout -k 5 300 tools/labbin/$b ${LAB_N:-64} 16 3 c5 || exit 1
done 2>&1 | tee $O/zlab.txt
