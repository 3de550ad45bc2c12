#!/bin/bash
# r02 session 2, call C: gzip lab A/B (wide lookahead + subtables vs HEAD), then the HEAD library's
# state check (GPU tests, smoke, bench lines).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r02s2b.sh || exit 1
bash tools/gpu_r02s2a.sh
