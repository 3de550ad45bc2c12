#!/bin/bash
# round 5: lone-shard latency (tools/dropin_latency.py) and the coalescer trace of the default drop-in policy
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-dropin7}; mkdir -p $O
timeout -k 10 240 python -u tools/dropin_latency.py 2> $O/lat.err | tee $O/latency.txt || exit 1
ZGPU_TRACE=1 timeout -k 10 240 python -u tools/dropin_sweep.py 8 200 2> $O/trace.txt | tail -1 || exit 1
python3 tools/co_trace.py $O/trace.txt | tail -14
