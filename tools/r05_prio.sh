#!/bin/bash
# round 5: C5 stream-lane priorities and executor segments re-measured (the L1 lane is the critical path)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-prio}; mkdir -p $O
run() {  # label, NAME=VALUE env setting, extra bench flags...
  local label=$1 ev=$2; shift 2
  echo "== $label"
  env "$ev" timeout -k 10 300 python3 -u bench.py --workload c5 --no-pmc --no-host-leg --no-cpu --secondary= --steps 10 --warmup 2 "$@" \
    > $O/$label.json 2> $O/$label.err || { tail -5 $O/$label.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$label.json')); print(d['ms_per_step'], d['value'])"
}
if [ "$2" = bz ]; then  # blosc-zstd: executor segments 4 vs 3 (vs 2 with "bz3")
  for r in a b; do for x in 4 3 ${3:-}; do
    echo "== bz xseg$x$r"
    ZGPU_ZSTD_XSEG=$x timeout -k 10 300 python3 -u bench.py --workload blosc-zstd --no-pmc --no-host-leg --no-cpu --secondary= \
      > $O/bz$x$r.json 2> $O/bz$x$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bz$x$r.json')); print(d['ms_per_step'], d['value'])"
  done; done
  exit 0
fi
if [ "$2" = lf ]; then  # C5: parts whose plans decode literals before sequences (0,1 L0 halves, 2 L1, 3-5 L2-L4)
  for r in a b; do for x in ${3:-none 2 2,3,4,5 3,4,5 0,1}; do
    v=$x; [ $x = none ] && v=
    run lf$x$r ZGPU_NONE=1 --lits-first=$v || exit 1
  done; done
  exit 0
fi
if [ "$2" = xseg ]; then  # second pass: executor segments 1-4, twice each (or the list in $3)
  for r in a b; do for x in ${3:-4 2 3 1}; do run xseg$x$r ZGPU_ZSTD_XSEG=$x || exit 1; done; done
  exit 0
fi
for pr in -1,-1,0,0 -1,-1,-1,0 0,0,-1,0 0,0,-1,-1 -1,-1,-1,-1; do
  run p$pr ZGPU_NONE=1 --lane-priorities=$pr || exit 1
done
run xseg8 ZGPU_ZSTD_XSEG=8 || exit 1
run xseg2 ZGPU_ZSTD_XSEG=2 || exit 1
