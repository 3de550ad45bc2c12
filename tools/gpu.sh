#!/bin/bash
# One parameterised GPU-box session, run from this container through gpurun:
#   gpurun --timeout T -- bash tools/gpu.sh <tag> <step> [<step> ...]
# Steps run in order, each under its own time limit; the session stops at the first failure.
#   test[:EXPR[:ENV]]    pytest -m gpu (-k EXPR when given; ENV: NAME=VALUE settings, comma-separated)
#   smoke                __graft_entry__.smoke()
#   bench:W[:FLAGS[:ENV]] bench.py --workload W, the full line (CPU baseline, PMC passes, host leg);
#                        FLAGS: extra bench flags, comma-separated (e.g. bench:c5:--c5-scale,2); ENV:
#                        NAME=VALUE settings, comma-separated
#   quick:W[:FLAGS]      bench.py --workload W without PMC passes / host leg, short CPU baseline
#   prof:W[:FLAGS]       rocprofv3 --kernel-trace --stats of bench.py --workload W (5 steps)
#   serial:W[:FLAGS]     the same with every plan on one stream (--serial-lanes: per-kernel split)
#   pmc:W:CTR[:FLAGS]    one rocprofv3 --pmc pass (a single counter) of bench.py --workload W
#   torchrun:N[:FLAGS]   bench.py --gpus N through torch.distributed.run (N processes)
#   lab:BIN:ARGS[:ENV]   tools/labbin/BIN with ARGS (comma-separated) and ENV (NAME=VALUE, comma-separated)
#   py:SCRIPT[:ARGS]     python3 SCRIPT with ARGS (comma-separated), e.g. a tools/*.py measurement
# Everything lands in gpurun_out/<tag>/ (step-numbered files).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-run}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
i=0
for step in "$@"; do
  i=$((i + 1))
  IFS=: read -r kind a b c <<< "$step"
  echo "== [$i] $step"
  case "$kind" in
    test)
      K=(); [ -n "$a" ] && K=(-k "$a"); E=(${b//,/ })
      env "${E[@]}" timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread "${K[@]}" \
        > "$O/$i.pytest.log" 2>&1; rc=$?
      tail -3 "$O/$i.pytest.log"
      [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 "$O/$i.pytest.log"; exit $rc; } ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/$i.smoke.log" 2>&1 \
        || { rc=$?; echo "smoke rc=$rc"; tail -20 "$O/$i.smoke.log"; exit $rc; }
      tail -1 "$O/$i.smoke.log" ;;
    bench|quick)
      F=(${b//,/ }); E=(${c//,/ }); [ "$kind" = quick ] && F+=(--no-pmc --no-host-leg --cpu-seconds 5 --secondary=)
      env "${E[@]}" timeout -k 10 900 python -u bench.py --workload "$a" "${F[@]}" > "$O/$i.bench_$a.json" 2> "$O/$i.bench_$a.err" \
        || { rc=$?; echo "bench rc=$rc"; tail -20 "$O/$i.bench_$a.err"; exit $rc; }
      cat "$O/$i.bench_$a.json" ;;
    prof|serial)
      F=(${b//,/ }); [ "$kind" = serial ] && F+=(--serial-lanes)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$i.prof_$a" -o run --output-format csv -- \
        python3 bench.py --workload "$a" --no-cpu --no-pmc --no-host-leg --secondary= --steps 5 --warmup 1 "${F[@]}" \
        > "$O/$i.prof_$a.json" 2> "$O/$i.prof_$a.err" || { rc=$?; echo "rocprof rc=$rc"; tail -20 "$O/$i.prof_$a.err"; exit $rc; }
      cat "$O/$i.prof_$a.json"
      f=$(ls "$O/$i.prof_$a"/run_kernel_stats.csv "$O/$i.prof_$a"/*/run_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && head -12 "$f" | cut -c1-200 ;;
    pmc)
      F=(${c//,/ })
      timeout -s KILL 300 rocprofv3 --pmc "$b" -d "$O/$i.pmc_${a}_$b" -o pmc --output-format csv -- \
        python3 bench.py --workload "$a" --child --no-cpu --no-pmc --no-host-leg --steps 2 --warmup 1 "${F[@]}" \
        > /dev/null 2> "$O/$i.pmc_${a}_$b.err" || { rc=$?; echo "pmc rc=$rc"; tail -20 "$O/$i.pmc_${a}_$b.err"; exit $rc; } ;;
    torchrun)
      F=(${b//,/ })
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$a" --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus "$a" --no-pmc --no-host-leg "${F[@]}" > "$O/$i.torchrun.json" \
        2> "$O/$i.torchrun.err" || { rc=$?; echo "torchrun rc=$rc"; tail -20 "$O/$i.torchrun.err"; exit $rc; }
      tail -1 "$O/$i.torchrun.json" ;;
    lab)
      A=(${b//,/ }); E=(${c//,/ })
      env "${E[@]}" timeout -k 10 300 "tools/labbin/$a" "${A[@]}" > "$O/$i.lab_$a.txt" 2>&1 \
        || { rc=$?; echo "lab rc=$rc"; tail -20 "$O/$i.lab_$a.txt"; exit $rc; }
      cat "$O/$i.lab_$a.txt" ;;
    py)
      A=(${b//,/ })
      timeout -k 10 600 python3 -u "$a" "${A[@]}" > "$O/$i.py.txt" 2>&1 \
        || { rc=$?; echo "py rc=$rc"; tail -30 "$O/$i.py.txt"; exit $rc; }
      tail -40 "$O/$i.py.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
