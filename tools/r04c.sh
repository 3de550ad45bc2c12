set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "general_chains or dropin" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --workload c3 --no-pmc --no-cpu --secondary= --steps 5 --dropin-sweep 1,2,4,8,16 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c -d $O/pmc_c5_$c -o pmc --output-format csv -- python3 bench.py --workload c5 --child --no-cpu --no-pmc --no-host-leg --steps 2 --warmup 1 --serial-lanes > /dev/null 2> $O/pmc_c5_$c.err || { echo "pmc $c failed"; tail -5 $O/pmc_c5_$c.err; exit 1; }
done
echo done
