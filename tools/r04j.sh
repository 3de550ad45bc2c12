# round-4 session: gzip segmented decode A/B (lab + C3), full GPU tests, C5 literal-window A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
export LD_LIBRARY_PATH=$PWD/tools/synth:$LD_LIBRARY_PATH
if [ -z "$SKIP_LAB" ]; then
for b in i1 i2 i2l8 i2l8w3; do  # k_zstd_lits: one vs two Huffman chains per lane (lab, 64 x 16 MiB C5 chunks)
  timeout -k 10 120 ./labx/zstd_lab_$b 64 16 3 c5 > $O/zstd_lab_$b.txt 2>&1; rc=$?
  echo "zstd_lab_$b rc=$rc $(grep -E '^ *lits|bad=' $O/zstd_lab_$b.txt | tr '\n' ' ')"
  [ $rc -gt 1 ] && exit 1
done
for v in seg lookahead; do
  ev=1; [ $v = lookahead ] && ev=0
  ZGPU_GZIP_SEG=$ev timeout -k 10 200 ./labx/gzip_lab 15625 > $O/gzip_lab_$v.txt 2>&1; rc=$?; tail -1 $O/gzip_lab_$v.txt; [ $rc -ne 0 ] && { echo "gzip_lab $v rc=$rc"; tail -5 $O/gzip_lab_$v.txt; exit 1; }
done
ZGPU_GZIP_SEG=1 timeout -k 10 200 ./labx/gzip_lab_prof 15625 > $O/gzip_lab_prof_seg.txt 2>&1 || { echo prof failed; tail -5 $O/gzip_lab_prof_seg.txt; exit 1; }
cat $O/gzip_lab_prof_seg.txt
fi
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit $rc; }
for v in seg lookahead; do
  ev=1; [ $v = lookahead ] && ev=0
  ZGPU_GZIP_SEG=$ev timeout -k 10 600 python -u bench.py --workload c3 --no-pmc --no-cpu --secondary= --steps 5 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); e=d['host_leg']['dropin_emulation']; print('$v', d['value'], d['ms_per_step'], d['roundtrip_ok'], 'dropin', e['GiBps'], e['threads_one_per_shard']['GiBps'])"
done
for v in seg lookahead; do
  ev=1; [ $v = lookahead ] && ev=0
  ZGPU_GZIP_SEG=$ev timeout -k 10 600 python -u bench.py --workload blosc-zlib --no-pmc --no-cpu --no-host-leg --secondary= --steps 5 > $O/bz_$v.json 2> $O/bz_$v.err || { tail -5 $O/bz_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bz_$v.json')); print('blosc-zlib $v', d['value'], d['ms_per_step'], d['roundtrip_ok'])"
done
for v in base gwin3 ilp2 ilp2l8; do
  lib=""; [ $v != base ] && lib=zarrs_amd/lib_variants/$v/libzgpu.so
  ZGPU_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --c5-scale 2 --no-cpu --no-pmc --no-host-leg --secondary= --steps 5 --warmup 2 > $O/c5_$v.json 2> $O/c5_$v.err || { echo "$v failed"; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('c5 $v', d['value'], d['ms_per_step'], d['roundtrip_ok'])"
done
echo done
