# Planned sends (round 3): the -m gpu suite on the shipped build, then the C2
# bench of the pinger-only builds with and without planned sends, alternating,
# then the k_step traffic passes of the shipped build. Every GPU step has its
# own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03c}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2 3; do
  for v in ${VARIANTS:-_p512 _p512np}; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 40 --warmup 5 \
      > gpurun_out/ab_${TAG}${v}_$r.json 2> gpurun_out/ab_${TAG}${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}${v}_$r.json')); print('$v', $r, round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_ms'], d['atomics'])"
  done
done
if [ -n "$PMC" ]; then
  OUT=gpurun_out/pmc_$TAG
  mkdir -p $OUT
  sha256sum ponyc_amd/libgpuactor.so | cut -c1-16 > $OUT/lib_sha16.txt
  i=0
  for sel in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    echo "pass $i: $sel"
    timeout -s KILL 90 rocprofv3 --pmc $sel --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --no-ring --steps 6 --warmup 2 > $OUT/bench_p$i.json 2> $OUT/err_p$i.txt || exit $?
  done
  find $OUT -name '*counter_collection.csv' | sort
fi
