# Round evidence for the shipped build, in two calls (each GPU step has its
# own limit; the first failure ends the call):
#   PART=A: -m gpu suite, smoke, the full bench (CPU baselines, ring; skipped
#           with SKIP_FULL_BENCH=1), rocprofv3 kernel stats of the bench, and
#           the k_step PMC traffic passes (one rocprofv3 run per pass);
#   PART=B: PMC passes and kernel stats of the general path (C2-det, C5
#           storm), the hot-receiver burst / backlog steps, and (CONFIGS=1)
#           every BASELINE config beside the reference runtime.
# PART unset runs both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04}
mkdir -p gpurun_out/prof
if [ -z "$PART" ] || [ "$PART" = A ]; then
  if [ -z "$SKIP_PYTEST" ]; then      # (SKIP_PYTEST=1: the caller ran the suite)
    timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1
    rc=$?
    echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
    [ $rc -eq 0 ] || exit $rc
  fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
  tail -3 gpurun_out/smoke_$TAG.log
  if [ -z "$SKIP_FULL_BENCH" ]; then
    timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || exit $?
    cat gpurun_out/bench_full_$TAG.json
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --no-ring > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
  find gpurun_out/prof/$TAG -name '*kernel_stats*'
  OUT=gpurun_out/pmc_$TAG
  mkdir -p $OUT
  sha256sum ponyc_amd/libgpuactor.so | cut -c1-16 > $OUT/lib_sha16.txt
  i=0
  for sel in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_REQ_sum"; do
    i=$((i+1))
    echo "pass $i: $sel"
    timeout -s KILL 90 rocprofv3 --pmc $sel --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --no-ring --steps 6 --warmup 2 > $OUT/bench_p$i.json 2> $OUT/err_p$i.txt || exit $?
  done
fi
if [ -z "$PART" ] || [ "$PART" = B ]; then
  for w in det storm; do
    OUT=gpurun_out/pmc_${TAG}_$w
    mkdir -p $OUT
    sha256sum ponyc_amd/libgpuactor.so | cut -c1-16 > $OUT/lib_sha16.txt
    i=0
    for sel in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
               "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
               "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
      i=$((i+1))
      echo "$w pass $i: $sel"
      timeout -s KILL 120 rocprofv3 --pmc $sel --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
        python3 scripts/profile_general.py $w > $OUT/out_p$i.txt 2> $OUT/err_p$i.txt || exit $?
    done
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/general_$TAG -o run -- \
    python3 scripts/profile_general.py > gpurun_out/general_prof_$TAG.jsonl 2> gpurun_out/general_prof_$TAG.err || exit $?
  cat gpurun_out/general_prof_$TAG.jsonl
  for r in 1 2; do
    timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}_$r.jsonl 2>&1 || exit $?
    cat gpurun_out/hot_${TAG}_$r.jsonl
  done
  if [ -n "$CONFIGS" ]; then
    timeout -k 10 600 python scripts/bench_configs.py --cpu > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit $?
    cat gpurun_out/configs_$TAG.jsonl
  fi
fi
