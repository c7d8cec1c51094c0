# Same-box A/B of one environment switch on the C2 bench (and optionally the
# general-path workloads), after an optional pytest selection. Every GPU step
# has its own time limit; the first failure ends the call.
#   TAG=r04b AB_VAR=PONYC_AMD_TWO_PASS AB_VALS="0 1" TESTS_K="ubench" REPS=3 \
#     bash scripts/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
REPS=${REPS:-3}
mkdir -p gpurun_out
if [ -n "$TESTS_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$TESTS_K" \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $REPS); do
  for v in $AB_VALS; do
    env $AB_VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 40 --warmup 5 \
      > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${v}_$r.json')); print('c2 $AB_VAR=$v', $r, round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
if [ -n "$GENERAL" ]; then
  for v in $AB_VALS; do
    env $AB_VAR=$v timeout -k 10 180 python scripts/profile_general.py $GENERAL > gpurun_out/general_${TAG}_$v.jsonl 2>&1 || exit $?
    echo "general $AB_VAR=$v"; cat gpurun_out/general_${TAG}_$v.jsonl
  done
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --no-ring > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
  find gpurun_out/prof/$TAG -name '*kernel_stats*' -exec head -5 {} \;
fi
