# Same-box A/B of engine builds (PONYC_AMD_LIB) on the C2 bench, after a
# parity selection run against each variant. Every GPU step has its own time
# limit; the first failure ends the call.
#   TAG=r04c LIBS="base:ponyc_amd/libgpuactor.so perm:ponyc_amd/variants/lib_perm.so" \
#     TESTS_K="ubench and not det" REPS=3 bash scripts/gpu_ab_lib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
REPS=${REPS:-3}
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-ring --steps 40 --warmup 5"}
mkdir -p gpurun_out
for nv in $LIBS; do
  n=${nv%%:*}; lib=$PWD/${nv#*:}
  if [ -n "$TESTS_K" ]; then
    PONYC_AMD_LIB=$lib timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 \
      --timeout-method thread -k "$TESTS_K" > gpurun_out/pytest_${TAG}_$n.log 2>&1
    rc=$?
    echo "pytest $n rc=$rc"; tail -2 gpurun_out/pytest_${TAG}_$n.log
    [ $rc -eq 0 ] || exit $rc
  fi
done
for r in $(seq 1 $REPS); do
  for nv in $LIBS; do
    n=${nv%%:*}; lib=$PWD/${nv#*:}
    PONYC_AMD_LIB=$lib timeout -k 10 120 python bench.py $BENCH_ARGS \
      > gpurun_out/ab_${TAG}_${n}_$r.json 2> gpurun_out/ab_${TAG}_${n}_$r.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${n}_$r.json')); print('c2 $n', $r, round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
if [ -n "$GENERAL" ]; then
  for nv in $LIBS; do
    n=${nv%%:*}; lib=$PWD/${nv#*:}
    PONYC_AMD_LIB=$lib timeout -k 10 180 python scripts/profile_general.py $GENERAL \
      > gpurun_out/general_${TAG}_$n.jsonl 2>&1 || exit $?
    echo "general $n"; cat gpurun_out/general_${TAG}_$n.jsonl
  done
fi
