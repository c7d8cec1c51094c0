# One iteration on the GPU box for a candidate build: the -m gpu suite (the
# library's sha is in the log header), a short bench line, the two-pass
# phase stamps (libgpuactor_stamps.so), the general path's step times and
# selected BASELINE configs. Every GPU step has its own limit; the first
# failure ends the call. TAG names the outputs; SKIP_PYTEST=1, CONFIGS="..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-iter}
mkdir -p gpurun_out
if [ -z "$SKIP_PYTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; sed -n 3,4p gpurun_out/pytest_$TAG.log; tail -2 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ring > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
timeout -k 10 180 python scripts/plan_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 || exit $?
cat gpurun_out/stamps_$TAG.txt
timeout -k 10 240 python scripts/profile_general.py det storm pinger > gpurun_out/gen_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/gen_$TAG.jsonl
if [ -n "$CONFIGS" ]; then
  timeout -k 10 600 python scripts/bench_configs.py $CONFIGS > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit $?
  cat gpurun_out/configs_$TAG.jsonl
fi
