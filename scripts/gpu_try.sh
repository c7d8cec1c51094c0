# Quick GPU check of the current build: GPU tests (stop at the first failure),
# then a short C2 bench. A crash, abort or time limit ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-try}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -3; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 30 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
brc=$?
cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
exit $rc
