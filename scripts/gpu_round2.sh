# Round-2 GPU call: every GPU test, smoke, the full bench (CPU baselines and
# ring included), rocprofv3 kernel stats of the bench, PMC passes of the same
# library. Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || exit $?
cat gpurun_out/bench_full_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python3 bench.py --no-cpu-baseline --no-ring > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
cat gpurun_out/prof_bench_$TAG.json
TAG=$TAG bash scripts/gpu_pmc.sh || exit $?
