# Quick GPU iteration: parity tests, short bench, phase stamps. Each GPU step
# has its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
if [ -f ponyc_amd/libgpuactor_stamps.so ]; then
  timeout -k 10 120 python scripts/phase_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 || exit $?
  cat gpurun_out/stamps_$TAG.txt
fi
