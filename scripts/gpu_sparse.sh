# Sparse-step changes: GPU parity tests, C1 configs, short headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-sp}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/bench_configs.py c1_ring c1_ring_one c3_fanin c4_gups > gpurun_out/configs_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/configs_$TAG.jsonl
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
