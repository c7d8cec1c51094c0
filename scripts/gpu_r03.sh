# Round 3 GPU check: the -m gpu suite, smoke, the N-rank bench rehearsal and
# its failure mode on one GPU, then the N=1 bench. Each GPU step has its own
# limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
cat gpurun_out/smoke_$TAG.log
PONYC_AMD_SAME_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --actors 262144 \
  > gpurun_out/bench_mr2_$TAG.json 2> gpurun_out/bench_mr2_$TAG.err || exit $?
cat gpurun_out/bench_mr2_$TAG.json
timeout -k 10 120 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_gpus2_fail_$TAG.json 2>&1
echo "bench --gpus 2 on one GPU without the flag: rc=$? (non-zero expected)"
tail -2 gpurun_out/bench_gpus2_fail_$TAG.json
timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || exit $?
cat gpurun_out/bench_full_$TAG.json
