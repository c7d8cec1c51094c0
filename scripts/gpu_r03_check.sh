# Round 3 check of the shipped build: the -m gpu suite, then the general-path
# and hot-receiver step times. Each GPU step has its own limit; the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03l}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/profile_general.py > gpurun_out/general_$TAG.jsonl 2> gpurun_out/general_$TAG.err || exit $?
cat gpurun_out/general_$TAG.jsonl
timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_$TAG.jsonl 2> gpurun_out/hot_$TAG.err || exit $?
cat gpurun_out/hot_$TAG.jsonl
