set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_backpressure.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_hot.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_hot.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_receiver_k8.jsonl 2>&1 || exit $?
cat gpurun_out/hot_receiver_k8.jsonl
