# GPU: 2-rank parity over the host transport (2 processes share the GPU), then
# one attempt at the RCCL exchange with 2 ranks on the same GPU (informational).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/test_multirank.py tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_mr.log 2>&1
rc=$?
echo "pytest multirank rc=$rc"; tail -30 gpurun_out/pytest_mr.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 tests/mr_worker.py ubench --rccl > gpurun_out/mr_rccl.log 2>&1
echo "rccl same-gpu rc=$?"; tail -15 gpurun_out/mr_rccl.log
exit 0
