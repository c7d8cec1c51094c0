set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
NCCL_DEBUG=WARN timeout -k 10 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 tests/mr_worker.py ubench --rccl --same-gpu > gpurun_out/mr_rccl.log 2>&1
echo "rccl same-gpu rc=$?"; grep -E "MR_RESULT|Error|NCCL WARN|Duplicate" gpurun_out/mr_rccl.log | head -20
exit 0
