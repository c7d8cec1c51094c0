# Rehearse the N>1 bench path on the one-GPU box: 2 ranks on device 0. RCCL
# refuses two ranks on one GPU, so bench.py falls back to the host transport;
# this exercises the launch, barriers, max-over-ranks timing and counter sums.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PONYC_AMD_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 2 \
  --actors 262144 > gpurun_out/bench_mr2.json 2> gpurun_out/bench_mr2.err
rc=$?; cat gpurun_out/bench_mr2.json; grep -v alt_rsmi gpurun_out/bench_mr2.err | tail -5; exit $rc
