# Evidence the DESIGN cites: hot receiver steps, the 2-rank host-transport
# bench rehearsal beside one rank at the same per-rank size, the scatter
# microbenchmark. Every GPU step has its own limit; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ev}
mkdir -p gpurun_out build
timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_receiver_$TAG.jsonl 2> gpurun_out/hot_receiver_$TAG.err || exit $?
cat gpurun_out/hot_receiver_$TAG.jsonl
timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 10 --warmup 2 --actors 262144 \
  > gpurun_out/bench_1rank_262144_$TAG.json 2> gpurun_out/bench_1rank_$TAG.err || exit $?
cat gpurun_out/bench_1rank_262144_$TAG.json
bash scripts/gpu_bench_mr.sh || exit $?
cp gpurun_out/bench_mr2.json gpurun_out/bench_mr2_$TAG.json
timeout -k 10 120 ./build/ubench_scatter > gpurun_out/ubench_scatter_$TAG.txt 2>&1 || exit $?
cat gpurun_out/ubench_scatter_$TAG.txt
