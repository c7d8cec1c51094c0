# rocprofv3 kernel trace of a short bench run (no CPU legs) and the launch
# timeline of its k_step dispatches (scripts/kernel_gaps.py). TAG names it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-trace}
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python3 bench.py --no-cpu-baseline --no-ring --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/trace_bench_$TAG.json 2> gpurun_out/trace_$TAG.err || exit $?
python3 scripts/kernel_gaps.py gpurun_out/prof/$TAG | tee gpurun_out/gaps_$TAG.txt
