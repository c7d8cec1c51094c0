# Full bench (with CPU baseline) + rocprofv3 kernel-trace stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
timeout -k 10 600 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || exit $?
cat gpurun_out/bench_full_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$TAG -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit $?
find gpurun_out/prof/$TAG -name '*stats*' | head
