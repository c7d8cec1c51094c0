# C1 one-ring (one zone): k_step_run vs per-step launches, reference on the host cores.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-c1one}
mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_configs.py --cpu c1_ring_one > gpurun_out/c1one_run_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/c1one_run_$TAG.jsonl
GPA_NO_RUN_KERNEL=1 timeout -k 10 120 python scripts/bench_configs.py c1_ring_one > gpurun_out/c1one_steps_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/c1one_steps_$TAG.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1one_$TAG -o run -- \
  python3 scripts/bench_configs.py c1_ring_one > gpurun_out/c1one_prof_$TAG.jsonl 2>&1 || exit $?
cut -c1-160 gpurun_out/prof_c1one_$TAG/run_kernel_stats.csv
