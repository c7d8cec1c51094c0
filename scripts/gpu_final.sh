# Round-end evidence for the shipped build: the round script (GPU tests,
# smoke, full bench, rocprofv3 stats, PMC passes), then every config beside
# the reference runtime.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-final} bash scripts/gpu_round2.sh || exit $?
timeout -k 10 600 python scripts/bench_configs.py --cpu > gpurun_out/configs_${TAG:-final}.jsonl 2> gpurun_out/configs_${TAG:-final}.err || exit $?
cat gpurun_out/configs_${TAG:-final}.jsonl
