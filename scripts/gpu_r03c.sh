# The general handler path measured like the headline: rocprofv3 kernel stats
# and PMC passes of C2-det (k_step<PINGER_DET>) and C5 (k_step<STORM>).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03c}
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/det_$TAG -o run -- \
  python3 scripts/bench_configs.py c2_ubench_det c5_storm_8m > gpurun_out/configs_det_$TAG.jsonl 2> gpurun_out/configs_det_$TAG.err || exit $?
cat gpurun_out/configs_det_$TAG.jsonl
find gpurun_out/prof/det_$TAG -name '*stats*'
TAG=det_$TAG PMC_CMD="scripts/bench_configs.py c2_ubench_det" bash scripts/gpu_pmc_cmd.sh || exit $?
TAG=storm_$TAG PMC_CMD="scripts/bench_configs.py c5_storm_8m" bash scripts/gpu_pmc_cmd.sh || exit $?
