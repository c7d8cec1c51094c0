# Quick GPU check + primitive microbenchmarks (atomic peak for SURVEY §8 d1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-q2}
mkdir -p gpurun_out
bash scripts/gpu_quick.sh || exit $?
timeout -k 10 120 ./scripts/ubench_mem > gpurun_out/ubench_mem_$TAG.txt 2>&1 || exit $?
cat gpurun_out/ubench_mem_$TAG.txt
