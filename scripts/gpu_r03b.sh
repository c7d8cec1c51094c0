# Microbenchmark of planned-chunk staging, phase stamps of C2 and C2-det, then
# the round-3 GPU check (tests, smoke, N-rank rehearsal, bench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03b}
mkdir -p gpurun_out
timeout -k 10 120 ./build/ubench_plan > gpurun_out/ubench_plan_$TAG.txt 2>&1 || exit $?
cat gpurun_out/ubench_plan_$TAG.txt
timeout -k 10 120 python scripts/phase_stamps.py > gpurun_out/stamps_c2_$TAG.txt 2>&1 || exit $?
cat gpurun_out/stamps_c2_$TAG.txt
TAG=$TAG bash scripts/gpu_r03.sh
