set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_mem 1048576 64 | tee gpurun_out/ubench_mem_1M_64.txt || exit $?
timeout -k 10 120 ./scripts/ubench_mem 1048576 8 | tee gpurun_out/ubench_mem_1M_8.txt || exit $?
