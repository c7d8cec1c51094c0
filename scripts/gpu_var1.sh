set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_variants.sh || exit $?
PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib_z12b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_z12b.log 2>&1; echo "z12b parity rc=$?"; tail -3 gpurun_out/pytest_z12b.log
