# A/B: bench every built variant, then the GPU parity suite on variant $VAR.
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=${VAR:-planned}
bash scripts/gpu_variants.sh || exit $?
PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib_$VAR.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$VAR.log 2>&1
echo "$VAR parity rc=$?"; tail -3 gpurun_out/pytest_$VAR.log
