# GPU tests of the in-tree build (= C), then a same-box A/B of builds A and C on the C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_abc2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_abc2.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="A C" bash scripts/gpu_ab.sh
