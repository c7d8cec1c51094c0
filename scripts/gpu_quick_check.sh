# Quick check of a build: the hot-path tests (FIFO, backlogs, mute, hot
# groups), the hot receivers, and the general-path step times. Each GPU step
# has its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-quick}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "${TESTS_K:-fifo or backlog or mute or hot or ubench_det or storm}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}.jsonl 2>&1 || exit $?
cat gpurun_out/hot_${TAG}.jsonl
for r in 1 2; do
  timeout -k 10 240 python scripts/profile_general.py det storm pinger > gpurun_out/gen_${TAG}_$r.jsonl 2>&1 || exit $?
  cat gpurun_out/gen_${TAG}_$r.jsonl
done
if [ -n "$STAMPS" ]; then
  timeout -k 10 180 python scripts/hot_stamps.py > gpurun_out/hot_stamps_$TAG.txt 2>&1 || exit $?
  cat gpurun_out/hot_stamps_$TAG.txt
fi
