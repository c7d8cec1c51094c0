# Hot-group MSD sort: the tests with hot groups (FIFO fan-in, backlogs, both
# geometries, two ranks), the 100K -> 4 FIFO burst / backlog steps, the burst
# zone's phase stamps, and the general path for regressions. Each GPU step
# has its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04j}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "fifo or backlog or mute or hot or fanin or priority" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}_$r.jsonl 2>&1 || exit $?
  cat gpurun_out/hot_${TAG}_$r.jsonl
done
timeout -k 10 180 python scripts/hot_stamps.py > gpurun_out/hot_stamps_$TAG.txt 2>&1 || exit $?
cat gpurun_out/hot_stamps_$TAG.txt
timeout -k 10 240 python scripts/profile_general.py det storm pinger > gpurun_out/gen_$TAG.jsonl 2>&1 || exit $?
cat gpurun_out/gen_$TAG.jsonl
for v in 0 1; do
  PONYC_AMD_DEFER_BIG=$v timeout -k 10 240 python scripts/profile_general.py det storm > gpurun_out/gen_${TAG}_defer$v.jsonl 2>&1 || exit $?
  echo "defer_big=$v"; cat gpurun_out/gen_${TAG}_defer$v.jsonl
done
