# Round-4 check of a candidate build: the full -m gpu suite, the hot
# receivers (burst / backlog steps and the burst zone's stamps), and the
# small-group selection bound (PONYC_AMD_SEL_BOUND=0/1) on det / storm /
# pinger, twice. Each GPU step has its own limit; the first failure ends the
# call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04m}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}_$r.jsonl 2>&1 || exit $?
  cat gpurun_out/hot_${TAG}_$r.jsonl
done
timeout -k 10 180 python scripts/hot_stamps.py > gpurun_out/hot_stamps_$TAG.txt 2>&1 || exit $?
cat gpurun_out/hot_stamps_$TAG.txt
for r in 1 2; do
  for v in 0 1; do
    PONYC_AMD_SEL_BOUND=$v timeout -k 10 240 python scripts/profile_general.py det storm pinger \
      > gpurun_out/gen_${TAG}_sel${v}_$r.jsonl 2>&1 || exit $?
    echo "sel_bound=$v $r"; cat gpurun_out/gen_${TAG}_sel${v}_$r.jsonl
  done
done
