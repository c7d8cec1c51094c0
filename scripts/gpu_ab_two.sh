# Same-box A/B of two engine builds (A = the in-tree library, B = $LIB_B):
# the hot-path tests against B, then det / storm / pinger step times and the
# hot-receiver burst for both, alternating, twice. Each GPU step has its own
# limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab2}
A=$PWD/ponyc_amd/libgpuactor.so
B=$PWD/$LIB_B
mkdir -p gpurun_out
# the tests run against B (the candidate; the C-ABI program links the in-tree name)
PONYC_AMD_LIB=$B timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "${TESTS_K:-(fifo or backlog or mute or hot or fanin) and not c_binary}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    PONYC_AMD_LIB=$lib timeout -k 10 240 python scripts/profile_general.py det storm pinger \
      > gpurun_out/gen_${TAG}_${v}_$r.jsonl 2>&1 || exit $?
    echo "$v $r"; cat gpurun_out/gen_${TAG}_${v}_$r.jsonl
    PONYC_AMD_LIB=$lib timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}_${v}_$r.jsonl 2>&1 || exit $?
    cat gpurun_out/hot_${TAG}_${v}_$r.jsonl
  done
done
