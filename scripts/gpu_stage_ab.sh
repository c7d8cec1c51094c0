# Same-box A/B of the staged drain: the -m gpu suite against the staged build,
# then the general-path step times (det, storm) of the base build, the staged
# build, the staged build with staging off (PONYC_AMD_STAGE=0) and C5 on
# 2048-actor zones (PONYC_AMD_ZONE_BITS=11). Every GPU step has its own limit;
# the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-stage}
NEW=$PWD/${NEW:-ponyc_amd/variants/lib_stage.so}
BASE=$PWD/ponyc_amd/variants/lib_base.so
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  PONYC_AMD_LIB=$NEW timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  PONYC_AMD_LIB=$BASE timeout -k 10 180 python scripts/profile_general.py det storm > gpurun_out/gen_${TAG}_base_$r.jsonl 2>&1 || exit $?
  echo "base $r"; cat gpurun_out/gen_${TAG}_base_$r.jsonl
  PONYC_AMD_LIB=$NEW timeout -k 10 180 python scripts/profile_general.py det storm > gpurun_out/gen_${TAG}_new_$r.jsonl 2>&1 || exit $?
  echo "new $r"; cat gpurun_out/gen_${TAG}_new_$r.jsonl
done
PONYC_AMD_LIB=$NEW PONYC_AMD_STAGE=0 timeout -k 10 180 python scripts/profile_general.py det storm > gpurun_out/gen_${TAG}_nostage.jsonl 2>&1 || exit $?
echo "new, stage off"; cat gpurun_out/gen_${TAG}_nostage.jsonl
PONYC_AMD_LIB=$NEW PONYC_AMD_ZONE_BITS=11 timeout -k 10 180 python scripts/profile_general.py storm > gpurun_out/gen_${TAG}_z11.jsonl 2>&1 || exit $?
echo "new, storm on 2048-actor zones"; cat gpurun_out/gen_${TAG}_z11.jsonl
