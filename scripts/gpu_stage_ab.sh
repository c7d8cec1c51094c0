# Same-box A/B of general-path builds: the -m gpu suite against one build
# (TESTLIB), then scripts/profile_general.py for each run of RUNS, REPS times:
#   RUNS="name|lib|ENV=V ENV2=V2|det storm;name2|...". Every GPU step has its
# own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-stage}
REPS=${REPS:-2}
mkdir -p gpurun_out
if [ -n "$TESTLIB" ]; then
  env PONYC_AMD_LIB=$PWD/$TESTLIB $TESTENV timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 \
    --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra RS <<< "$RUNS"
for r in $(seq 1 $REPS); do
  for run in "${RS[@]}"; do
    IFS='|' read -r name lib envs cases <<< "$run"
    env PONYC_AMD_LIB=$PWD/$lib $envs timeout -k 10 240 python scripts/profile_general.py $cases \
      > gpurun_out/gen_${TAG}_${name}_$r.jsonl 2>&1 || exit $?
    echo "$name $r"; cat gpurun_out/gen_${TAG}_${name}_$r.jsonl
  done
done
