# Hot receivers (round 3, last pass): the -m gpu suite on the shipped build,
# the 100K -> 4 FIFO burst / backlog steps of the shipped build (with and
# without backlog copies handed to k_carry_big: PONYC_AMD_DEFER_BIG) beside
# the previous build (PONYC_AMD_LIB), the zone's phase stamps, and same-box C2
# / general-path A/Bs. Every GPU step has its own limit; the first failure
# ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03x}
NEW=$PWD/ponyc_amd/libgpuactor.so
PREV=$PWD/ponyc_amd/variants/lib_prev.so
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
# variant name -> environment
run_v() {  # v cmd...
  v=$1; shift
  case $v in
    new) PONYC_AMD_LIB=$NEW "$@" ;;
    nodefer) PONYC_AMD_LIB=$NEW PONYC_AMD_DEFER_BIG=0 "$@" ;;
    prev) PONYC_AMD_LIB=$PREV "$@" ;;
  esac
}
for r in 1 2; do
  for v in new nodefer prev; do
    run_v $v timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_${TAG}_${v}_$r.jsonl 2>&1 || exit $?
    echo "hot $v $r"; cat gpurun_out/hot_${TAG}_${v}_$r.jsonl
  done
done
if [ -f ponyc_amd/libgpuactor_stamps.so ]; then
  PONYC_AMD_DEFER_BIG=0 timeout -k 10 180 python scripts/hot_stamps.py > gpurun_out/hot_stamps_$TAG.txt 2>&1 || exit $?
  cat gpurun_out/hot_stamps_$TAG.txt
fi
for r in 1 2 3; do
  for v in new prev; do
    run_v $v timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 40 --warmup 5 \
      > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${v}_$r.json')); print('c2 $v', $r, round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
for v in new nodefer prev; do
  run_v $v timeout -k 10 180 python scripts/profile_general.py det storm > gpurun_out/general_${TAG}_$v.jsonl 2>&1 || exit $?
  echo "general $v"; cat gpurun_out/general_${TAG}_$v.jsonl
done
