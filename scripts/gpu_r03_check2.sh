# The -m gpu suite on the shipped build, the hot-receiver steps, and a same-box
# C2 A/B of two pinger-only builds (VARIANTS). First failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03o}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/hot_receiver_bench.py > gpurun_out/hot_$TAG.jsonl 2> gpurun_out/hot_$TAG.err || exit $?
cat gpurun_out/hot_$TAG.jsonl
timeout -k 10 180 python scripts/profile_general.py > gpurun_out/general_$TAG.jsonl 2> gpurun_out/general_$TAG.err || exit $?
cat gpurun_out/general_$TAG.jsonl
for r in 1 2 3; do
  for v in $VARIANTS; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 40 --warmup 5 \
      > gpurun_out/ab_${TAG}${v}_$r.json 2> gpurun_out/ab_${TAG}${v}_$r.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}${v}_$r.json')); print('$v', $r, round(d['value']/1e9,2), d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
