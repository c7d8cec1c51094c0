# A/B of two library builds on the C1 ring (bench.py's ring leg) after the
# sparse-path GPU tests of the new build; alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PONYC_AMD_LIB=$PWD/ponyc_amd/variants/libC.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ring.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ring.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in A C; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 2 \
      > gpurun_out/abr_${v}_$r.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abr_${v}_$r.json')); print('$v', $r, d['ring']['value'], d['ring']['ms_per_step'])"
  done
done
