# GPU tests of the in-tree build (= C), then a same-box A/B of builds A and C
# on chosen BASELINE configs (scripts/bench_configs.py), alternating, 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_abcfg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_abcfg.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in A C; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 300 python scripts/bench_configs.py ${CONFIGS:-c2_ubench_det c5_storm_8m} \
      > gpurun_out/abcfg_${v}_$r.jsonl 2>/dev/null || exit $?
    python -c "
import json
for l in open('gpurun_out/abcfg_${v}_$r.jsonl'):
    d = json.loads(l); print('$v', $r, d['config'], round(d['msgs_per_s'] / 1e9, 3), 'G/s', d['steps'], 'steps')"
  done
done
