# Same-box A/B of variant builds on chosen BASELINE configs (scripts/bench_configs.py),
# alternating, 2 rounds: VARIANTS="_s8np _s8h" CONFIGS="c5_storm_8m".
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-cfg2}
for r in 1 2; do
  for v in $VARIANTS; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 300 python scripts/bench_configs.py $CONFIGS \
      > gpurun_out/abcfg_${TAG}${v}_$r.jsonl 2> gpurun_out/abcfg_${TAG}${v}_$r.err || exit $?
    python -c "
import json
for l in open('gpurun_out/abcfg_${TAG}${v}_$r.jsonl'):
    d = json.loads(l); print('$v', $r, d['config'], round(d['msgs_per_s'] / 1e9, 3), 'G/s', d['steps'], 'steps')"
  done
done
