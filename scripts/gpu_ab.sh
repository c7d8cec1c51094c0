# A/B of two builds of the library on one box: the C2 bench, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in ${VARIANTS:-A B}; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-ring --steps 40 --warmup 5 \
      > gpurun_out/ab_${v}_$r.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_${v}_$r.json')); print('$v', $r, d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
