# Bench every built variant (ponyc_amd/variants/lib_*.so) on the GPU: short
# bench each, one process per variant, each under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in ponyc_amd/variants/lib_*.so; do
  n=$(basename $f .so)
  PONYC_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/var_$n.json')); print('$n', round(d['value']/1e9,2), 'G msgs/s', 'k_ms', d['roofline']['kernel_ms'])"
done
