# Inter-step gap experiment: per-step events (marker packets or the dispatch's
# own timestamps via hipExtLaunchKernel) vs strided events.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "1 0" "1 1" "8 1" "1000 1"; do
  set -- $cfg
  GPA_EVENT_STRIDE=$1 GPA_EXT_EVENTS=$2 timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline \
    > gpurun_out/gap_$1_$2.json 2>gpurun_out/gap_$1_$2.err || exit $?
  echo "stride=$1 ext=$2 $(python -c "import json;d=json.load(open('gpurun_out/gap_$1_$2.json'));print(d['ms_per_step'], d['value']/1e9, d['roofline']['kernel_ms'])")"
done
