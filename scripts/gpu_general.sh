# The general handler path: k_step per-step time of the
# pinger, C2-det and C5 storm, rocprofv3 kernel stats of the same runs, phase
# stamps, and PMC passes (one rocprofv3 run per pass) of det and storm.
# Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03f}
mkdir -p gpurun_out/prof
timeout -k 10 180 python scripts/profile_general.py > gpurun_out/general_$TAG.jsonl 2> gpurun_out/general_$TAG.err || exit $?
cat gpurun_out/general_$TAG.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/general_$TAG -o run -- \
  python3 scripts/profile_general.py > gpurun_out/general_prof_$TAG.jsonl 2> gpurun_out/general_prof_$TAG.err || exit $?
find gpurun_out/prof/general_$TAG -name '*stats*'
if [ -f ponyc_amd/libgpuactor_stamps.so ]; then
  timeout -k 10 180 python scripts/profile_general.py --stamps > gpurun_out/general_stamps_$TAG.jsonl 2>&1 || exit $?
  cat gpurun_out/general_stamps_$TAG.jsonl
fi
for w in det storm; do
  OUT=gpurun_out/pmc_${TAG}_$w
  mkdir -p $OUT
  sha256sum ponyc_amd/libgpuactor.so | cut -c1-16 > $OUT/lib_sha16.txt
  i=0
  for sel in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    echo "$w pass $i: $sel"
    timeout -s KILL 120 rocprofv3 --pmc $sel --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/profile_general.py $w > $OUT/out_p$i.txt 2> $OUT/err_p$i.txt || exit $?
  done
done
