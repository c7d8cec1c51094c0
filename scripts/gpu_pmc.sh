# PMC passes for the step kernel, one rocprofv3 run per pass (separate --pmc
# runs, kernel-trace only; MI355X_MICROARCH.md HBM/rocprofv3 section).
# Counters missing from `rocprofv3 -L` on the box are dropped from a pass.
# PMC_CMD overrides the profiled program (default: a short bench.py run),
# e.g. PMC_CMD="python3 scripts/bench_configs.py c4_gups_wide" for C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
# the library these passes profile: bench.py uses the summary only for this build
sha256sum ponyc_amd/libgpuactor.so | cut -c1-16 > $OUT/lib_sha16.txt
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || exit $?
have() { grep -qw "$1" $OUT/counters_list.txt; }
i=0
while read -r line; do
  [ -z "$line" ] && continue
  sel=""
  for c in $line; do base=${c%_sum}; if have $c || have $base; then sel="$sel $c"; fi; done
  [ -z "$sel" ] && continue
  i=$((i+1))
  echo "pass $i:$sel"
  timeout -s KILL 90 rocprofv3 --pmc $sel --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    ${PMC_CMD:-python3 bench.py --no-cpu-baseline --no-ring --steps 6 --warmup 2} > $OUT/bench_p$i.json 2> $OUT/err_p$i.txt || exit $?
done <<'PASSES'
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_REQ_sum
TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum TCC_EA0_WRREQ_64B_sum
TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr
PASSES
find $OUT -name '*counter_collection.csv' | sort
