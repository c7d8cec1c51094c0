# PMC passes for the step kernel (separate passes: FETCH_SIZE, WRITE_SIZE, L2 hit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
TAG=${TAG:-r01}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc/${TAG}_$N -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/pmc/bench_$N.json 2> gpurun_out/pmc/err_$N.txt || exit $?
done
ls -R gpurun_out/pmc | head -40
