# Same-box A/B of variant builds on the general-path cases of
# scripts/profile_general.py (fixed busy steps, event-timed k_step):
# PAIRS="d3:det d3s:det s8:storm s8s:storm", alternating, 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-gab}
for r in 1 2; do
  for pc in $PAIRS; do
    v=${pc%%:*}; c=${pc##*:}
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib_$v.so timeout -k 10 180 python scripts/profile_general.py $c \
      > gpurun_out/gab_${TAG}_${v}_$r.jsonl 2> gpurun_out/gab_${TAG}_${v}_$r.err || exit $?
    echo "$v $r $(cat gpurun_out/gab_${TAG}_${v}_$r.jsonl)"
  done
done
