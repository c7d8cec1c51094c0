# Same-box A/B of k_step variants built by scripts/build_ab.py into
# ponyc_amd/variants/lib_<name>.so: scripts/profile_general.py <cases> for
# each variant, REPS rounds, alternating. VARIANTS="name1 name2 ..",
# CASES="pinger det storm". Each GPU step has its own limit; the first failure
# ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
REPS=${REPS:-3}
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  for v in $VARIANTS; do
    PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib_$v.so timeout -k 10 240 python scripts/profile_general.py ${CASES:-pinger} \
      > gpurun_out/ab_${TAG}_${v}_$r.jsonl 2>&1 || { cat gpurun_out/ab_${TAG}_${v}_$r.jsonl; exit 1; }
    echo "$v $r $(tr '\n' ' ' < gpurun_out/ab_${TAG}_${v}_$r.jsonl)"
  done
done
