# Same-box A/B of k_step variants built by scripts/build_ab.py into
# ponyc_amd/variants/lib_<name>.so: scripts/profile_general.py <cases> for
# each variant, REPS rounds, alternating. VARIANTS="lib[:ENV=V[,ENV2=V2]] ..."
# (a variant may also be the same library under other environment settings),
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
    lib=${v%%:*}
    envs=""
    [ "$lib" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
    name=$(echo "$v" | tr ':=,' '___')
    env PONYC_AMD_LIB=$PWD/ponyc_amd/variants/lib_$lib.so $envs timeout -k 10 240 python scripts/profile_general.py ${CASES:-pinger} \
      > gpurun_out/ab_${TAG}_${name}_$r.jsonl 2>&1 || { cat gpurun_out/ab_${TAG}_${name}_$r.jsonl; exit 1; }
    echo "$v $r $(tr '\n' ' ' < gpurun_out/ab_${TAG}_${name}_$r.jsonl)"
  done
done
