# Plain-zone split for C2-det and the storm (k_step PM 1 / 2 for the general
# path's tables): same-build A/B (PONYC_AMD_SPLIT_PLAN=0 is the one-launch
# step), then evidence part A on the in-tree library. Every GPU step has its
# own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
TESTLIB=ponyc_amd/libgpuactor.so \
RUNS="one|ponyc_amd/libgpuactor.so|PONYC_AMD_SPLIT_PLAN=0|pinger det storm;two|ponyc_amd/libgpuactor.so||pinger det storm" \
  REPS=2 TAG=w bash scripts/gpu_stage_ab.sh || exit $?
SKIP_PYTEST=1 PART=A TAG=r04w bash scripts/gpu_evidence.sh
