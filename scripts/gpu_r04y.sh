# Round-4 late candidate (the two-pass step as two launches + zone offsets in
# SGPRs): same-box A/B against the one-launch build, then evidence part A on
# the in-tree library. Every GPU step has its own limit; the first failure ends
# the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
RUNS="mono|ponyc_amd/variants/split/libgpuactor.so|PONYC_AMD_SPLIT_PLAN=0|pinger det storm;new|ponyc_amd/libgpuactor.so||pinger det storm" \
  REPS=2 TAG=${ABTAG:-y} bash scripts/gpu_stage_ab.sh || exit $?
PART=A TAG=${EVTAG:-r04y} bash scripts/gpu_evidence.sh
