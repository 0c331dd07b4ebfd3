# Counter evidence for the learner and the acting step on the GPU box (one call):
#   learner  : same-box kernel-trace A/B (tools/lt_ab.sh) of the given variants, then the MFMA /
#              LDS / HBM passes and the stall passes of tools/learner_only.py;
#   act      : tools/gpu_act_pmc.sh (isolated phases + counters of the fused policy step).
# Stops at the first failure.
#   bash tools/gpu_evidence.sh <tag> learner|act|both ["VAR=v ..." ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; what=$2; shift 2
if [ "$what" = learner ] || [ "$what" = both ]; then
  timeout -k 10 240 python tools/learner_only.py --steps 5 > gpurun_out/${tag}_learner.log 2>&1 || exit 2
  echo "learner: $(tail -1 gpurun_out/${tag}_learner.log)"
  if [ $# -gt 0 ]; then bash tools/lt_ab.sh ${tag} "$@" || exit 3; fi
  bash tools/pmc.sh ${tag}_l tools/learner_only.py --steps 2 || exit 4
  bash tools/pmc_wait.sh ${tag}_l res_fwd16,res_bwd16,conv0_row,pool_bwd,wgrad,conv_fwd \
    tools/learner_only.py --steps 2 || exit 5
  cat gpurun_out/${tag}_l_pmc.md gpurun_out/${tag}_l_wait.md
fi
if [ "$what" = act ] || [ "$what" = both ]; then
  bash tools/gpu_act_pmc.sh ${tag}_a || exit 6
fi
