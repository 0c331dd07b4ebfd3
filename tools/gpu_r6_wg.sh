# stage-0 weight-gradient A/B: conv / parity tests, then isolated learner timings and kernel
# profiles for the variants/base library against the tree's (learner_only --active 0.023)
#   bash tools/gpu_r6_wg.sh <tag> [pytest targets...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 3; }
  tail -2 gpurun_out/${tag}_pytest.log
fi
for occ in ${OCCS-0 1}; do
  for lib in base new; do
    la=""; [ $lib = base ] && la="--lib variants/base"
    timeout -k 10 200 python tools/learner_only.py --active 0.023 --steps 10 --bwd_occ $occ $la \
      > gpurun_out/${tag}_lo_${lib}_$occ.log 2>&1 || { tail -20 gpurun_out/${tag}_lo_${lib}_$occ.log; exit 4; }
    echo "$lib occ=$occ: $(tail -1 gpurun_out/${tag}_lo_${lib}_$occ.log)"
  done
done
for lib in base new; do
  la=""; [ $lib = base ] && la="--lib $R/variants/base"
  bash tools/prof.sh ${tag}_prof_$lib tools/learner_only.py --active 0.023 --steps 3 --bwd_occ 1 $la || exit 5
  grep -i "wgrad_kernel" gpurun_out/${tag}_prof_${lib}_summary.md | head -4
done
