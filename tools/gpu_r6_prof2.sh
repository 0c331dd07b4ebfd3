# Round-6 evidence pass: acting counters (both launches), then kernel profiles of the config-4
# (24x24 deep) and config-2 (10x10 GridNet) learners.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_act_pmc.sh r6act > gpurun_out/r6act_all.log 2>&1 || { tail -20 gpurun_out/r6act_all.log; exit 2; }
head -30 gpurun_out/r6act_all.log
bash tools/prof.sh r6c4lo tools/learner_only.py --arch impala_deep --size 24 --active 0.02 --steps 4 || exit 3
head -30 gpurun_out/r6c4lo_summary.md
bash tools/prof.sh r6c2lo tools/learner_only.py --arch gridnet --size 10 --active 0.02 --steps 4 || exit 4
head -30 gpurun_out/r6c2lo_summary.md
