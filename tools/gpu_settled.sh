# Where the settled headline step's time goes: a kernel-trace profile of bench.py after the
# default --settle updates, and the isolated learner at the settled active-cell fraction.
#   bash tools/gpu_settled.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1
timeout -k 10 200 python tools/learner_only.py --steps 5 --active 0.025 > gpurun_out/${tag}_learner.log 2>&1 || exit 2
echo "learner at 2.5 % active: $(tail -1 gpurun_out/${tag}_learner.log)"
LT_ARGS="--active 0.025" bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 3
bash tools/prof.sh ${tag}_bench bench.py --steps 60 --warmup 5 || exit 4
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
head -60 gpurun_out/${tag}_bench_summary.md
