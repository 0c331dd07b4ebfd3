# Where the settled headline step's time goes: the driver's short form and a 150-step form of
# bench.py (both after the default --settle updates), then a kernel-trace profile of the bench.
#   bash tools/gpu_settled.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1
for st in 20 150; do
  timeout -k 10 300 python bench.py --steps $st --warmup 5 > gpurun_out/${tag}_s$st.log 2>&1 || { tail -20 gpurun_out/${tag}_s$st.log; exit 2; }
  echo "settled, steps $st: $(tail -1 gpurun_out/${tag}_s$st.log | cut -c1-200)"
done
bash tools/prof.sh ${tag}_bench bench.py --steps 60 --warmup 5 || exit 4
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
head -45 gpurun_out/${tag}_bench_summary.md
