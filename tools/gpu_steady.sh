# Steady-state study of the headline bench: window frames/s and active cells
# over a long run from random init, then the driver's short form and a long form, both after the
# default --settle updates.
#   bash tools/gpu_steady.sh <tag> [long steps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; n=${2:-600}
timeout -k 10 400 python bench.py --settle 0 --steps $n --warmup 5 --report_every 20 > gpurun_out/${tag}_long.log 2>&1 || { tail -20 gpurun_out/${tag}_long.log; exit 2; }
grep window gpurun_out/${tag}_long.log; tail -1 gpurun_out/${tag}_long.log | cut -c1-200
for st in 20 150; do
  timeout -k 10 300 python bench.py --steps $st --warmup 5 > gpurun_out/${tag}_s$st.log 2>&1 || { tail -20 gpurun_out/${tag}_s$st.log; exit 3; }
  echo "settled, steps $st: $(tail -1 gpurun_out/${tag}_s$st.log | cut -c1-200)"
done
