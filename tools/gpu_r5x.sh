# Full GPU suite + settled bench (20 steps) + isolated learner timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/r5x_gpu.log 2>&1 || { tail -40 gpurun_out/r5x_gpu.log; exit 1; }
tail -2 gpurun_out/r5x_gpu.log
for act in 0.007 0.025; do
  timeout -k 10 200 python tools/learner_only.py --steps 5 --active $act > gpurun_out/r5x_learner_$act.log 2>&1 || exit 2
  echo "learner (active $act): $(tail -1 gpurun_out/r5x_learner_$act.log)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5x_bench.log 2>&1 || { tail -20 gpurun_out/r5x_bench.log; exit 3; }
tail -1 gpurun_out/r5x_bench.log | cut -c1-400
