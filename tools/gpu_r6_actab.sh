# Isolated acting launches in both pair distributions (+ optional bench kernel trace).
#   bash tools/gpu_r6_actab.sh <tag> [prof]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
tag=${1:-act}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py tests/test_gpu_head.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
for sp in "" "--spread"; do
  timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 30 $sp > gpurun_out/${tag}_phases$sp.log 2>&1 || { tail -20 gpurun_out/${tag}_phases$sp.log; exit 4; }
  echo "spread=$sp"; head -4 gpurun_out/${tag}_phases$sp.log | tail -3
done
if [ "$2" = prof ]; then
  bash tools/prof.sh ${tag}_bench bench.py --steps 60 --warmup 5 || exit 5
  tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
  head -40 gpurun_out/${tag}_bench_summary.md
fi
