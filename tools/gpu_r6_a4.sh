set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
tag=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_act.py tests/test_gpu_head.py > gpurun_out/${tag}_t.log 2>&1 || { tail -30 gpurun_out/${tag}_t.log; exit 3; }
tail -1 gpurun_out/${tag}_t.log
for m in "" "--spread --settled_rows"; do
  timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 40 $m > gpurun_out/${tag}_ph.log 2>&1 || { tail -20 gpurun_out/${tag}_ph.log; exit 4; }
  echo "[$m] $(grep 'launch A' gpurun_out/${tag}_ph.log)"
  grep -E "first tile|barrier|decode|rows" gpurun_out/${tag}_ph.log | head -5
done
if [ "$2" = bench ]; then bash tools/gpu_r6_var2.sh ${tag}b "1 2 3" base; fi
