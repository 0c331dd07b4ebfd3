# Pipeline knobs re-measured after the engine's ready-only slot / publish change (one box).
#   bash tools/gpu_r4s.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4s}
i=0
for rep in 1 2 3; do
for v in "--lanes 2 --groups 3" "--lanes 3 --groups 3" "--lanes 4" ""; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 $v > gpurun_out/${tag}_b$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/${tag}_b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d["ms_per_step"], d["policy_lag_updates"])')"
done
done
