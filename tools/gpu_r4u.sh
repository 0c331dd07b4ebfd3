# Acting knobs re-measured on the 2-lane x 3-group pipeline (one box, alternating reps).
#   bash tools/gpu_r4u.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4u}
i=0
for rep in 1 2 3; do
for v in "MBK_HEAD_ACT_GRID=16" "MBK_HEAD_ACT_GRID=8" "MBK_HEAD_ACT_GRID=4"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/${tag}_b$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/${tag}_b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d["ms_per_step"], d["policy_lag_updates"]["mean"])')"
done
done
