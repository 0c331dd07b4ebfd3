# BASELINE configs 5 / 4 / 2 and the headline bench on the new pipeline defaults (2 policy lanes
# x 3 groups, engine ready-only slots / publishes) vs the old 1 lane x 4 groups, one box.
#   bash tools/gpu_r4t.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4t}
show() { tail -1 $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d["ms_per_step"], d.get("policy_lag_updates"))'; }
for v in ""; do
  n=$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $v > gpurun_out/${tag}_c3_$n.log 2>&1 || exit 1
  echo "headline [$v] $(show gpurun_out/${tag}_c3_$n.log)"
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 --selfplay_groups 1 $v > gpurun_out/${tag}_c5_$n.log 2>&1 || exit 2
  echo "c5 [$v] $(show gpurun_out/${tag}_c5_$n.log)"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 24 --arch impala_deep $v > gpurun_out/${tag}_c4_$n.log 2>&1 || exit 3
  echo "c4 [$v] $(show gpurun_out/${tag}_c4_$n.log)"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 10 --arch gridnet $v > gpurun_out/${tag}_c2_$n.log 2>&1 || exit 4
  echo "c2 [$v] $(show gpurun_out/${tag}_c2_$n.log)"
done
