# Env-side knobs on the 2-lane x 3-group pipeline (one box, alternating): worker threads and
# envs per work item.
#   bash tools/gpu_r4w.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4w}
i=0
for rep in 1 2; do
for v in "MBK_NOP=0|" "MBK_NOP=0|--groups 2" "MBK_NOP=0|--lanes 3" "MBK_NOP=0|--groups 4"; do
  i=$((i+1))
  e=${v%%|*}; a=${v#*|}
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 $a > gpurun_out/${tag}_b$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/${tag}_b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["actor_stats"]; print(round(d["value"]/1e6,3), a["env_worker_busy_frac"], a["env_phase_ms"], a["gpu_phase_ms"])')"
done
done
