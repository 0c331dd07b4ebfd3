# bench.py regime check of other trees (git worktrees built in-tree): bash tools/gpu_r6_wt.sh <tag> "<seeds>" <dir>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; seeds=$2; shift 2
for d in "$@"; do
  for sd in $seeds; do
    (cd $R/$d && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seed $sd) > gpurun_out/${tag}_${d}_$sd.log 2>&1 || { tail -20 gpurun_out/${tag}_${d}_$sd.log; exit 5; }
    grep metric gpurun_out/${tag}_${d}_$sd.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('$d seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'envms', a['env_phase_ms'], 'ent', round(d['last_losses']['entropy'],2))"
  done
done
