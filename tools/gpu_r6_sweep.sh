# pipeline-shape sweep of the headline (bench.py --groups / --lanes), 2 seeds each, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for sd in 1 2; do
  for gl in "4 2" "3 2" "5 2" "4 3" "6 3"; do
    set -- $gl; i=$((i+1))
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seed $sd --groups $1 --lanes $2 > gpurun_out/r6sw_$i.log 2>&1 || { tail -20 gpurun_out/r6sw_$i.log; exit 5; }
    grep metric gpurun_out/r6sw_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('groups $1 lanes $2 seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'lag', d['policy_lag_updates']['mean'], 'q', a['full_slots_waiting'])"
  done
done
