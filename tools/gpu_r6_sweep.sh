# pipeline-shape sweep of the headline (bench.py --groups / --lanes), interleaved over seeds:
#   bash tools/gpu_r6_sweep.sh <tag> "<seeds>" "4 2" "5 2" ...   (groups lanes per shape)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; seeds=$2; shift 2
shapes=("$@")
i=0
for sd in $seeds; do
  for gl in "${shapes[@]}"; do
    g=${gl% *}; l=${gl#* }; i=$((i+1))
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seed $sd --groups $g --lanes $l > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 5; }
    grep metric gpurun_out/${tag}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('groups $g lanes $l seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'envms', a['env_phase_ms'], 'gpums', a['gpu_phase_ms'], 'lag', d['policy_lag_updates']['mean'], 'q', a['full_slots_waiting'])"
  done
done
