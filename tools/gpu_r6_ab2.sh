# interleaved bench regime A/B: bash tools/gpu_r6_ab2.sh <tag> "<seeds>" "<dirA>|<argsA>" "<dirB>|<argsB>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; seeds=$2; shift 2
i=0
for sd in $seeds; do
  for spec in "$@"; do
    d=${spec%%|*}; args=${spec#*|}; i=$((i+1))
    (cd $R/$d && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seed $sd $args) > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 5; }
    grep metric gpurun_out/${tag}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('$d [$args] seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'envms', a['env_phase_ms'], 'ent', round(d['last_losses']['entropy'],2))"
  done
done
