# Settled-regime spread: bench.py runs over seeds x an option, one JSON summary line each.
#   bash tools/gpu_r6_regime.sh <tag> "<seeds>" "<extra args A>" "<extra args B>" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
tag=$1; seeds=$2; shift 2
i=0
for opt in "$@"; do
  for sd in $seeds; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --seed $sd $opt > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 5; }
    grep metric gpurun_out/${tag}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('[$opt] seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'stepped', round(a['env_frames_stepped_per_s_rank0']/1e6,2), 'busy', a['env_worker_busy_frac'], 'envms', a['env_phase_ms'], 'gpums', a['gpu_phase_ms'], 'ent', round(d['last_losses']['entropy'],2), 'lrn', d['learner_phase_ms_rank0']['fwd'], d['learner_phase_ms_rank0']['bwd'], 'q', a['full_slots_waiting'])"
  done
done
