# BASELINE configs 2-5 on one box (bench.py defaults: 500 settle updates, 20 timed steps).
#   bash tools/gpu_r6_configs.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-cfg}
run() {
  name=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/${tag}_$name.log 2>&1 || { tail -20 gpurun_out/${tag}_$name.log; exit 5; }
  grep metric gpurun_out/${tag}_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('$name', round(d['value']/1e6,3), 'M frames/s; active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'lrn', d['learner_phase_ms_rank0']['fwd'], d['learner_phase_ms_rank0']['bwd'], 'ms/step', d['ms_per_step'], d['config']['model'])"
}
run c3_headline
run c5_selfplay_bf16 --selfplay_groups 1
run c5_selfplay_fp8 --selfplay_groups 1 --fp8_policy
run c4_deep24 --size 24 --arch impala_deep
run c2_gridnet10 --size 10 --arch gridnet
