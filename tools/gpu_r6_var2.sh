# bench.py vs tools/bench_variant.py settings, interleaved over seeds:
#   bash tools/gpu_r6_var2.sh <tag> "<seeds>" "<variant sets | 'base' | --bench,--flags>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; seeds=$2; shift 2
i=0
for sd in $seeds; do
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = base ]; then cmd="python bench.py"
    elif [ "${v:0:2}" = "--" ]; then cmd="python bench.py ${v//,/ }"   # bench flags, comma-joined
    else cmd="python tools/bench_variant.py $v --"; fi
    timeout -k 10 300 $cmd --steps 20 --warmup 5 --seed $sd > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 5; }
    grep metric gpurun_out/${tag}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['actor_stats']; print('[$v] seed $sd', round(d['value']/1e6,2), 'active', d['active_cells_per_env'], 'busy', a['env_worker_busy_frac'], 'envms', a['env_phase_ms'], 'gpums', a['gpu_phase_ms'], 'lrn', d['learner_phase_ms_rank0']['fwd'], d['learner_phase_ms_rank0']['bwd'])"
  done
done
