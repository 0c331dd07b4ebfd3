# Headline-bench A/B sweep: each variant "ENV=VAL ... [-- bench args]" runs bench.py once
# (20 timed steps) under its own time limit; prints frames/s and the phase split per variant.
# usage: bash tools/gpu_ab.sh "MBK_X=1" "MBK_Y=0 -- --lanes 2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "$@"; do
  envs="${v%%--*}"; args=""
  [[ "$v" == *"--"* ]] && args="${v#*--}"
  env $envs timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  echo "[$v] $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); a=d['actor_stats']; l=d['learner_phase_ms_rank0']; print(round(d['value']/1e6,3), 'gpu', a['gpu_phase_ms'], 'env', a['env_phase_ms'], 'fwd', l['fwd'], 'bwd', l['bwd'])")"
done
